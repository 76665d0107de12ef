"""Marked point-process priors (drop-in for smcdet/prior.py).

Kept: `PointProcessPrior` (prior.py:8-75), `PoissonProcessPrior` (:78-101),
`ParetoStarPrior` (:157-189), `M71Prior` (:192-226) with the reference
constructors, attributes, `sample()` and `log_prob()`.

`sample(stratify_by_count=True, ...)` — what SMCsampler.initialize uses — and
`log_prob` run as gfx950 kernels (smcdet_prior_sample / smcdet_log_prior).
The non-stratified `sample()` draw (used only to generate synthetic truth
catalogs, images.py:186) is plain torch on the HIP device.
"""
from __future__ import annotations

import numpy as np
import torch
from torch.distributions import Uniform

from . import _hip
from ._rng import PhiloxStream
from .distributions import DiscreteUniform, TruncatedPareto


def _f32(x):
    return float(np.float32(x))


def _check_pad_mode(mode):
    if mode not in ("tile", "partition"):
        raise ValueError("pad_mode must be either tile or partition.")
    return mode


def partition_boxes(tiles_shape, tile_h, tile_w, pad, device=None):
    """[numH*numW, 4] float32 (lo_h, lo_w, hi_h, hi_w) per tile, in tile
    coordinates: [0, H) x [0, W), widened by `pad` on the sides that are the
    image's outer edges."""
    nH, nW = tiles_shape
    i = torch.arange(nH, dtype=torch.float32).reshape(nH, 1).expand(nH, nW)
    j = torch.arange(nW, dtype=torch.float32).reshape(1, nW).expand(nH, nW)
    p = float(pad)
    lo_h = torch.where(i == 0, -p, 0.0)
    lo_w = torch.where(j == 0, -p, 0.0)
    hi_h = torch.where(i == nH - 1, tile_h + p, float(tile_h))
    hi_w = torch.where(j == nW - 1, tile_w + p, float(tile_w))
    b = torch.stack([lo_h, lo_w, hi_h, hi_w], -1).reshape(nH * nW, 4)
    return b.to(device=device).contiguous()


def _device(device=None):
    if device is not None:
        return torch.device(device)
    d = torch.get_default_device()
    if d.type == "cuda":
        return d
    return torch.device("cuda", torch.cuda.current_device())


class PointProcessPrior(object):
    """prior.py:8-75: discrete-uniform count, uniform locations over the
    padded tile [-pad, H+pad) x [-pad, W+pad).

    pad_mode (keyword-only extension): "tile" (the reference: every tile of an
    image is padded on all four sides, so neighbouring tiles' boxes overlap)
    or "partition" (only the image's outer edges are padded: the tiles' boxes
    partition the padded image, and the product of the tiles' priors is the
    whole image's prior -- what tile aggregation needs to be exact,
    DESIGN.md §9)."""

    def __init__(self, min_objects, max_objects, image_height, image_width, pad=0, *,
                 pad_mode="tile"):
        self.min_objects = min_objects
        self.max_objects = max_objects
        self.image_height = image_height
        self.image_width = image_width
        self.pad = pad
        self.pad_mode = _check_pad_mode(pad_mode)
        self.update_attrs()

    def update_attrs(self):
        self.num_counts = self.max_objects - self.min_objects + 1
        self.count_prior = DiscreteUniform(self.min_objects, self.max_objects)
        self.loc_prior = Uniform(
            (0 - self.pad) * torch.ones(2, device="cpu"),
            torch.tensor((self.image_height + self.pad, self.image_width + self.pad),
                         dtype=torch.float32, device="cpu"))

    def tile_boxes(self, tiles_shape, device=None):
        """Per-tile location boxes for a numH x numW grid of image tiles of
        this prior's size: None with pad_mode "tile" (every tile uses the
        prior's own box), else partition_boxes()."""
        if getattr(self, "pad_mode", "tile") == "tile":
            return None
        return partition_boxes(tiles_shape, self.image_height, self.image_width, self.pad,
                               device)

    def log_count_prior_per_tile(self, boxes):
        """log p(s), s = min..max, per tile box [T, NS]: a Poisson count mean
        scales with the box area (prior.py:91-97)."""
        s = torch.arange(self.min_objects, self.max_objects + 1, dtype=torch.float64)
        b = boxes.detach().cpu().double()
        if isinstance(self, PoissonProcessPrior):
            area = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
            mu = torch.tensor([_f32(self.counts_rate * float(a)) for a in area],
                              dtype=torch.float64)[:, None]
            return s * torch.log(mu) - mu - torch.lgamma(s + 1)
        return torch.full((b.shape[0], s.numel()), -float(np.log(s.numel())),
                          dtype=torch.float64)

    # --- C-ABI description ----------------------------------------------------
    @_hip.cached_struct
    def _cprior(self):
        raise NotImplementedError(
            f"{type(self).__name__} has no flux prior; the HIP path supports M71Prior and "
            "ParetoStarPrior")

    def _fill_common(self, c):
        c.min_objects = int(self.min_objects)
        c.max_objects = int(self.max_objects)
        c.loc_low = _f32(-self.pad)
        c.loc_high_h = _f32(self.image_height + self.pad)
        c.loc_high_w = _f32(self.image_width + self.pad)
        return c

    def _sample_counts(self, shape, device):
        idx = self.count_prior.sample(shape).long().cpu()
        counts = torch.arange(self.min_objects, self.max_objects + 1)[idx]
        return counts.to(device=device, dtype=torch.float32)

    def _sample_flux(self, shape, device):
        raise NotImplementedError

    def sample(self, num_catalogs=1, num_tiles_per_side=1, stratify_by_count=False,
               num_catalogs_per_count=None, device=None):
        """prior.py:25-64 (+ the flux draws of :175-180, :212-217)."""
        if stratify_by_count is True and num_catalogs_per_count is None:
            raise ValueError("If stratify_by_count is True, need to specify catalogs_per_count.")
        elif stratify_by_count is False and num_catalogs_per_count is not None:
            raise ValueError("If stratify_by_count is False, do not specify catalogs_per_count.")
        device = _device(device)
        T = num_tiles_per_side
        S = self.max_objects
        if stratify_by_count:
            self.num = self.num_counts * num_catalogs_per_count
            counts, locs, fluxes = self.sample_stratified(T, num_catalogs_per_count,
                                                          device=device)
        else:
            self.num = num_catalogs
            counts = self._sample_counts([T, T, self.num], device)
            lo, hi = self.loc_prior.low.to(device), self.loc_prior.high.to(device)
            u = torch.rand(T, T, self.num, S, 2, device=device)
            locs = lo + u * (hi - lo)
            fluxes = self._sample_flux([T, T, self.num, S], device)
            mask = torch.arange(S, device=device) < counts.unsqueeze(-1)
            locs = locs * mask.unsqueeze(-1)
            fluxes = fluxes * mask
        self.counts_mask = torch.arange(S, device=device) < counts.unsqueeze(-1)
        return [counts, locs, fluxes]

    def sample_stratified(self, num_tiles_per_side, num_catalogs_per_count, device=None,
                          rng: PhiloxStream | None = None, uloc=None, uflux=None,
                          tiles_shape=None, tile_boxes=None):
        """Stratified draw on device: counts = min..max (each repeated
        num_catalogs_per_count times), uniform locs, prior fluxes, masked past
        each count.  uloc/uflux replay the reference's torch.rand draws.
        tiles_shape=(numH, numW) overrides the square num_tiles_per_side grid;
        tile_boxes [T,4] (optional) gives each tile its own location box."""
        device = _device(device)
        nH, nW = tiles_shape if tiles_shape is not None else (num_tiles_per_side,) * 2
        N = self.num_counts * num_catalogs_per_count
        S = self.max_objects
        counts = torch.empty(nH, nW, N, device=device, dtype=torch.float32)
        locs = torch.zeros(nH, nW, N, S, 2, device=device, dtype=torch.float32)
        fluxes = torch.zeros(nH, nW, N, S, device=device, dtype=torch.float32)
        rng = rng or PhiloxStream()
        off = rng.take(S)  # counters per particle (the kernel keys draws by particle)
        cp = self._cprior()
        if uloc is not None:
            uloc = _hip.dev_f32(uloc.to(device), "uloc")
            uflux = _hip.dev_f32(uflux.to(device), "uflux")
        if tile_boxes is not None:
            tile_boxes = _hip.dev_f32(tile_boxes.to(device), "tile_boxes")
        _hip.check(_hip.lib().smcdet_prior_sample(
            _hip.ref(cp), nH * nW, num_catalogs_per_count, rng.seed, off, _hip.ptr(uloc),
            _hip.ptr(uflux), _hip.ptr(tile_boxes), _hip.ptr(counts), _hip.ptr(locs),
            _hip.ptr(fluxes), _hip.stream_of(counts)), "smcdet_prior_sample")
        return counts, locs, fluxes

    def log_prob(self, counts, locs, fluxes, *, tile_boxes=None):
        """prior.py:67-75 (+ flux terms of :183-189 / :220-226): [numH,numW,N].
        tile_boxes [T,4] (optional): each tile's own location box."""
        counts = _hip.dev_f32(counts, "counts")
        locs = _hip.dev_f32(locs, "locs")
        fluxes = _hip.dev_f32(fluxes, "fluxes")
        nH, nW, n, d, _ = locs.shape
        out = torch.empty(nH, nW, n, device=locs.device, dtype=torch.float32)
        cp = self._cprior()
        if tile_boxes is not None:
            tile_boxes = _hip.dev_f32(tile_boxes.to(locs.device), "tile_boxes")
        _hip.check(_hip.lib().smcdet_log_prior(_hip.ref(cp), _hip.ptr(counts), _hip.ptr(locs),
                                               _hip.ptr(fluxes), nH * nW, n, d,
                                               _hip.ptr(tile_boxes), _hip.ptr(out),
                                               _hip.stream_of(locs)), "smcdet_log_prior")
        self.counts_mask = torch.arange(d, device=counts.device) < counts.unsqueeze(-1)
        return out


class PoissonProcessPrior(PointProcessPrior):
    """prior.py:78-101: Poisson(counts_rate * (H+2pad)(W+2pad)) count prior."""

    def __init__(self, min_objects, max_objects, counts_rate, image_height, image_width, pad=0, *,
                 pad_mode="tile"):
        self.min_objects = min_objects
        self.max_objects = max_objects
        self.counts_rate = counts_rate
        self.image_height = image_height
        self.image_width = image_width
        self.pad = pad
        self.pad_mode = _check_pad_mode(pad_mode)
        self.update_attrs()

    def update_attrs(self):
        self.num_counts = self.max_objects - self.min_objects + 1
        self.count_prior = torch.distributions.Poisson(
            torch.tensor(self.poisson_mean, dtype=torch.float32))
        self.loc_prior = Uniform(
            (0 - self.pad) * torch.ones(2, device="cpu"),
            torch.tensor((self.image_height + self.pad, self.image_width + self.pad),
                         dtype=torch.float32, device="cpu"))

    @property
    def poisson_mean(self):
        return _f32(self.counts_rate * (self.image_height + 2 * self.pad)
                    * (self.image_width + 2 * self.pad))


class ParetoStarPrior(PointProcessPrior):
    """prior.py:157-189: Pareto(flux_scale, flux_alpha) fluxes."""

    def __init__(self, *args, flux_scale, flux_alpha, **kwargs):
        super().__init__(*args, **kwargs)
        self.flux_scale = flux_scale
        self.flux_alpha = flux_alpha
        self.flux_prior = torch.distributions.Pareto(torch.tensor(float(flux_scale)),
                                                     torch.tensor(float(flux_alpha)))

    def _sample_flux(self, shape, device):
        u = torch.rand(*shape, device=device)
        return _f32(self.flux_scale) * (1.0 - u) ** (-1.0 / _f32(self.flux_alpha))

    @_hip.cached_struct
    def _cprior(self):
        c = self._fill_common(_hip.PriorC())
        c.kind = _hip.SMCDET_PRIOR_PARETO
        c.flux_alpha = _f32(self.flux_alpha)
        c.flux_lower = _f32(self.flux_scale)
        c.flux_upper = 0.0
        return c


class M71Prior(PoissonProcessPrior):
    """prior.py:192-226: Poisson counts, truncated-Pareto(alpha, lower, upper) fluxes."""

    def __init__(self, *args, flux_alpha, flux_lower, flux_upper, **kwargs):
        super().__init__(*args, **kwargs)
        self.flux_alpha = flux_alpha
        self.flux_lower = flux_lower
        self.flux_upper = flux_upper
        self.flux_prior = TruncatedPareto(flux_alpha, flux_lower, flux_upper)

    def _sample_flux(self, shape, device):
        return self.flux_prior.sample(shape, device=device)

    def _sample_counts(self, shape, device):
        k = torch.poisson(torch.full(shape, self.poisson_mean, dtype=torch.float32)).long()
        counts = torch.arange(self.min_objects, self.max_objects + 1)[k]
        return counts.to(device=device, dtype=torch.float32)

    @_hip.cached_struct
    def _cprior(self):
        c = self._fill_common(_hip.PriorC())
        c.kind = _hip.SMCDET_PRIOR_M71
        c.poisson_mean = self.poisson_mean
        c.flux_alpha = _f32(self.flux_alpha)
        c.flux_lower = _f32(self.flux_lower)
        c.flux_upper = _f32(self.flux_upper)
        return c
