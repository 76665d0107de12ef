"""Image models (drop-in for smcdet/images.py).

`ImageModel` (Normal-pdf PSF, Poisson noise; reference images.py:6-102) and
`M71ImageModel` (SDSS-fitted 3-component PSF, Gaussian noise with
variance noise_additive + noise_multiplicative*rate; images.py:105-175) keep
the reference constructors, attributes and methods.  `psf`, `loglikelihood`
and `sample` run as gfx950 kernels (smcdet_amd/csrc/model_kernels.hip); the
dense PSF tensor is never materialised on the likelihood path.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _hip
from ._rng import torch_seed


def _as_float_list(x):
    if isinstance(x, torch.Tensor):
        return [float(v) for v in x.detach().cpu().reshape(-1).tolist()]
    return [float(v) for v in x]


def _f32(x):
    return float(np.float32(x))


class ImageModel(object):
    """smcdet/images.py:6-102 — Normal(0, psf_stdev) radial PSF profile,
    Poisson likelihood (Normal(rate, sqrt(rate)) where rate > 5e4)."""

    def __init__(self, image_height, image_width, background, psf_radius: int, psf_stdev=None):
        self.image_height = image_height
        self.image_width = image_width
        self.background = background
        self.psf_radius = psf_radius
        self.psf_stdev = psf_stdev
        seq = torch.arange(-self.psf_radius, self.psf_radius + 1)
        ph, pw = torch.meshgrid(seq, seq, indexing="ij")
        self.psf_patch = torch.stack([ph, pw], dim=-1)

    # -- reference helper (images.py:25-26); elementwise, not on the hot path
    def _compute_normalized_psf(self, r):
        s = float(self.psf_stdev)
        return torch.exp(-(r ** 2) / (2 * s * s) - math.log(s) - 0.5 * math.log(2 * math.pi))

    def update_psf_grid(self):
        """Called by Aggregate.join after the tile dimensions change
        (aggregate.py:241; no reference image model defines it).  The kernels
        read image_height / image_width on every call: nothing to update."""

    # -- C-ABI description -------------------------------------------------
    @_hip.cached_struct
    def _cmodel(self):
        if self.psf_stdev is None:
            raise NotImplementedError("ImageModel needs psf_stdev for the HIP path")
        c = _hip.ImageModelC()
        c.model = _hip.SMCDET_MODEL_POISSON
        c.H, c.W = int(self.image_height), int(self.image_width)
        c.psf_radius = int(self.psf_radius)
        c.background = _f32(self.background)
        c.adu_per_nmgy = 1.0
        c.psf_params[0] = _f32(self.psf_stdev)
        c.psf_norm = 1.0
        return c

    def _check_shapes(self, locs):
        if locs.dim() != 5 or locs.shape[-1] != 2:
            raise ValueError(f"locs must be [numH,numW,N,S,2], got {tuple(locs.shape)}")

    def psf(self, locs):
        """images.py:28-76: dense psf [numH,numW,H,W,N,S]."""
        self._check_shapes(locs)
        locs = _hip.dev_f32(locs, "locs")
        nH, nW, n, d, _ = locs.shape
        out = torch.empty(nH, nW, self.image_height, self.image_width, n, d,
                          device=locs.device, dtype=torch.float32)
        cm = self._cmodel()
        _hip.check(_hip.lib().smcdet_psf_dense(_hip.ref(cm), _hip.ptr(locs), nH * nW, n, d,
                                               _hip.ptr(out), _hip.stream_of(locs)),
                   "smcdet_psf_dense")
        return out

    def rate(self, locs, fluxes):
        """Noise-free rate image [numH,numW,H,W,N] (images.py:80-82 / :149-154)."""
        self._check_shapes(locs)
        locs = _hip.dev_f32(locs, "locs")
        fluxes = _hip.dev_f32(fluxes, "fluxes")
        nH, nW, n, d, _ = locs.shape
        out = torch.empty(nH, nW, self.image_height, self.image_width, n, device=locs.device,
                          dtype=torch.float32)
        cm = self._cmodel()
        _hip.check(_hip.lib().smcdet_render(_hip.ref(cm), _hip.ptr(locs), _hip.ptr(fluxes),
                                            nH * nW, n, d, _hip.ptr(out), _hip.stream_of(locs)),
                   "smcdet_render")
        return out

    def sample(self, locs, fluxes):
        """images.py:78-83 / :147-157: a noisy image per catalog, [numH,numW,H,W,N]."""
        rate = self.rate(locs, fluxes)
        cm = self._cmodel()
        _hip.check(_hip.lib().smcdet_sample_image(_hip.ref(cm), _hip.ptr(rate), rate.numel(),
                                                  torch_seed(), 0, _hip.ptr(rate),
                                                  _hip.stream_of(rate)), "smcdet_sample_image")
        return rate

    def loglikelihood(self, tiled_image, locs, fluxes):
        """images.py:85-102 / :159-175: log p(tile | catalog), [numH,numW,N]."""
        self._check_shapes(locs)
        tiled_image = _hip.dev_f32(tiled_image, "tiled_image")
        locs = _hip.dev_f32(locs, "locs")
        fluxes = _hip.dev_f32(fluxes, "fluxes")
        nH, nW, n, d, _ = locs.shape
        if tuple(tiled_image.shape) != (nH, nW, self.image_height, self.image_width):
            raise ValueError(f"tiled_image {tuple(tiled_image.shape)} does not match "
                             f"[{nH},{nW},{self.image_height},{self.image_width}]")
        out = torch.empty(nH, nW, n, device=locs.device, dtype=torch.float32)
        cm = self._cmodel()
        _hip.check(_hip.lib().smcdet_loglik(_hip.ref(cm), _hip.ptr(tiled_image), _hip.ptr(locs),
                                            _hip.ptr(fluxes), nH * nW, n, d, _hip.ptr(out),
                                            _hip.stream_of(locs)), "smcdet_loglik")
        return out


def m71_psf_unnormalized(r2, psf_params):
    """images.py:137-141 in r^2, float64 numpy (normaliser computation)."""
    s1, s2, sp, beta, b, p0 = (float(np.float32(v)) for v in psf_params)
    t1 = np.exp(-r2 / (2 * s1))
    t2 = b * np.exp(-r2 / (2 * s2))
    t3 = p0 * (1 + r2 / (beta * sp)) ** (-beta / 2)
    return (t1 + t2 + t3) / (1 + b + p0)


class M71ImageModel(ImageModel):
    """smcdet/images.py:105-175."""

    def __init__(self, *args, adu_per_nmgy, psf_params, noise_additive=0,
                 noise_multiplicative=1, **kwargs):
        super().__init__(*args, **kwargs)
        self.adu_per_nmgy = adu_per_nmgy
        pp = _as_float_list(psf_params)
        if len(pp) != 6:
            raise ValueError("psf_params must hold (sigma1, sigma2, sigmap, beta, b, p0)")
        self.psf_params = pp
        self.sigma1, self.sigma2, self.sigmap, self.beta, self.b, self.p0 = pp
        self.noise_additive = noise_additive
        self.noise_multiplicative = noise_multiplicative
        # normalising constant: unnormalised PSF summed over a (32R)^2 grid
        # centred at (16R, 16R) with pixel-centre offsets (images.py:122-135)
        n = 32 * self.psf_radius
        g = np.arange(n, dtype=np.float64) - n / 2.0 + 0.5
        r2 = g[:, None] ** 2 + g[None, :] ** 2
        self.psf_normalizing_constant = torch.tensor(
            float(m71_psf_unnormalized(r2, pp).sum()), dtype=torch.float32)

    def _compute_unnormalized_psf(self, r):
        term1 = torch.exp(-(r ** 2) / (2 * self.sigma1))
        term2 = self.b * torch.exp(-(r ** 2) / (2 * self.sigma2))
        term3 = self.p0 * (1 + r ** 2 / (self.beta * self.sigmap)) ** (-self.beta / 2)
        return (term1 + term2 + term3) / (1 + self.b + self.p0)

    def _compute_normalized_psf(self, r):
        return self._compute_unnormalized_psf(r) / self.psf_normalizing_constant.to(r.device)

    @_hip.cached_struct
    def _cmodel(self):
        c = _hip.ImageModelC()
        c.model = _hip.SMCDET_MODEL_M71
        c.H, c.W = int(self.image_height), int(self.image_width)
        c.psf_radius = int(self.psf_radius)
        c.background = _f32(self.background)
        c.adu_per_nmgy = _f32(self.adu_per_nmgy)
        for i, v in enumerate(self.psf_params):
            c.psf_params[i] = _f32(v)
        c.psf_norm = float(self.psf_normalizing_constant)
        c.noise_additive = _f32(self.noise_additive)
        c.noise_multiplicative = _f32(self.noise_multiplicative)
        return c


def generate_images(Prior, ImageModel, flux_threshold, loc_threshold_lower, loc_threshold_upper,
                    num_images=1):
    """smcdet/images.py:178-228: draw catalogs from the prior, render noisy
    images, and prune to detectable in-bounds sources."""
    catalogs = Prior.sample(num_catalogs=num_images)
    unpruned_counts, unpruned_locs, unpruned_fluxes = catalogs
    images = ImageModel.sample(unpruned_locs, unpruned_fluxes)
    hi = torch.tensor((loc_threshold_upper, loc_threshold_upper), device=unpruned_locs.device,
                      dtype=unpruned_locs.dtype)
    mask = torch.all((unpruned_locs > loc_threshold_lower) & (unpruned_locs < hi), dim=-1)
    mask = mask & (unpruned_fluxes > flux_threshold)
    pruned_counts = mask.sum(-1)
    order = torch.sort((~mask).to(torch.int8), dim=3, stable=True)[1]
    pruned_locs = torch.gather(mask.unsqueeze(-1) * unpruned_locs, 3,
                               order.unsqueeze(-1).expand_as(unpruned_locs))
    pruned_fluxes = torch.gather(mask * unpruned_fluxes, 3, order)
    sq = lambda x: x.squeeze(0).squeeze(0)  # noqa: E731
    images = sq(images).permute(2, 0, 1)
    return [sq(unpruned_counts), sq(unpruned_locs), sq(unpruned_fluxes), sq(pruned_counts),
            sq(pruned_locs), sq(pruned_fluxes), images]
