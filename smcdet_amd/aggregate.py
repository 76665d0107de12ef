"""Tile aggregation: divide-and-conquer SMC over neighbouring tiles
(drop-in for smcdet/aggregate.py:8-639, Aggregate).

After per-tile samplers have run, `Aggregate.run()` merges tiles pairwise,
alternating the height and width axes (2*log2(numH) levels for a numH x numH
grid), until one catalog population covers the whole image.  At each level
the joint tile's population starts as the product of its two children's
(resampled by their weights, the sources in the padding the children share
dropped from one side) and is tempered from the children's likelihoods to the
joint tile's:
    log pi_tau(z) = log p(z) + (1 - tau) * [l_c1(z_1) + l_c2(z_2)] + tau * l_p(z)
with the particles grouped by source count, each count group tempered,
reweighted and resampled on its own (the tile's increment is the smallest of
its groups'), and MH moves between steps.

The reference's Aggregate does not run at HEAD (join calls a missing
ImageModel.update_psf_grid; mutate passes nine arguments to a six-argument
SingleComponentMH.run).  This module is the repaired design of DESIGN.md §9:
  * the MH moves a present source (component < count), not any of the
    max_objects slots (kernel.py:35-37 would turn an empty slot into a source
    the prior does not count);
  * each joint tile's log-likelihood increment pairs ITS two children (the
    reference's unjoin concatenates the children half-major and then pairs
    consecutive tiles, aggregate.py:296-322 + :536-541, which mixes up the
    children as soon as more than one joint tile lies along the axis);
  * the merged groups' log evidences are log Z_c1 + log Z_c2 + log(n_j / N)
    (the reference's merge_pmf reads child counts that drop_sources_from_overlap
    has already overwritten in place, aggregate.py:355-407).
What the reference does and this keeps: the tempering target, brentq per
group with ESS target ess_threshold_prop * group size, the minimum over
groups, per-group softmax weights and log evidences, intracount multinomial
resampling every iteration, overall weights = within-group weights x
softmax of the group log evidences, the final resample and prune.

Device work (smcdet_amd/csrc):
    mutate        -> smcdet_aggregate_sweep   (MH on the bridging target, fused
                                               intracount gather, returns l_p
                                               and l_c1 + l_c2 of the new state)
    temper        -> smcdet_aggregate_temper  (brentq per count group) + a
                                               per-tile scatter-min
    update_weights-> smcdet_aggregate_reweight (weights, group log Z, next
                                               intracount resampling indices)
    merge         -> smcdet_resample_index + smcdet_gather, then the drop /
                     join bookkeeping as torch ops once per level
"""
from __future__ import annotations

import math
from copy import deepcopy

import torch

from . import _hip
from ._rng import PhiloxStream
from .kernel import SingleComponentMALA
from .prior import partition_boxes


def _f32(t):
    return t.to(torch.float32)


def compact(keep, locs, fluxes):
    """Kept slots to the front in their order, zeros behind (the reference's
    sort-by-nonzero + gather, aggregate.py:252-261, :280-317).  Returns
    (counts float32, locs, fluxes)."""
    order = torch.sort((~keep).to(torch.int8), dim=-1, stable=True)[1]
    l = torch.gather(locs * keep.unsqueeze(-1), -2, order.unsqueeze(-1).expand_as(locs))
    f = torch.gather(fluxes * keep, -1, order)
    return keep.sum(-1).to(torch.float32), l, f


def _axis_sel(x, axis, start):
    return x[start::2] if axis == 0 else x[:, start::2]


def drop_overlap(axis, locs, fluxes, dim):
    """aggregate.py:189-215 on [numH,numW,N,S,...] catalogs: tiles at even
    positions along `axis` drop their sources at coordinate >= dim or == 0
    (the padding they share with the next tile), odd tiles those at
    coordinate <= 0.  Returns compacted (counts, locs, fluxes)."""
    c = locs[..., axis]
    n_ax = locs.shape[axis]
    even = (torch.arange(n_ax, device=locs.device) % 2 == 0).reshape(
        [n_ax if i == axis else 1 for i in range(c.dim())])
    keep = (fluxes != 0) & torch.where(even, (c < dim) & (c != 0), c > 0)
    return compact(keep, locs, fluxes)


def join_tiles(axis, data, locs, fluxes, dim):
    """aggregate.py:217-263 without the model bookkeeping: tiles 2i and 2i+1
    along `axis` stacked into one, the second tile's sources shifted by the
    child side `dim`, catalogs concatenated and compacted (all 2S slots)."""
    dat = torch.cat([_axis_sel(data, axis, 0), _axis_sel(data, axis, 1)], dim=2 + axis)
    l1 = _axis_sel(locs, axis, 1).clone()
    f1 = _axis_sel(fluxes, axis, 1)
    l1[..., axis] = torch.where(f1 != 0, l1[..., axis] + dim, torch.zeros_like(f1))
    ls = torch.cat([_axis_sel(locs, axis, 0), l1], dim=-2)
    fs = torch.cat([_axis_sel(fluxes, axis, 0), f1], dim=-1)
    cs, ls, fs = compact(fs != 0, ls, fs)
    return dat.contiguous(), cs, ls, fs


def unjoin_tiles(axis, data, locs, fluxes, dim):
    """aggregate.py:265-324: joint tiles of side `dim` along `axis` back into
    their halves (source coordinate <= dim/2 -> first half), the children of
    joint tile i at 2i and 2i+1.  Returns (data, counts, locs, fluxes)."""
    half = dim // 2
    d0 = data[:, :, :half] if axis == 0 else data[:, :, :, :half]
    d1 = data[:, :, half:] if axis == 0 else data[:, :, :, half:]
    p = fluxes != 0
    m = locs[..., axis] <= dim / 2
    k0, l0, f0 = compact(p & m, locs, fluxes)
    k1, l1, f1 = compact(p & ~m, locs, fluxes)
    l1 = l1.clone()
    l1[..., axis] = torch.where(f1 != 0, l1[..., axis] - dim / 2, torch.zeros_like(f1))

    def inter(x, y):
        st = torch.stack([x, y], dim=axis + 1)
        sh = list(x.shape)
        sh[axis] *= 2
        return st.reshape(sh)
    return inter(d0, d1), inter(k0, k1), inter(l0, l1), inter(f0, f1)


class CountGroups(object):
    """Count groups ("segments") of a count-sorted population [numH,numW,N]:
    per segment its tile, first particle and length (int32 device arrays, the
    layout smcdet_aggregate_temper / _reweight take), per particle its global
    segment id, and the segments' counts."""

    def __init__(self, counts_sorted):
        nH, nW, N = counts_sorted.shape
        T = nH * nW
        c = counts_sorted.reshape(T, N)
        new = torch.ones_like(c, dtype=torch.bool)
        new[:, 1:] = c[:, 1:] != c[:, :-1]
        flat = new.reshape(-1)
        self.seg_id = (torch.cumsum(flat.to(torch.int64), 0) - 1).reshape(T, N)
        starts = torch.nonzero(flat, as_tuple=False).reshape(-1)
        ends = torch.cat([starts[1:], torch.tensor([T * N], device=c.device)])
        self.tile = (starts // N).to(torch.int32).contiguous()
        self.start = (starts % N).to(torch.int32).contiguous()
        self.length = (ends - starts).to(torch.int32).contiguous()
        self.count = c.reshape(-1)[starts]
        self.G = int(starts.numel())
        self.T, self.N = T, N

    def sizes(self, numW):
        """[h][w] -> list of group sizes (the reference's num_catalogs_per_count)."""
        out = [[[] for _ in range(numW)] for _ in range(self.T // numW)]
        for t, n in zip(self.tile.cpu().tolist(), self.length.cpu().tolist()):
            out[t // numW][t % numW].append(n)
        return out


def aggregate_sweep(image_model, prior, mh, axis, data, temperature, counts, locs, fluxes, *,
                    num_iters=None, ancestors=None, replay=None, seed=0, offset=0,
                    acc_workspace=None, tile_boxes=None):
    """One smcdet_aggregate_sweep launch on joint tiles data [numH,numW,H,W]
    (image_model / prior at the joint dimensions, mh a SingleComponentMH):
    num_iters (default mh.num_iters) MH iterations on the bridging target.
    Returns (counts, locs, fluxes, loglik_parent, loglik_children, acc_rate);
    acc_rate is None without acc_workspace ([2T] zeroed int32).  tile_boxes
    [T,4] (optional): each joint tile's own location box."""
    data = _hip.dev_f32(data, "data")
    locs = _hip.dev_f32(locs, "locs")
    fluxes = _hip.dev_f32(fluxes, "fluxes")
    counts = _hip.dev_f32(counts, "counts")
    temperature = _hip.dev_f32(temperature, "temperature")
    nH, nW, N, S, _ = locs.shape
    T = nH * nW
    if S > _hip.MAX_AGG_SOURCES:
        raise ValueError(f"Aggregate: {S} sources in a joint tile > {_hip.MAX_AGG_SOURCES}")
    dev = locs.device
    ch = mh._cmh(prior)
    if num_iters is not None:
        # (a copy: _cmh returns the kernel's cached struct)
        ch = _hip.MHC.from_buffer_copy(ch)
        ch.num_iters = int(num_iters)
    co, lo, lf = torch.empty_like(counts), torch.empty_like(locs), torch.empty_like(fluxes)
    lp = torch.empty(nH, nW, N, device=dev)
    lc = torch.empty(nH, nW, N, device=dev)
    acc = torch.empty(nH, nW, device=dev) if acc_workspace is not None else None
    rp, keep = None, []
    if replay is not None:
        rc = replay["comp"].to(device=dev, dtype=torch.int32).contiguous()
        ru = [_hip.dev_f32(replay[k].to(dev), k) for k in ("uloc", "uflux", "uacc")]
        keep = [rc] + ru
        rp = _hip.ReplayC(_hip.ptr(rc).value, _hip.ptr(ru[0]).value, _hip.ptr(ru[1]).value,
                          _hip.ptr(ru[2]).value)
    if ancestors is not None:
        ancestors = ancestors.to(device=dev, dtype=torch.int64).contiguous()
    if tile_boxes is not None:
        tile_boxes = _hip.dev_f32(tile_boxes.to(dev), "tile_boxes")
    cm = image_model._cmodel()
    # joint tiles beyond the LDS budget: rate images and catalog per particle in
    # a device workspace (the global-memory sweep, M71)
    need = int(_hip.lib().smcdet_aggregate_workspace(_hip.ref(cm), T, N, S))
    if need < 0:
        _hip.check(need, "smcdet_aggregate_workspace")
    work = torch.empty(need, device=dev, dtype=torch.float32) if need > 0 else None
    _hip.check(_hip.lib().smcdet_aggregate_sweep(
        _hip.ref(cm), _hip.ref(prior._cprior()), _hip.ref(ch), int(axis),
        _hip.ptr(data), _hip.ptr(temperature), T, N, S, _hip.ptr(ancestors), _hip.ptr(counts),
        _hip.ptr(locs), _hip.ptr(fluxes), _hip.ptr(co), _hip.ptr(lo), _hip.ptr(lf), int(seed),
        int(offset), _hip.ref(rp) if rp is not None else None, _hip.ptr(lp), _hip.ptr(lc),
        _hip.ptr(acc), _hip.ptr(acc_workspace), _hip.ptr(tile_boxes), _hip.ptr(work),
        _hip.stream_of(lo)), "smcdet_aggregate_sweep")
    del keep, work
    return co, lo, lf, lp, lc, acc


def temper_groups(loglik_parent, loglik_children, temperature, groups, ess_threshold_prop):
    """aggregate.py:140-174: per count group, the brentq tempering increment
    (smcdet_aggregate_temper); the tile's increment is the minimum over its
    groups.  Returns (new temperature [numH,numW], per-group deltas [G])."""
    delta = torch.empty(groups.G, device=temperature.device)
    _hip.check(_hip.lib().smcdet_aggregate_temper(
        _hip.ptr(_hip.dev_f32(loglik_parent, "loglik_parent")),
        _hip.ptr(_hip.dev_f32(loglik_children, "loglik_children")),
        _hip.ptr(_hip.dev_f32(temperature, "temperature")), groups.T, groups.N, groups.G,
        _hip.ptr(groups.tile), _hip.ptr(groups.start), _hip.ptr(groups.length),
        float(ess_threshold_prop), _hip.ptr(delta), _hip.stream_of(delta)),
        "smcdet_aggregate_temper")
    dmin = torch.full((groups.T,), math.inf, device=delta.device).scatter_reduce(
        0, groups.tile.long(), delta, "amin")
    return (temperature.reshape(-1) + dmin).reshape(temperature.shape), delta


def reweight_groups(loglik_parent, loglik_children, temperature, temperature_prev, groups, lnc,
                    *, seed=0, offset=0, u=None, want_index=True):
    """aggregate.py:439-483 (+ the intracount resampling indices of :485-521)
    per count group (smcdet_aggregate_reweight); lnc [G] is updated in place.
    Returns (log_weights_unnorm, weights_intracount, ess [G], idx or None)."""
    shape = loglik_parent.shape
    dev = loglik_parent.device
    lw = torch.empty(shape, device=dev)
    wi = torch.empty(shape, device=dev)
    ess = torch.empty(groups.G, device=dev)
    idx = torch.empty(shape, device=dev, dtype=torch.int64) if want_index else None
    if u is not None:
        u = _hip.dev_f32(u.to(dev), "u")
    _hip.check(_hip.lib().smcdet_aggregate_reweight(
        _hip.ptr(_hip.dev_f32(loglik_parent, "loglik_parent")),
        _hip.ptr(_hip.dev_f32(loglik_children, "loglik_children")),
        _hip.ptr(_hip.dev_f32(temperature, "temperature")),
        _hip.ptr(_hip.dev_f32(temperature_prev, "temperature_prev")), groups.T, groups.N,
        groups.G, _hip.ptr(groups.tile), _hip.ptr(groups.start), _hip.ptr(groups.length),
        _hip.ptr(lw), _hip.ptr(wi), _hip.ptr(lnc), _hip.ptr(ess), int(seed), int(offset),
        _hip.ptr(u), _hip.ptr(idx), _hip.stream_of(lw)), "smcdet_aggregate_reweight")
    return lw, wi, ess, idx


def log_sum_groups(lnc, groups):
    """[T]: per tile, log of the sum of its groups' exp(lnc)."""
    st = groups.tile.long()
    m = torch.full((groups.T,), -math.inf, device=lnc.device).scatter_reduce(0, st, lnc, "amax")
    s = torch.zeros(groups.T, device=lnc.device).index_add_(0, st, torch.exp(lnc - m[st]))
    return m + torch.log(s)


def group_probs(lnc, groups):
    """softmax of the group log evidences within each tile, per group."""
    st = groups.tile.long()
    m = torch.full((groups.T,), -math.inf, device=lnc.device).scatter_reduce(0, st, lnc, "amax")
    e = torch.exp(lnc - m[st])
    s = torch.zeros(groups.T, device=lnc.device).index_add_(0, st, e)
    return e / s[st]


class Aggregate(object):
    def __init__(self, Prior, ImageModel, MutationKernel, data, counts, locs, fluxes, weights,
                 log_normalizing_constant, flux_detection_threshold, resample_method,
                 ess_threshold_prop, print_every=5, *, seed=None, device=None):
        if isinstance(MutationKernel, SingleComponentMALA):
            raise NotImplementedError("Aggregate runs SingleComponentMH moves (the fused "
                                      "aggregation sweep has no MALA variant)")
        self.Prior = deepcopy(Prior)
        self.ImageModel = deepcopy(ImageModel)
        self.MutationKernel = deepcopy(MutationKernel)
        self.MutationKernel.locs_min = self.Prior.loc_prior.low
        self.MutationKernel.locs_max = self.Prior.loc_prior.high
        self.mutation_acc_rates = None

        if device is None:
            device = data.device if data.is_cuda else torch.device(
                "cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        dev = self.device
        self.data = _f32(data.to(dev)).contiguous()
        self.counts = _f32(counts.to(dev)).contiguous()
        self.locs = _f32(locs.to(dev)).contiguous()
        self.fluxes = _f32(fluxes.to(dev)).contiguous()
        self.weights = _f32(weights.to(dev)).contiguous()
        self.weights_intracount = None

        self.numH, self.numW, self.dimH, self.dimW = self.data.shape
        if self.numH != self.numW or self.numH & (self.numH - 1):
            raise ValueError(f"Aggregate needs a square power-of-two grid of tiles, got "
                             f"{self.numH}x{self.numW} (aggregate.py:40)")
        self.num_aggregation_levels = int(round(2 * math.log2(self.numH)))
        fh, fw = self.numH * self.dimH, self.numW * self.dimW
        # joint tiles beyond the LDS budget run the global-memory sweep (M71)
        from .images import M71ImageModel
        limit = (_hip.MAX_TILE_PIXELS_GLOBAL if isinstance(ImageModel, M71ImageModel)
                 else _hip.MAX_TILE_PIXELS)
        if fh * fw > limit:
            raise ValueError(f"Aggregate: the aggregated {fh}x{fw} image exceeds {limit} pixels")
        lnc = torch.as_tensor(log_normalizing_constant, dtype=torch.float32)
        if lnc.dim() != 2 or tuple(lnc.shape) != (self.numH, self.numW):
            raise ValueError("log_normalizing_constant must be [numH, numW]")
        # one group (the whole population) per tile until the first merge
        self._lnc = lnc.to(dev).reshape(-1).contiguous()
        self._build_segments(torch.zeros_like(self.counts))

        self.flux_detection_threshold = flux_detection_threshold
        self.num_catalogs = self.weights.shape[-1]
        self.num_catalogs_per_count = [[None for _ in range(self.numW)]
                                       for _ in range(self.numH)]
        self.temperature_prev = torch.zeros(self.numH, self.numW, device=dev)
        self.temperature = torch.zeros(self.numH, self.numW, device=dev)
        if resample_method not in {"multinomial", "systematic"}:
            raise ValueError("resample_method must be either multinomial or systematic.")
        self.resample_method = resample_method
        self.ess_threshold_prop = ess_threshold_prop
        self.print_every = print_every
        self.has_run = False
        self.rng = PhiloxStream(seed)
        self._pending_idx = None
        self._acc_ws = None
        self.loglik_parent = self.loglik_children = None
        # Prior pad_mode "partition" (the tiles' boxes partition the padded
        # image): nothing to drop at a merge, and every joint tile keeps the
        # partition box of its place in the grid -- the exact variant of §9
        self.partition = getattr(self.Prior, "pad_mode", "tile") == "partition"

    # ------------------------------------------------------------ bookkeeping
    @property
    def _T(self):
        return self.numH * self.numW

    @property
    def tile_boxes(self):
        """[T,4] location boxes of the current (joint) tiles in partition
        mode, else None (every tile uses the prior's padded box)."""
        if not self.partition:
            return None
        return partition_boxes((self.numH, self.numW), self.dimH, self.dimW, self.Prior.pad,
                               self.device)

    def _build_segments(self, counts_sorted):
        self._groups = CountGroups(counts_sorted)

    @property
    def log_normalizing_constant(self):
        """Per tile, the log evidences of its count groups (the reference's
        nested lists, aggregate.py:42-45, :460-465)."""
        lnc = self._lnc.detach().cpu().tolist()
        tiles = self._groups.tile.cpu().tolist()
        out = [[[] for _ in range(self.numW)] for _ in range(self.numH)]
        for v, t in zip(lnc, tiles):
            out[t // self.numW][t % self.numW].append(v)
        return out

    @property
    def log_evidence(self):
        """[numH, numW]: log of the sum over count groups of their evidences."""
        return log_sum_groups(self._lnc, self._groups).reshape(self.numH, self.numW)

    def _group_probs(self):
        return group_probs(self._lnc, self._groups)

    def _refresh_weights(self):
        """overall weights = within-group weights x group probabilities
        (aggregate.py:467-483)."""
        p = self._group_probs()
        w = self.weights_intracount.reshape(self._T, -1) * p[self._groups.seg_id]
        self.weights = w.reshape(self.numH, self.numW, -1)

    # --------------------------------------------------- the reference methods
    def get_resampled_index(self, weights, multiplier):
        """aggregate.py:69-84 (multiplier 1: N draws per tile)."""
        N = weights.shape[-1]
        if int(multiplier * N) != N:
            raise ValueError("only multiplier = 1 is supported")
        idx = torch.empty(weights.shape, device=self.device, dtype=torch.int64)
        method = (_hip.SMCDET_RESAMPLE_SYSTEMATIC if self.resample_method == "systematic"
                  else _hip.SMCDET_RESAMPLE_MULTINOMIAL)
        off = self.rng.take(1 if self.resample_method == "systematic" else N)
        w = _hip.dev_f32(weights, "weights")
        _hip.check(_hip.lib().smcdet_resample_index(
            _hip.ptr(w), w.shape[0] * w.shape[1], N, method, self.rng.seed, off, None,
            _hip.ptr(idx), _hip.stream_of(idx)), "smcdet_resample_index")
        return idx

    def apply_resampled_index(self, resampled_index, counts, locs, fluxes):
        """aggregate.py:86-103."""
        nH, nW, N = resampled_index.shape
        S = locs.shape[-2]
        cs, ls, fs = torch.empty_like(counts), torch.empty_like(locs), torch.empty_like(fluxes)
        _hip.check(_hip.lib().smcdet_gather(
            _hip.ptr(resampled_index), nH * nW, N, S, _hip.ptr(counts), _hip.ptr(locs),
            _hip.ptr(fluxes), _hip.ptr(cs), _hip.ptr(ls), _hip.ptr(fs),
            _hip.stream_of(counts)), "smcdet_gather")
        ws = torch.full((nH, nW, N), 1.0 / N, device=counts.device)
        return cs, ls, fs, ws

    def log_target(self, axis, ChildImageModel, child_data, child_locs, child_fluxes, parent_data,
                   parent_counts, parent_locs, parent_fluxes, temperature):
        """aggregate.py:105-130 (host helper; the sweep evaluates it in-kernel).
        child_* in unjoin's layout (children of joint tile i at 2i, 2i+1)."""
        logprior = self.Prior.log_prob(parent_counts, parent_locs, parent_fluxes,
                                       tile_boxes=self.tile_boxes)
        child = ChildImageModel.loglikelihood(child_data, child_locs, child_fluxes)
        child = _axis_sel(child, axis, 0) + _axis_sel(child, axis, 1)
        parent = self.ImageModel.loglikelihood(parent_data, parent_locs, parent_fluxes)
        t = temperature.unsqueeze(-1)
        return logprior + (1 - t) * child + t * parent

    def tempering_objective(self, loglikelihood, delta):
        """aggregate.py:132-138 (host helper)."""
        log_numerator = 2 * ((delta * loglikelihood).logsumexp(0))
        log_denominator = (2 * delta * loglikelihood).logsumexp(0)
        return (log_numerator - log_denominator).exp() - \
            self.ess_threshold_prop * loglikelihood.shape[0]

    def temper(self):
        """aggregate.py:140-174: brentq per count group on device; the tile's
        increment is the smallest of its groups'."""
        new_t, _ = temper_groups(self.loglik_parent, self.loglik_children, self.temperature,
                                 self._groups, self.ess_threshold_prop)
        self.temperature_prev = self.temperature
        self.temperature = new_t

    def mutate(self, axis, ChildImageModel=None):
        """aggregate.py:176-187: K MH iterations per particle on the bridging
        target (the intracount resampling indices, if pending, are gathered
        inside the sweep)."""
        T = self._T
        if self._acc_ws is None or self._acc_ws.numel() < 2 * T:
            self._acc_ws = torch.zeros(2 * T, device=self.device, dtype=torch.int32)
        anc = self._pending_idx
        self._pending_idx = None
        off = self.rng.take(int(self.MutationKernel.num_iters))
        (self.counts, self.locs, self.fluxes, self.loglik_parent, self.loglik_children,
         self.mutation_acc_rates) = aggregate_sweep(
            self.ImageModel, self.Prior, self.MutationKernel, axis, self.data, self.temperature,
            self.counts, self.locs, self.fluxes, ancestors=anc, seed=self.rng.seed, offset=off,
            acc_workspace=self._acc_ws, tile_boxes=self.tile_boxes)

    def evaluate(self, axis):
        """l_p and l_c1 + l_c2 of the current state (the sweep with K = 0)."""
        _, _, _, self.loglik_parent, self.loglik_children, _ = aggregate_sweep(
            self.ImageModel, self.Prior, self.MutationKernel, axis, self.data, self.temperature,
            self.counts, self.locs, self.fluxes, num_iters=0, tile_boxes=self.tile_boxes)
        return self.loglik_parent, self.loglik_children

    @property
    def loglik_diff(self):
        """l_p - (l_c1 + l_c2) per particle (aggregate.py:539-541)."""
        return self.loglik_parent - self.loglik_children

    def drop_sources_from_overlap(self, axis, counts, locs, fluxes):
        """aggregate.py:189-215 (drop_overlap); counts are recomputed."""
        return drop_overlap(axis, locs, fluxes, self.dimH if axis == 0 else self.dimW)

    def join(self, axis, data, counts, locs, fluxes):
        """aggregate.py:217-263: tiles 2i and 2i+1 along `axis` become one tile
        of twice the size; the second tile's sources shift by the child side;
        catalogs concatenated and compacted to max(1, max count) slots.  The
        image model, prior box and MH bounds move to the joint dimensions."""
        dim = self.dimH if axis == 0 else self.dimW
        if axis == 0:
            self.numH //= 2
            self.dimH *= 2
            self.ImageModel.image_height *= 2
            self.Prior.image_height *= 2
        else:
            self.numW //= 2
            self.dimW *= 2
            self.ImageModel.image_width *= 2
            self.Prior.image_width *= 2
        dat, cs, ls, fs = join_tiles(axis, data, locs, fluxes, dim)
        smax = max(1, int(cs.max().item()))
        if smax > _hip.MAX_AGG_SOURCES:
            raise ValueError(f"Aggregate: a joint catalog of {smax} sources exceeds "
                             f"{_hip.MAX_AGG_SOURCES}")
        self.Prior.max_objects = smax
        self.Prior.update_attrs()
        self.ImageModel.update_psf_grid()
        self.MutationKernel.locs_min = self.Prior.loc_prior.low
        self.MutationKernel.locs_max = self.Prior.loc_prior.high
        return (dat.contiguous(), cs.contiguous(), ls[..., :smax, :].contiguous(),
                fs[..., :smax].contiguous())

    def unjoin(self, axis, data, locs, fluxes):
        """aggregate.py:265-324: the joint tiles back into their halves (source
        coordinate <= dim/2 -> first half), children of joint tile i at 2i and
        2i+1 along the axis.  Returns (data, counts, locs, fluxes)."""
        return unjoin_tiles(axis, data, locs, fluxes, self.dimH if axis == 0 else self.dimW)

    def prune(self, locs, fluxes):
        """aggregate.py:326-345 (the final tile is square)."""
        locs = _hip.dev_f32(locs, "locs")
        fluxes = _hip.dev_f32(fluxes, "fluxes")
        if self.dimH != self.dimW:
            raise ValueError("prune needs a square tile")
        nH, nW, N, S, _ = locs.shape
        counts = torch.empty(nH, nW, N, device=locs.device, dtype=torch.int64)
        pl, pf = torch.empty_like(locs), torch.empty_like(fluxes)
        _hip.check(_hip.lib().smcdet_prune(
            _hip.ptr(locs), _hip.ptr(fluxes), nH * nW, N, S, float(self.dimH),
            float(self.flux_detection_threshold), _hip.ptr(counts), _hip.ptr(pl), _hip.ptr(pf),
            _hip.stream_of(locs)), "smcdet_prune")
        return counts, pl, pf

    def merge(self, level):
        """aggregate.py:347-422 (repaired log evidences, see the module
        docstring): resample each tile by its weights, drop the shared-padding
        sources, join pairs along axis level % 2."""
        axis = level % 2
        # the children's total log evidences, before the bookkeeping moves on
        child_lz = self.log_evidence
        index = self.get_resampled_index(self.weights, 1)
        cs, ls, fs, _ = self.apply_resampled_index(index, self.counts, self.locs, self.fluxes)
        if not self.partition:  # partition boxes do not overlap: nothing to drop
            cs, ls, fs = self.drop_sources_from_overlap(axis, cs, ls, fs)
        self.data, self.counts, self.locs, self.fluxes = self.join(axis, self.data, cs, ls, fs)
        self._child_log_evidence = _axis_sel(child_lz, axis, 0) + _axis_sel(child_lz, axis, 1)

    def sort_by_count(self):
        """aggregate.py:424-437 (stable sort), plus the count groups and their
        merged log evidences log Z_c1 + log Z_c2 + log(n_j / N)."""
        self.counts, indices = torch.sort(self.counts, dim=-1, stable=True)
        self.locs = torch.gather(self.locs, 2, indices[..., None, None].expand_as(self.locs))
        self.fluxes = torch.gather(self.fluxes, 2, indices[..., None].expand_as(self.fluxes))
        self.counts, self.locs, self.fluxes = (self.counts.contiguous(), self.locs.contiguous(),
                                               self.fluxes.contiguous())
        self._build_segments(self.counts)
        g = self._groups
        self.num_catalogs_per_count = g.sizes(self.numW)
        base = getattr(self, "_child_log_evidence", None)
        if base is not None:
            self._lnc = (base.reshape(-1)[g.tile.long()]
                         + torch.log(g.length.to(torch.float32) / g.N)).contiguous()
            self._child_log_evidence = None

    def update_weights(self):
        """aggregate.py:439-483 + the next intracount resampling indices
        (:485-521), one launch over the count groups."""
        off = self.rng.take(self.num_catalogs)
        self.weights_log_unnorm, self.weights_intracount, self.ess_per_group, idx = \
            reweight_groups(self.loglik_parent, self.loglik_children, self.temperature,
                            self.temperature_prev, self._groups, self._lnc, seed=self.rng.seed,
                            offset=off)
        self._pending_idx = idx
        self._refresh_weights()

    def resample_intracount(self):
        """aggregate.py:485-521: multinomial resampling within each count group
        (indices drawn by update_weights; run() gathers them inside the next
        sweep instead)."""
        if self._pending_idx is None:
            return
        cs, ls, fs, _ = self.apply_resampled_index(self._pending_idx, self.counts, self.locs,
                                                   self.fluxes)
        self.counts, self.locs, self.fluxes = cs, ls, fs
        self._pending_idx = None
        g = self._groups
        self.weights_intracount = (1.0 / g.length.to(torch.float32))[g.seg_id].reshape(
            self.numH, self.numW, -1)
        self._refresh_weights()

    def _print_progress(self):
        if self.print_every and self.iter % self.print_every == 0:
            msg = (f"iteration {self.iter}: "
                   f"temperature in [{round(self.temperature.min().item(), 2)}, "
                   f"{round(self.temperature.max().item(), 2)}]")
            if self.mutation_acc_rates is not None:
                msg += (f", accept rate in [{round(self.mutation_acc_rates.min().item(), 2)}, "
                        f"{round(self.mutation_acc_rates.max().item(), 2)}]")
            print(msg)

    def run(self):
        """aggregate.py:523-593."""
        print("aggregating tile catalogs...")
        self.iters_per_level = []
        for level in range(self.num_aggregation_levels):
            print(f"level {level}")
            axis = level % 2
            ChildImageModel = deepcopy(self.ImageModel)
            self.merge(level)
            self.sort_by_count()
            self.evaluate(axis)
            self.temperature_prev = torch.zeros(self.numH, self.numW, device=self.device)
            self.temperature = torch.zeros(self.numH, self.numW, device=self.device)
            self.temper()
            self.update_weights()
            self.iter = 0
            while bool((self.temperature < 1).any().item()):
                self.iter += 1
                self._print_progress()
                # resample_intracount() happens inside the sweep (ancestors)
                self.mutate(axis, ChildImageModel)
                self.temper()
                self.update_weights()
            self.iters_per_level.append(self.iter)
        index = self.get_resampled_index(self.weights, 1)
        self.counts, self.locs, self.fluxes, self.weights = self.apply_resampled_index(
            index, self.counts, self.locs, self.fluxes)
        self.pruned_counts, self.pruned_locs, self.pruned_fluxes = self.prune(self.locs,
                                                                              self.fluxes)
        self.has_run = True
        print("done!\n")

    # ---------------------------------------------------------------- summaries
    @property
    def ess(self):
        return 1 / (self.weights ** 2).sum(-1)

    def posterior_mean_count(self, counts):
        return (self.weights * counts).sum(-1)

    def posterior_mean_total_flux(self, fluxes):
        return (self.weights * fluxes.sum(-1)).sum(-1)

    @property
    def posterior_predictive_total_observed_flux(self):
        return self.ImageModel.sample(self.locs, self.fluxes).sum([-2, -3]).squeeze()

    def summarize(self):
        """aggregate.py:609-638."""
        if self.has_run is False:
            raise ValueError("aggregation procedure hasn't been run yet.")
        print("posterior distribution of number of detectable stars within image boundary:")
        u, c = self.pruned_counts.unique(return_counts=True)
        print(u.cpu())
        print((c / self.pruned_counts.shape[-1]).round(decimals=3).cpu(), "\n")
        print("posterior mean total intrinsic flux (including undetectable and/or in padding) =",
              f"{self.posterior_mean_total_flux(self.fluxes).item()}\n")
        print("posterior mean total intrinsic flux of detectable stars within image boundary =",
              f"{self.posterior_mean_total_flux(self.pruned_fluxes).item()}\n")
        print(f"number of unique catalogs = {self.fluxes[0, 0].sum(-1).unique(dim=0).shape[0]}")
