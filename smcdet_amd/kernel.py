"""Mutation kernels (drop-ins for smcdet/kernel.py:7-130, SingleComponentMH,
and smcdet/kernel.py:133-275, SingleComponentMALA).

`SingleComponentMH.run(data, counts, locs, fluxes, temperature, log_target)`
keeps the reference signature and return value `[locs, fluxes, acc_rate]`.
The reference evaluates `log_target` (a Python callback, sampler.py:87-91) in
every iteration; a fused gfx950 kernel cannot call back into Python, so the
callback is resolved once to the (Prior, ImageModel) pair it closes over —
the bound `SMCsampler.log_target`, or the `prior=`/`image_model=` keywords —
and all `num_iters` iterations run in one launch
(smcdet_amd/csrc/mh_kernel.hip).  Priors/image models without a HIP
description raise NotImplementedError: there is no fallback dispatch.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _hip
from ._rng import PhiloxStream


def _f32(x):
    return float(np.float32(float(x)))


class SingleComponentMH(object):
    _entry = "smcdet_mh_sweep"

    def __init__(self, num_iters, locs_stdev, fluxes_stdev, fluxes_min, fluxes_max, *,
                 full_recompute=False):
        self.num_iters = num_iters
        self.locs_stdev = torch.tensor(locs_stdev)
        self.locs_min = None  # defined automatically within SMCsampler
        self.locs_max = None  # defined automatically within SMCsampler
        self.fluxes_stdev = fluxes_stdev * torch.ones(1)
        self.fluxes_min = fluxes_min * torch.ones(1)
        self.fluxes_max = fluxes_max * torch.ones(1)
        # True: re-render every source at every step (the reference's arithmetic);
        # False: incremental delta log-likelihood over the moved source's windows
        self.full_recompute = full_recompute
        # True: the moved component is drawn from 0..count-1 (fixed-count
        # strata padded to S sources, see cssmc.py); False: 0..S-1 (kernel.py:35-37)
        self.component_by_count = False
        self.rng = None           # PhiloxStream; SMCsampler installs its own
        self.debug_flags = 0      # SMCDET_MH_ABLATE_* timing diagnostics (never for sampling)
        self.last_loglik = None   # log-likelihood of the state returned by run()
        self._acc_ws = {}

    @staticmethod
    def _resolve(log_target, prior, image_model):
        if prior is None or image_model is None:
            owner = getattr(log_target, "__self__", None)
            if owner is None or not hasattr(owner, "Prior") or not hasattr(owner, "ImageModel"):
                raise NotImplementedError(
                    "SingleComponentMH.run needs log_target bound to an SMCsampler (or the "
                    "prior=/image_model= keywords): arbitrary Python targets cannot run inside "
                    "the fused HIP kernel")
            prior = prior or owner.Prior
            image_model = image_model or owner.ImageModel
        return prior, image_model

    def _cmh(self, prior):
        """The smcdet_mh_params_t of this kernel, rebuilt only when a parameter
        attribute is rebound (the reference's SMCsampler assigns locs_min /
        locs_max once; every tensor parameter is read-only), so the per-step
        host path skips its tensor -> float conversions.  The struct is shared:
        a caller that changes a field works on a copy (from_buffer_copy)."""
        key = (id(prior), self.num_iters, id(self.locs_stdev), id(self.fluxes_stdev),
               id(self.fluxes_min), id(self.fluxes_max), id(self.locs_min), id(self.locs_max),
               id(prior.loc_prior.low), id(prior.loc_prior.high))
        hit = getattr(self, "_cmh_cached", None)
        if hit is not None and hit[0] == key:
            return hit[1]
        c = self._cmh_build(prior)
        # (the key's objects are kept alive with it, so their ids stay theirs)
        self._cmh_cached = (key, c, (prior, self.locs_stdev, self.fluxes_stdev, self.fluxes_min,
                                     self.fluxes_max, self.locs_min, self.locs_max,
                                     prior.loc_prior.low, prior.loc_prior.high))
        return c

    def _cmh_build(self, prior):
        c = _hip.MHC()
        c.num_iters = int(self.num_iters)
        c.locs_stdev = _f32(self.locs_stdev)
        c.fluxes_stdev = _f32(self.fluxes_stdev.reshape(-1)[0])
        c.fluxes_min = _f32(self.fluxes_min.reshape(-1)[0])
        c.fluxes_max = _f32(self.fluxes_max.reshape(-1)[0])
        lo = self.locs_min if self.locs_min is not None else prior.loc_prior.low
        hi = self.locs_max if self.locs_max is not None else prior.loc_prior.high
        lo = torch.as_tensor(lo).reshape(-1).cpu().float()
        hi = torch.as_tensor(hi).reshape(-1).cpu().float()
        c.locs_min_h, c.locs_min_w = float(lo[0]), float(lo[-1])
        c.locs_max_h, c.locs_max_w = float(hi[0]), float(hi[-1])
        return c

    def _acc_workspace(self, T, dev):
        """[2T] int32, zeroed once: the kernel leaves it zero after every call
        (per-tile accept counters + workgroup tickets, smcdet_hip.h)."""
        key = (T, str(dev))
        ws = self._acc_ws.get(key)
        if ws is None:
            ws = torch.zeros(2 * T, device=dev, dtype=torch.int32)
            self._acc_ws[key] = ws
        return ws

    @staticmethod
    def rate_row(H, W):
        """Row length of a persisted rate image: H*W, or H*W + 64 for tiles
        above the LDS budget, whose sweep works in the row in global memory
        (64 dummy cells for masked lanes, smcdet_hip.h)."""
        return H * W + (64 if H * W > _hip.MAX_TILE_PIXELS else 0)

    @classmethod
    def _rate_buffer(cls, buf, name, TN, data):
        if buf is None:
            return None
        row = cls.rate_row(data.shape[-2], data.shape[-1])
        if buf.numel() != TN * row or not buf.is_contiguous():
            raise ValueError(f"{name} must be a contiguous [numH,numW,N,{row}] buffer")
        return _hip.dev_f32(buf, name)

    def run(self, data, counts, locs, fluxes, temperature, log_target=None, *, prior=None,
            image_model=None, ancestors=None, replay=None, want_loglik=True, rate_in=None,
            rate_out=None, flags=0, go=None, tile_boxes=None, tail=None, tail_take=0):
        """kernel.py:26-130.  ancestors [numH,numW,N] (int64, optional) gathers
        the starting state (a fused resample); with the fused step's `tail`
        it may instead be an _hip.AncestorBins (the previous tile pass's bins:
        each wave of the sweep finds its own ancestor); replay = dict(comp, uloc, uflux,
        uacc) replays recorded draws; rate_in / rate_out [numH,numW,N,H*W]
        (optional) are persisted per-particle rate images: rate_in must be the
        images of (locs, fluxes), rate_out receives those of the result
        (ignored in full_recompute mode).  go (int32 device scalar, optional):
        the launch does nothing when *go == 0 (speculative enqueue, see
        SMCsampler.run).  tile_boxes [T,4] (optional): each tile's own
        location box (Prior pad_mode "partition").  tail (smcdet_smc_tail_t,
        optional; SingleComponentMH only): the temper / reweight / next
        resampling pass that follows in SMCsampler.run, run by the same
        launch (smcdet_mh_sweep_step) on the returned log-likelihoods;
        `temperature` is then updated in place; tail_take counters of the
        random stream are reserved for its resampling right after the
        sweep's own (tail.offset), the order of the separate launches."""
        prior, image_model = self._resolve(log_target, prior, image_model)
        data = _hip.dev_f32(data, "data")
        counts = _hip.dev_f32(counts, "counts")
        locs = _hip.dev_f32(locs, "locs")
        fluxes = _hip.dev_f32(fluxes, "fluxes")
        dev = locs.device
        temperature_arg = temperature
        temperature = _hip.dev_f32(torch.as_tensor(temperature, device=dev, dtype=torch.float32),
                                   "temperature")
        if tail is not None and not (isinstance(temperature_arg, torch.Tensor) and
                                     temperature.data_ptr() == temperature_arg.data_ptr()):
            raise ValueError("the fused SMC step updates `temperature` in place: pass the "
                             "sampler's contiguous float32 device tensor")
        nH, nW, N, S, _ = locs.shape
        T = nH * nW
        if temperature.numel() != T:
            raise ValueError(f"temperature has {temperature.numel()} entries, need {T}")
        if self.rng is None:
            self.rng = PhiloxStream()
        locs_out = torch.empty_like(locs)
        fluxes_out = torch.empty_like(fluxes)
        counts_out = None
        anc_p = None
        if isinstance(ancestors, _hip.AncestorBins):
            # the previous tile pass's bins: each wave of the sweep finds its
            # own ancestor (the fused step's tail carries the buffer)
            if tail is None:
                raise ValueError("AncestorBins ancestors need the fused SMC step (tail)")
            counts_out = torch.empty_like(counts)
            tail.anc_bins = _hip.ptr(ancestors.buf)
        elif ancestors is not None:
            ancestors = ancestors.to(device=dev, dtype=torch.int64).contiguous()
            counts_out = torch.empty_like(counts)
            anc_p = _hip.ptr(ancestors)
        acc = torch.empty(nH, nW, device=dev, dtype=torch.float32)
        acc_ws = self._acc_workspace(T, dev)
        ll = torch.empty(nH, nW, N, device=dev, dtype=torch.float32) if want_loglik else None
        rp = None
        keep = []
        if replay is not None:
            rc = replay["comp"].to(device=dev, dtype=torch.int32).contiguous()
            ru = [_hip.dev_f32(replay[k].to(dev), k) for k in ("uloc", "uflux", "uacc")]
            keep = [rc] + ru
            rp = _hip.ReplayC(_hip.ptr(rc).value, _hip.ptr(ru[0]).value, _hip.ptr(ru[1]).value,
                              _hip.ptr(ru[2]).value)
            # optional decision trace (MH sweep): replay["trace_loga"] float32 /
            # replay["trace_accept"] uint8 device tensors [K,numH,numW,N]
            for fld, dt in (("trace_loga", torch.float32), ("trace_accept", torch.uint8)):
                buf = replay.get(fld)
                if buf is not None:
                    if (not buf.is_cuda or buf.dtype != dt or not buf.is_contiguous()
                            or buf.numel() != self.num_iters * T * N):
                        raise ValueError(f"replay['{fld}'] must be a contiguous {dt} device "
                                         f"tensor of {self.num_iters * T * N} elements")
                    setattr(rp, fld, buf.data_ptr())
        off = self.rng.take(self.num_iters)
        if tail is not None and tail_take:
            tail.offset = self.rng.take(tail_take)
        if (self._entry == "smcdet_mh_sweep" and rate_out is None
                and data.shape[-1] * data.shape[-2] > _hip.MAX_TILE_PIXELS):
            # tiles above the LDS budget: the sweep needs working rate images
            rate_out = torch.empty(T * N * self.rate_row(data.shape[-2], data.shape[-1]),
                                   device=dev, dtype=torch.float32)
            rate_in = None
        cm, cp, ch = image_model._cmodel(), prior._cprior(), self._cmh(prior)
        extra_flags = flags
        flags = (_hip.SMCDET_MH_FULL_RECOMPUTE if self.full_recompute else 0) | self.debug_flags
        if self.component_by_count:
            flags |= _hip.SMCDET_MH_COMPONENT_BY_COUNT
        flags |= int(extra_flags)
        extra = []
        if self._entry == "smcdet_mh_sweep":
            if tile_boxes is not None:
                tile_boxes = _hip.dev_f32(tile_boxes.to(dev), "tile_boxes")
            extra = [_hip.ptr(tile_boxes)]
        elif tile_boxes is not None:
            raise NotImplementedError(f"{type(self).__name__}: per-tile location boxes "
                                      "(pad_mode='partition') need SingleComponentMH")
        entry = self._entry
        if tail is not None:
            if entry != "smcdet_mh_sweep":
                raise NotImplementedError(f"{type(self).__name__}: the fused SMC step runs "
                                          "SingleComponentMH sweeps")
            if ll is None:
                raise ValueError("the fused SMC step needs want_loglik=True")
            entry = "smcdet_mh_sweep_step"
            extra = extra + [_hip.ref(tail)]
        _hip.check(getattr(_hip.lib(), entry)(
            _hip.ref(cm), _hip.ref(cp), _hip.ref(ch), _hip.ptr(data), _hip.ptr(temperature),
            T, N, S, anc_p, _hip.ptr(counts), _hip.ptr(locs), _hip.ptr(fluxes),
            _hip.ptr(counts_out), _hip.ptr(locs_out), _hip.ptr(fluxes_out),
            _hip.ptr(self._rate_buffer(rate_in, "rate_in", T * N, data)),
            _hip.ptr(self._rate_buffer(rate_out, "rate_out", T * N, data)),
            self.rng.seed, off,
            _hip.ref(rp) if rp is not None else None, flags, _hip.ptr(ll), _hip.ptr(acc),
            _hip.ptr(acc_ws), _hip.ptr(go), *extra, _hip.stream_of(locs)), entry)
        del keep
        self.last_loglik = ll
        self.last_counts = counts_out if counts_out is not None else counts
        return [locs_out, fluxes_out, acc]


class SingleComponentMALA(SingleComponentMH):
    """smcdet/kernel.py:133-275: single-component Metropolis-adjusted Langevin
    moves.  The chosen source's (location, flux) is proposed from truncated
    normals centred at x + step^2/2 * grad log_target(x) and accepted with the
    Metropolis-Hastings ratio including both truncated-proposal densities.
    The reference obtains the gradient with torch.autograd.grad over the
    whole image in every iteration; the fused gfx950 kernel
    (smcdet_amd/csrc/mala_kernel.hip) evaluates it analytically over the
    moved source's PSF window.  `run` has SingleComponentMH.run's signature
    and return value."""
    _entry = "smcdet_mala_sweep"

    def __init__(self, num_iters, locs_step, fluxes_step, fluxes_min, fluxes_max):
        super().__init__(num_iters, locs_step, fluxes_step, fluxes_min, fluxes_max)
        self.locs_step = torch.tensor(locs_step)
        self.fluxes_step = torch.tensor(fluxes_step)

    @property
    def locs_stdev(self):  # the C ABI's proposal-scale fields carry the steps
        return self.locs_step

    @locs_stdev.setter
    def locs_stdev(self, v):
        self.locs_step = torch.as_tensor(v)

    @property
    def fluxes_stdev(self):
        return self.fluxes_step

    @fluxes_stdev.setter
    def fluxes_stdev(self, v):
        self.fluxes_step = torch.as_tensor(v)
