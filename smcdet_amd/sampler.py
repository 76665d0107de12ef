"""Likelihood-tempered SMC sampler (drop-in for smcdet/sampler.py:9-298).

`SMCsampler` keeps the reference constructor, methods (`initialize`,
`log_target`, `tempering_objective`, `temper`, `resample`, `mutate`,
`update_weights`, `prune`, `run`, `summarize`, posterior summaries) and the
public attributes drivers read after `run()`.  Every per-particle step runs as
a gfx950 kernel on the HIP device:

    initialize   -> smcdet_prior_sample + smcdet_loglik
    temper       -> smcdet_temper      (device root-find; the reference copies
                                        the log-likelihoods to the host for
                                        scipy brentq, sampler.py:99-125)
    update_weights -> smcdet_update_weights
    resample     -> smcdet_resample_index + smcdet_gather
    mutate       -> smcdet_mh_sweep    (all num_iters MH iterations, one launch)
    prune        -> smcdet_prune

`run()` uses the fused schedule: per SMC iteration one MH launch (which also
gathers the resampled ancestors and returns the log-likelihood of the new
state) and one per-tile launch doing temper + reweight + the next resampling
indices, with one 4-byte-per-tile device->host read for the loop condition.
The random-stream order is the same as calling the methods one by one.
"""
from __future__ import annotations

import torch

from . import _hip
from ._rng import PhiloxStream


def _scalar_or_tiles(v):
    """.item() as the reference prints it for a single tile; the per-tile
    values for a tiled image (where the reference's .item() raises)."""
    return v.item() if v.numel() == 1 else v.cpu()


class SMCsampler(object):
    def __init__(self, image, tile_dim, Prior, ImageModel, MutationKernel, num_catalogs,
                 ess_threshold_prop, resample_method, flux_detection_threshold, max_smc_iters,
                 print_every=5, *, seed=None, device=None, fused=True, persist_rate_images=True,
                 rate_refresh_every=8, stopping="lockstep", tile_boxes=None):
        # shapes the kernels cannot run raise here, naming the limit (before
        # anything touches the device)
        nt = (image.shape[0] * image.shape[1] if image.dim() == 4
              else (image.shape[0] // tile_dim) ** 2)
        # tiles above the LDS budget: SingleComponentMH sweeps with the M71
        # image model run from global memory
        from .images import M71ImageModel
        from .kernel import SingleComponentMALA, SingleComponentMH
        global_ok = (isinstance(MutationKernel, SingleComponentMH)
                     and not isinstance(MutationKernel, SingleComponentMALA)
                     and isinstance(ImageModel, M71ImageModel))
        _hip.check_limits(tile_dim, tile_dim, Prior.max_objects,
                          self._particles_per_tile(Prior, num_catalogs), nt,
                          getattr(ImageModel, "psf_radius", None), where="SMCsampler",
                          global_ok=global_ok)
        if stopping == "independent" and not fused:
            # the method-by-method schedule (resample / mutate / temper /
            # update_weights, fused=False) is the reference's lockstep loop;
            # freezing finished tiles lives in the fused step's kernels
            raise ValueError("stopping='independent' needs the fused schedule (fused=True)")
        if device is None:
            device = image.device if image.is_cuda else torch.device(
                "cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self.image = image.to(self.device, torch.float32)
        self.image_dim = image.shape[0]

        self.tile_dim = tile_dim
        self.num_tiles_per_side = self.image_dim // self.tile_dim
        if image.dim() == 4:  # pre-tiled [numH, numW, tile, tile] (see from_tiles)
            self.tiled_image = self.image.contiguous()
        else:
            self.tiled_image = (self.image.unfold(0, self.tile_dim, self.tile_dim)
                                .unfold(1, self.tile_dim, self.tile_dim).contiguous())
        self.tiles_shape = tuple(self.tiled_image.shape[:2])
        # per-tile location boxes [T,4]: explicit, or from the prior's pad_mode
        # ("partition": only the image's outer edges padded)
        if tile_boxes is None:
            tile_boxes = Prior.tile_boxes(self.tiles_shape, self.device) \
                if hasattr(Prior, "tile_boxes") else None
        self.tile_boxes = (None if tile_boxes is None else
                           tile_boxes.to(self.device, torch.float32).reshape(-1, 4).contiguous())
        if self.tile_boxes is not None and self.tile_boxes.shape[0] != self.tiles_shape[0] * \
                self.tiles_shape[1]:
            raise ValueError("tile_boxes must hold one (lo_h, lo_w, hi_h, hi_w) row per tile")

        self.Prior = Prior
        self.ImageModel = ImageModel
        self.MutationKernel = MutationKernel
        self.MutationKernel.locs_min = self.Prior.loc_prior.low
        self.MutationKernel.locs_max = self.Prior.loc_prior.high

        self.num_catalogs = num_catalogs
        self.ess_threshold = ess_threshold_prop * num_catalogs

        if resample_method not in {"multinomial", "systematic"}:
            raise ValueError("resample_method must be either multinomial or systematic.")
        self.resample_method = resample_method
        self.flux_detection_threshold = flux_detection_threshold
        self.max_smc_iters = max_smc_iters
        self.print_every = print_every
        self.has_run = False

        # "lockstep": the reference's rule (sampler.py:230) -- every tile is
        # resampled and mutated until all tiles reach temperature 1;
        # "independent": a tile stops (its final resampled particles stay put)
        # as soon as it reaches temperature 1 -- less work, same per-tile target
        if stopping not in {"lockstep", "independent"}:
            raise ValueError("stopping must be either lockstep or independent.")
        self.stopping = stopping
        self.rng = PhiloxStream(seed)
        self.MutationKernel.rng = self.rng
        self.fused = fused
        # Per-particle rate images kept on device between MH sweeps (double
        # buffered, [numH,numW,N,H*W] each): a sweep then starts from its
        # ancestor's image instead of re-rendering all sources.  Every
        # `rate_refresh_every`-th sweep re-renders from the state, bounding the
        # float32 drift of the incrementally maintained images.
        self.persist_rate_images = persist_rate_images
        self.rate_refresh_every = max(1, int(rate_refresh_every))
        self._rate = [None, None]
        self._rate_cur = 0
        self._rate_valid = False
        self._rate_age = 0
        self._fresh_loglik = None   # loglik of the current state, if already known
        self._pending_idx = None    # resampling indices computed by the fused tile launch
        # optional callback(sampler) after every SMC iteration (e.g. to take a
        # state_dict() checkpoint); runs the loop without speculation
        self.on_iteration = None

    @staticmethod
    def _particles_per_tile(Prior, num_catalogs):
        """The stratified initial draw holds num_catalogs particles per count."""
        return getattr(Prior, "num_counts", 1) * num_catalogs

    @classmethod
    def from_tiles(cls, tiles, *args, **kwargs):
        """A sampler over an explicit [numH, numW, tile, tile] grid of tiles
        (need not be square or contiguous in the sky: a rank's shard of a
        larger image, or a batch of independent images)."""
        if tiles.dim() != 4 or tiles.shape[2] != tiles.shape[3]:
            raise ValueError("tiles must be [numH, numW, tile, tile]")
        return cls(tiles, tiles.shape[2], *args, **kwargs)

    # ------------------------------------------------------------------ helpers
    @property
    def _T(self):
        return self.tiles_shape[0] * self.tiles_shape[1]

    def _zeros_tiles(self):
        return torch.zeros(*self.tiles_shape, device=self.device, dtype=torch.float32)

    def _method_code(self):
        return (_hip.SMCDET_RESAMPLE_SYSTEMATIC if self.resample_method == "systematic"
                else _hip.SMCDET_RESAMPLE_MULTINOMIAL)

    def _resample_offset(self, N):
        return self.rng.take(1 if self.resample_method == "systematic" else N)

    # ------------------------------------------------------------ the methods
    def _initial_particles(self):
        """Stratified prior draw (prior.py:25-64): [numH,numW,N,...]."""
        return self.Prior.sample_stratified(self.tiles_shape[0], self.num_catalogs,
                                            device=self.device, rng=self.rng,
                                            tiles_shape=self.tiles_shape,
                                            tile_boxes=self.tile_boxes)

    def initialize(self):
        """sampler.py:57-85."""
        nH, nW = self.tiles_shape
        self.counts, self.locs, self.fluxes = self._initial_particles()
        self.Prior.num = self.counts.shape[-1]
        self._rate_valid = False
        self.temperature_prev = self._zeros_tiles()
        self.temperature = self._zeros_tiles()
        self.loglik = self.ImageModel.loglikelihood(self.tiled_image, self.locs, self.fluxes)
        self._fresh_loglik = self.loglik
        N = self.counts.shape[-1]
        self.weights_log_unnorm = torch.zeros(nH, nW, N, device=self.device)
        self.weights = torch.full((nH, nW, N), 1.0 / N, device=self.device)
        self.log_normalizing_constant = self._zeros_tiles()
        self.ess = torch.full((nH, nW), float(N), device=self.device)
        self._pending_idx = None
        # SMC iteration at which each tile reached temperature 1 (-1: not yet)
        self.iters_per_tile = torch.full((nH, nW), -1, device=self.device, dtype=torch.int32)
        self._live_valid = False

    def log_target(self, data, counts, locs, fluxes, temperature):
        """sampler.py:87-91."""
        logprior = self.Prior.log_prob(counts, locs, fluxes, tile_boxes=self.tile_boxes)
        loglik = self.ImageModel.loglikelihood(data, locs, fluxes)
        return logprior + temperature.unsqueeze(-1) * loglik

    def tempering_objective(self, loglikelihood, delta):
        """sampler.py:93-97 (host helper; temper() solves it on device)."""
        log_numerator = 2 * ((delta * loglikelihood).logsumexp(0))
        log_denominator = (2 * delta * loglikelihood).logsumexp(0)
        return (log_numerator - log_denominator).exp() - self.ess_threshold

    def _current_loglik(self):
        if self._fresh_loglik is None:
            self._fresh_loglik = self.ImageModel.loglikelihood(self.tiled_image, self.locs,
                                                               self.fluxes)
        return self._fresh_loglik

    def temper(self):
        """sampler.py:99-125, root-finding on device."""
        self.loglik = self._current_loglik()
        # temperature / log Z are updated in place by the kernel (no per-step
        # device copies); temperature_prev is a second persistent buffer
        new_t = self.temperature
        prev_t = getattr(self, "temperature_prev", None)
        if prev_t is None or prev_t is new_t or prev_t.shape != new_t.shape:
            prev_t = torch.empty_like(new_t)
        _hip.check(_hip.lib().smcdet_temper(
            _hip.ptr(self.loglik), _hip.ptr(new_t), _hip.ptr(prev_t), self._T,
            self.loglik.shape[-1], float(self.ess_threshold), _hip.stream_of(new_t)),
            "smcdet_temper")
        self.temperature_prev = prev_t
        self.temperature = new_t
        self._live_valid = False
        self._mark_finished()

    def update_weights(self):
        """sampler.py:181-196."""
        N = self.loglik.shape[-1]
        self.weights_log_unnorm = torch.empty_like(self.loglik)
        self.weights = torch.empty_like(self.loglik)
        self.ess = torch.empty_like(self.temperature)
        self.log_normalizing_constant = self.log_normalizing_constant.clone()
        _hip.check(_hip.lib().smcdet_update_weights(
            _hip.ptr(self.loglik), _hip.ptr(self.temperature), _hip.ptr(self.temperature_prev),
            _hip.ptr(self.weights_log_unnorm), _hip.ptr(self.weights), _hip.ptr(self.ess),
            _hip.ptr(self.log_normalizing_constant), self._T, N, _hip.stream_of(self.weights)),
            "smcdet_update_weights")

    def resample_index(self, u=None):
        """Resampling indices [numH,numW,N] (sampler.py:128-150); u replays the
        uniforms ([numH,numW] systematic, [numH,numW,N] multinomial)."""
        N = self.weights.shape[-1]
        idx = torch.empty(self.weights.shape, device=self.device, dtype=torch.int64)
        off = self._resample_offset(N)
        if u is not None:
            u = _hip.dev_f32(u.to(self.device), "u")
        _hip.check(_hip.lib().smcdet_resample_index(
            _hip.ptr(self.weights), self._T, N, self._method_code(), self.rng.seed, off,
            _hip.ptr(u), _hip.ptr(idx), _hip.stream_of(idx)), "smcdet_resample_index")
        return idx

    def _gather(self, idx):
        idx = _hip.as_index(idx)  # (AncestorBins from a fused step: searched first)
        N = idx.shape[-1]
        S = self.locs.shape[-2]
        c, l, f = (torch.empty_like(self.counts), torch.empty_like(self.locs),
                   torch.empty_like(self.fluxes))
        _hip.check(_hip.lib().smcdet_gather(
            _hip.ptr(idx), self._T, N, S, _hip.ptr(self.counts), _hip.ptr(self.locs),
            _hip.ptr(self.fluxes), _hip.ptr(c), _hip.ptr(l), _hip.ptr(f), _hip.stream_of(idx)),
            "smcdet_gather")
        self.counts, self.locs, self.fluxes = c, l, f
        self.weights = torch.full_like(self.weights, 1.0 / N)
        self._fresh_loglik = None
        self._rate_valid = False  # persisted rate images describe the pre-gather state

    def resample(self):
        """sampler.py:127-169."""
        idx = self._pending_idx if self._pending_idx is not None else self.resample_index()
        self._pending_idx = None
        self._gather(idx)

    def _rate_buffers(self):
        """(rate_in, rate_out) for the next sweep, or (None, None)."""
        if not self.persist_rate_images or getattr(self.MutationKernel, "full_recompute", False):
            return None, None
        shape = (*self.locs.shape[:3],
                 self.MutationKernel.rate_row(self.tile_dim, self.tile_dim))
        for i in (0, 1):
            if self._rate[i] is None or tuple(self._rate[i].shape) != shape:
                self._rate[i] = torch.empty(shape, device=self.device, dtype=torch.float32)
                self._rate_valid = False
        fresh = (not self._rate_valid) or self._rate_age + 1 >= self.rate_refresh_every
        rin = None if fresh else self._rate[self._rate_cur]
        return rin, self._rate[1 - self._rate_cur]

    def mutate(self, ancestors=None, **fused):
        """sampler.py:171-179.  (fused: tail / tail_take of the fused SMC
        step, _step.)"""
        rin, rout = self._rate_buffers()
        kw = {} if rout is None else {"rate_in": rin, "rate_out": rout}
        if self.stopping == "independent":
            kw["flags"] = _hip.SMCDET_MH_SKIP_DONE
        if getattr(self, "_go", None) is not None:
            kw["go"] = self._go
        if self.tile_boxes is not None:
            kw["tile_boxes"] = self.tile_boxes
        kw.update(fused)
        self.locs, self.fluxes, self.mutation_acc_rates = self.MutationKernel.run(
            self.tiled_image, self.counts, self.locs, self.fluxes, self.temperature,
            self.log_target, ancestors=ancestors, **kw)
        if rout is not None:
            self._rate_cur = 1 - self._rate_cur
            self._rate_age = 0 if rin is None else self._rate_age + 1
            self._rate_valid = True
        if ancestors is not None:
            # fused resample: the gather happened inside the sweep.  The uniform
            # 1/N weights it implies are not materialised: the next
            # _temper_reweight (which always follows in run()) overwrites them.
            self.counts = self.MutationKernel.last_counts
        self._fresh_loglik = self.MutationKernel.last_loglik

    def _tr_prepare(self, with_resample, bins=False):
        """Output buffers of the temper / reweight (/ next resampling indices)
        pass, shared by its own launch (_temper_reweight) and the fused step
        (_step).  temperature / log Z are updated in place by the kernel (no
        per-step device copies); temperature_prev is a second persistent
        buffer.  bins: the next resampling as AncestorBins (the step's tail
        hands the bins to the next sweep, which searches the ancestors)."""
        new_t = self.temperature
        shape = tuple(self.counts.shape)
        prev_t = getattr(self, "temperature_prev", None)
        if prev_t is None or prev_t is new_t or prev_t.shape != new_t.shape:
            prev_t = torch.empty_like(new_t)
        self.weights_log_unnorm = torch.empty(shape, device=new_t.device, dtype=torch.float32)
        self.weights = torch.empty_like(self.weights_log_unnorm)
        if self.stopping != "independent" or getattr(self, "ess", None) is None or \
                self.ess.shape != new_t.shape:
            self.ess = torch.empty_like(new_t)
        # (independent stopping: updated in place -- a finished tile keeps the
        # ESS of its last step)
        live = self._live_ws()
        idx = None
        if with_resample and bins:
            idx = _hip.AncestorBins.empty(shape, new_t.device)
        elif with_resample:
            idx = torch.empty(shape, device=new_t.device, dtype=torch.int64)
        return prev_t, live, idx

    def _tr_finish(self, prev_t, live, idx):
        self.temperature_prev = prev_t
        self._pending_idx = idx
        self._live = live
        self._live_valid = True

    def _temper_reweight(self, with_resample):
        """temper + update_weights (+ next resampling indices), one launch."""
        self.loglik = self._current_loglik()
        N = self.loglik.shape[-1]
        prev_t, live, idx = self._tr_prepare(with_resample)
        off = self._resample_offset(N) if with_resample else 0
        new_t = self.temperature
        _hip.check(_hip.lib().smcdet_temper_reweight(
            _hip.ptr(self.loglik), _hip.ptr(new_t), _hip.ptr(prev_t),
            _hip.ptr(self.weights_log_unnorm), _hip.ptr(self.weights), _hip.ptr(self.ess),
            _hip.ptr(self.log_normalizing_constant), self._T, N, float(self.ess_threshold),
            self._method_code(), self.rng.seed, off, _hip.ptr(idx),
            _hip.SMCDET_SMC_FREEZE_DONE if self.stopping == "independent" else 0,
            _hip.ptr(self.iters_per_tile), int(getattr(self, "iter", 0)), _hip.ptr(live),
            _hip.ptr(getattr(self, "_go", None)), getattr(self, "_live_host", None),
            _hip.stream_of(new_t)), "smcdet_temper_reweight")
        self._tr_finish(prev_t, live, idx)

    # True (systematic resampling): the step's tile pass hands the next
    # resampling to the next sweep as bins + offset (AncestorBins), whose
    # waves search their own ancestors -- the tile pass skips the index search
    # (DESIGN.md §4.2); False: int64 indices, as smcdet_temper_reweight writes
    ancestor_bins = True

    # True: SMC iterations run as one launch (smcdet_mh_sweep_step: the MH
    # sweep's last workgroup per tile tempers, reweights and draws the next
    # indices); False (default): the sweep and the 512-thread tile kernel as
    # two back-to-back launches of the same entry point (SMCDET_SMC_TWO_LAUNCH),
    # measured 2.5% faster per C2 step on gfx950.  Same
    # results either way.
    fused_step = False

    def _step_entry(self):
        """The SMC step runs through smcdet_mh_sweep_step (one call: sweep +
        tile pass) -- the reference's own mutate / temper hooks are not
        overridden and the kernel is the MH sweep."""
        return (self.fused
                and getattr(self.MutationKernel, "_entry", None) == "smcdet_mh_sweep"
                and all(h not in self.__dict__ and getattr(type(self), h) is getattr(SMCsampler, h)
                        for h in ("mutate", "_temper_reweight", "_current_loglik")))

    def _step_fusable(self):
        """The step's tile pass runs inside the sweep's launch (fused_step and
        the entry; the C side still falls back to two launches for shapes it
        cannot fuse, smcdet_mh_sweep_step_fused)."""
        return self.fused_step and self._step_entry()

    def _step(self, idx, resample_u=None, replay=None):
        """One SMC iteration of the fused schedule (sampler.py:221-237: the
        resampling gather of idx, mutate, temper, update_weights, the next
        resampling indices).  Tests: resample_u [numH,numW] replays the next
        systematic offsets, replay the MH draws (SingleComponentMH.run)."""
        if not self._step_entry():
            if resample_u is not None or replay is not None:
                raise ValueError("resample_u / replay need SingleComponentMH's step entry")
            self.mutate(ancestors=idx)
            self._temper_reweight(with_resample=True)
            return
        N = self.counts.shape[-1]
        use_bins = self.ancestor_bins and self.resample_method == "systematic"
        prev_t, live, idx_next = self._tr_prepare(True, bins=use_bins)
        tail = _hip.SmcTailC()
        tail.temperature_prev = _hip.ptr(prev_t)
        tail.log_weights_unnorm = _hip.ptr(self.weights_log_unnorm)
        tail.weights = _hip.ptr(self.weights)
        tail.ess = _hip.ptr(self.ess)
        tail.log_norm_const = _hip.ptr(self.log_normalizing_constant)
        tail.ess_threshold = float(self.ess_threshold)
        tail.resample_method = self._method_code()
        tail.flags = ((_hip.SMCDET_SMC_FREEZE_DONE if self.stopping == "independent" else 0)
                      | (0 if self.fused_step else _hip.SMCDET_SMC_TWO_LAUNCH))
        tail.seed = self.rng.seed
        if use_bins:
            tail.bins_out = _hip.ptr(idx_next.buf)
        else:
            tail.idx = _hip.ptr(idx_next)
        ru = None
        if resample_u is not None:
            ru = _hip.dev_f32(torch.as_tensor(resample_u, device=self.device,
                                              dtype=torch.float32), "resample_u")
            tail.resample_u = _hip.ptr(ru)
        tail.finished_iter = _hip.ptr(getattr(self, "iters_per_tile", None))
        tail.live = _hip.ptr(live)
        tail.live_host = getattr(self, "_live_host", None)
        tail.iter = int(getattr(self, "iter", 0))
        take = 1 if self.resample_method == "systematic" else N
        extra = {} if replay is None else {"replay": replay}
        self.mutate(ancestors=idx, tail=tail, tail_take=take, **extra)
        del ru
        self.loglik = self._fresh_loglik
        self._tr_finish(prev_t, live, idx_next)

    def _live_ws(self):
        """The next of two [3] int32 buffers (zeroed once, alternating per
        call); the tile kernel leaves the number of tiles below temperature 1
        in [2] (smcdet_temper_reweight).  Two, so that a speculatively
        enqueued iteration can run while the previous count is read."""
        bufs = getattr(self, "_live_bufs", None)
        if bufs is None or bufs[0].device != self.temperature.device:
            bufs = [torch.zeros(3, device=self.temperature.device, dtype=torch.int32)
                    for _ in range(2)]
            self._live_bufs = bufs
            self._live_next = 0
        ws = bufs[self._live_next]
        self._live_next ^= 1
        return ws

    def _mark_finished(self):
        it = getattr(self, "iters_per_tile", None)
        if it is not None:
            done = (self.temperature >= 1) & (it < 0)
            it.masked_fill_(done, int(getattr(self, "iter", 0)))

    def prune(self, locs, fluxes):
        """sampler.py:198-219: detectable (flux > threshold) sources strictly
        inside the tile, compacted to the front; counts int64."""
        locs = _hip.dev_f32(locs, "locs")
        fluxes = _hip.dev_f32(fluxes, "fluxes")
        nH, nW, N, S, _ = locs.shape
        counts = torch.empty(nH, nW, N, device=locs.device, dtype=torch.int64)
        pl, pf = torch.empty_like(locs), torch.empty_like(fluxes)
        _hip.check(_hip.lib().smcdet_prune(
            _hip.ptr(locs), _hip.ptr(fluxes), nH * nW, N, S, float(self.tile_dim),
            float(self.flux_detection_threshold), _hip.ptr(counts), _hip.ptr(pl), _hip.ptr(pf),
            _hip.stream_of(locs)), "smcdet_prune")
        return counts, pl, pf

    def _print_progress(self):
        if self.iter % self.print_every == 0:
            acc = getattr(self, "mutation_acc_rates", None)
            msg = (f"iteration {self.iter}: "
                   f"temperature in [{round(self.temperature.min().item(), 2)}, "
                   f"{round(self.temperature.max().item(), 2)}]")
            if acc is not None:
                msg += (f", acceptance rate in [{round(acc.min().item(), 2)}, "
                        f"{round(acc.max().item(), 2)}]")
            print(msg)

    def _progress_capture(self, stream):
        """(event, pinned host copy) of this iteration's progress values
        [tau min, tau max, acc min, acc max], or None when it prints nothing."""
        if self.iter % self.print_every != 0:
            return None
        acc = getattr(self, "mutation_acc_rates", None)
        t = self.temperature
        vals = [t.min(), t.max()] + ([acc.min(), acc.max()] if acc is not None else [])
        host = torch.empty(len(vals), dtype=torch.float32, pin_memory=True)
        host.copy_(torch.stack(vals), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        return ev, host

    def _progress_emit(self, line):
        if line is None:
            return
        ev, host = line
        ev.synchronize()
        v = host.tolist()
        msg = (f"iteration {self.iter}: "
               f"temperature in [{round(v[0], 2)}, {round(v[1], 2)}]")
        if len(v) == 4:
            msg += f", acceptance rate in [{round(v[2], 2)}, {round(v[3], 2)}]"
        print(msg)

    # ------------------------------------------------------- speculative loop
    _SNAPSHOT = ("locs", "fluxes", "counts", "mutation_acc_rates", "_fresh_loglik", "loglik",
                 "weights", "weights_log_unnorm", "ess", "temperature_prev", "_pending_idx",
                 "_rate_cur", "_rate_age", "_rate_valid", "_live", "_live_next", "iter")
    _host_flags = None

    def _can_speculate(self):
        """The speculative loop needs the default stopping rule and schedule
        hooks (the distributed lockstep mode and instrumented test samplers
        replace them) and a kernel that honours the `go` predicate."""
        hooks = ("_keep_going", "_temper_reweight", "mutate")
        return (all(h not in self.__dict__ and getattr(type(self), h) is getattr(SMCsampler, h)
                    for h in hooks)
                and hasattr(self.MutationKernel, "_entry")
                and getattr(self, "on_iteration", None) is None)

    def _run_speculative(self):
        """sampler.py:230-237 without a host round trip per iteration: the
        next iteration is enqueued BEFORE the previous loop condition is known,
        predicated on the device-side count of unfinished tiles (`go`: the
        kernels return immediately when it is 0).  The tile kernel also writes
        the count into pinned, device-mapped host memory, which the host reads
        once that launch's event has completed -- while the GPU already works
        on the next iteration (no copy launch, which would queue behind the
        full-occupancy MH sweep).  When the count turns out to be 0, the enqueued
        iteration did nothing on the device and its host-side bookkeeping
        (attribute rebinding, random-stream offsets) is rolled back, so the
        result is identical to the synchronous loop."""
        main = torch.cuda.current_stream(self.device)
        # the tile kernel writes each iteration's count of unfinished tiles into
        # pinned, device-mapped host memory (two slots, alternating) next to
        # its device copy
        if getattr(self, "_host_flags", None) is None:
            self._host_flags = _hip.HostInts(2)
        pinned = self._host_flags

        def launched():
            ev = torch.cuda.Event()
            ev.record(main)
            return ev

        # the initial temper/reweight has run synchronously with respect to the
        # host count: read it from the device copy once
        pinned[0] = int(self._live[2])
        live_prev, slot = self._live, 0
        ev_prev = None
        try:
            while self.iter <= self.max_smc_iters:
                snap = {k: getattr(self, k, None) for k in self._SNAPSHOT}
                rng_off = self.rng.offset
                self.iter += 1
                # the progress line of this iteration is printed only once the
                # previous iteration's count shows that it runs (the reference
                # prints it after its loop check); its values are captured now,
                # asynchronously, before the kernels update them in place
                line = self._progress_capture(main)
                self._go = live_prev[2:3]
                self._live_host = pinned.dev(1 - slot)
                idx, self._pending_idx = self._pending_idx, None
                self._step(idx)
                self._go = self._live_host = None
                ev = launched()
                if ev_prev is not None:
                    ev_prev.synchronize()
                if int(pinned[slot]) == 0:
                    # every tile had finished: the iteration just enqueued was a no-op
                    for k, v in snap.items():
                        setattr(self, k, v)
                    self.rng.offset = rng_off
                    break
                self._progress_emit(line)
                live_prev, ev_prev, slot = self._live, ev, 1 - slot
        finally:
            self._go = self._live_host = None
            torch.cuda.synchronize(self.device)

    def _keep_going(self):
        """sampler.py:230: continue while any tile has temperature < 1 (one
        device->host read per SMC iteration; after the fused temper launch the
        count of unfinished tiles is already on the device)."""
        if getattr(self, "_live_valid", False):
            return int(self._live[2]) > 0
        return bool((self.temperature < 1).any())

    def run(self):
        """sampler.py:221-256."""
        self.iter = 0
        print("starting...")
        self.initialize()
        if self.fused:
            self._temper_reweight(with_resample=True)
        else:
            self.temper()
            self.update_weights()
        self._loop()
        self._finish()

    def resume(self):
        """Continues a run from a state restored by load_state_dict() (a
        state_dict() taken between SMC iterations, e.g. by `on_iteration`):
        the rest of the loop, the final resample and prune.  With the rate
        images in the checkpoint the result equals the uninterrupted run's."""
        print("resuming...")
        self._loop()
        self._finish()

    def _loop(self):
        if self.fused and self._can_speculate() and getattr(self, "_live_valid", False):
            self._run_speculative()
        elif self.fused:
            while self._keep_going() and self.iter <= self.max_smc_iters:
                self.iter += 1
                self._print_progress()
                idx, self._pending_idx = self._pending_idx, None
                self._step(idx)
                if self.on_iteration is not None:
                    self.on_iteration(self)
        else:
            while self._keep_going() and self.iter <= self.max_smc_iters:
                self.iter += 1
                self._print_progress()
                self.resample()
                self.mutate()
                self.temper()
                self.update_weights()
                if self.on_iteration is not None:
                    self.on_iteration(self)

    def _finish(self):
        self.resample()
        self.pruned_counts, self.pruned_locs, self.pruned_fluxes = self.prune(self.locs,
                                                                              self.fluxes)
        self.has_run = True
        print("done!\n")

    # ------------------------------------------------------------ summaries
    @property
    def weights_intercount(self):
        """The final particle weights under the name the reference's drivers
        pass to Aggregate (experiments/m71/run_smc.py:141-151)."""
        return self.weights

    def posterior_mean_count(self, counts):
        return (self.weights * counts).sum(-1)

    def posterior_mean_total_flux(self, fluxes):
        return (self.weights * fluxes.sum(-1)).sum(-1)

    @property
    def posterior_predictive_total_observed_flux(self):
        return self.ImageModel.sample(self.locs, self.fluxes).sum([-2, -3]).squeeze()

    def summarize(self):
        if self.has_run is False:
            raise ValueError("Sampler hasn't been run yet.")
        vals, cnts = self.pruned_counts.unique(return_counts=True)
        print("posterior distribution of number of detectable stars within image boundary:")
        print(vals.cpu())
        print((cnts / self.pruned_counts.shape[-1]).round(decimals=3).cpu(), "\n")
        print("posterior mean total intrinsic flux (including undetectable and/or in padding) =",
              f"{_scalar_or_tiles(self.posterior_mean_total_flux(self.fluxes))}\n")
        print("posterior mean total intrinsic flux of detectable stars within image boundary =",
              f"{_scalar_or_tiles(self.posterior_mean_total_flux(self.pruned_fluxes))}\n")
        print(f"number of unique catalogs = {self.fluxes[0, 0].sum(-1).unique(dim=0).shape[0]}")

    # ------------------------------------------------------------ checkpoint
    _CKPT_TENSORS = ("counts", "locs", "fluxes", "weights", "weights_log_unnorm", "ess",
                     "log_normalizing_constant", "temperature", "temperature_prev", "loglik",
                     "mutation_acc_rates", "iters_per_tile", "_pending_idx", "_fresh_loglik")

    def state_dict(self, with_rate_images=True):
        """Sampler state between SMC iterations, for checkpoint / resume
        (copies of the device tensors: the kernels update some buffers in
        place).  with_rate_images keeps the persisted per-particle rate images
        ([numH,numW,N,H*W] float32), so that a resumed run continues exactly
        as the uninterrupted one; without them the next sweep re-renders."""
        st = {k: getattr(self, k).clone() for k in self._CKPT_TENSORS
              if torch.is_tensor(getattr(self, k, None))}
        if isinstance(getattr(self, "_pending_idx", None), _hip.AncestorBins):
            st["_pending_idx"] = self._pending_idx.to_index()
        st["iter"] = int(getattr(self, "iter", 0))
        st["rng"] = self.rng.state()
        if with_rate_images and self._rate_valid and self._rate[self._rate_cur] is not None:
            st["rate_image"] = self._rate[self._rate_cur].clone()
            st["rate_age"] = int(self._rate_age)
        return st

    def load_state_dict(self, st):
        """Restores a state_dict(); then resume() continues the run."""
        for k in self._CKPT_TENSORS:
            if k in st:
                setattr(self, k, st[k].to(self.device).clone())
            elif k in ("_pending_idx", "_fresh_loglik"):
                setattr(self, k, None)
        self.iter = int(st.get("iter", 0))
        self.rng.load_state(st["rng"])
        self.MutationKernel.rng = self.rng
        if self.fused and self._pending_idx is None and torch.is_tensor(getattr(self, "weights",
                                                                               None)):
            # a checkpoint without the pending indices (taken from a fused=False
            # run, or an older one): the fused schedule gathers the resampled
            # ancestors inside the next sweep, so draw them now from the
            # restored weights (resample -> mutate, sampler.py:231-235), at the
            # random-stream offset the unfused resample() would have taken
            self._pending_idx = self.resample_index()
        self._live_valid = False
        self._rate_valid = False
        if "rate_image" in st:
            r = st["rate_image"].to(self.device).clone()
            self._rate = [r, torch.empty_like(r)]
            self._rate_cur = 0
            self._rate_age = int(st.get("rate_age", 0))
            self._rate_valid = True
        self.Prior.num = self.counts.shape[-1]


class MHsampler(object):
    """Single-component MH chains (drop-in for smcdet/sampler.py:301-576).

    The reference runs one chain per tile at temperature 1 for
    num_samples_total - 1 iterations, stores every sample and keeps
    burn_thin_idx = arange(burnin, total, keep_every_k) of them
    (experiments/m71/run_mcmc.py:71-132: 50,000 samples per 8x8 image).  Here
    all tiles' chains run in one gfx950 launch per `print_every` iterations
    (smcdet_mh_chain), one wavefront per chain, and only the kept samples are
    written.  `num_chains=C` (keyword) runs C independent chains per tile; their
    kept samples are pooled along the sample axis (chain-major).

    Attributes after run(), as the reference: counts [nH,nW,M] (= max_objects),
    locs [nH,nW,M,S,2], fluxes [nH,nW,M,S], accept [nH,nW,total-1] (int32;
    [nH,nW,C,total-1] for C > 1), pruned_counts / pruned_locs / pruned_fluxes,
    has_run.  Before run(), locs / fluxes hold the initial state
    [nH,nW,C,S,2] / [nH,nW,C,S] (the reference's sample 0); assigning them
    sets the chains' starting points.
    """

    def __init__(self, image, tile_dim, Prior, ImageModel, locs_stdev, fluxes_stdev,
                 flux_detection_threshold, num_samples_total, num_samples_burnin,
                 keep_every_k: int = 1, print_every: int = 1000, *, num_chains=1, seed=None,
                 device=None):
        _hip.check_limits(tile_dim, tile_dim, Prior.max_objects,
                          R=getattr(ImageModel, "psf_radius", None), where="MHsampler")
        if device is None:
            device = image.device if image.is_cuda else torch.device(
                "cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self.image = image.to(self.device, torch.float32)
        self.image_dim = image.shape[0]
        self.tile_dim = tile_dim
        self.num_tiles_per_side = self.image_dim // self.tile_dim
        if image.dim() == 4:  # pre-tiled [numH, numW, tile, tile] (see from_tiles)
            self.tiled_image = self.image.contiguous()
        else:
            self.tiled_image = (self.image.unfold(0, self.tile_dim, self.tile_dim)
                                .unfold(1, self.tile_dim, self.tile_dim).contiguous())
        self.tiles_shape = tuple(self.tiled_image.shape[:2])

        self.Prior = Prior
        self.ImageModel = ImageModel
        self.locs_stdev = torch.tensor(locs_stdev)
        self.locs_min = Prior.loc_prior.low
        self.locs_max = Prior.loc_prior.high
        self.fluxes_stdev = torch.tensor(fluxes_stdev)
        self.fluxes_min = torch.tensor(Prior.flux_lower)
        self.fluxes_max = torch.tensor(Prior.flux_upper)
        self.flux_detection_threshold = flux_detection_threshold

        if num_samples_burnin >= num_samples_total:
            raise ValueError("num_samples_burnin must be smaller than num_samples_total.")
        self.num_samples_total = num_samples_total
        self.num_samples_burnin = num_samples_burnin
        self.keep_every_k = int(keep_every_k)
        self.burn_thin_idx = torch.arange(num_samples_burnin, num_samples_total,
                                          step=keep_every_k)
        self.num_chains = int(num_chains)
        self.rng = PhiloxStream(seed)

        nH, nW = self.tiles_shape
        C, S = self.num_chains, Prior.max_objects
        # Prior.sample(stratify_by_count=True, num_catalogs_per_count=1), first
        # catalog per chain (sampler.py:358-364); the target's counts are
        # max_objects (:343-348)
        _, l, f = Prior.sample_stratified(None, C, device=self.device, rng=self.rng,
                                          tiles_shape=(nH, nW))
        self.locs = l[:, :, :C].contiguous()
        self.fluxes = f[:, :, :C].contiguous()
        self.counts = torch.full((nH, nW, C), float(S), device=self.device)
        self.accept = torch.zeros(nH, nW, num_samples_total - 1, dtype=torch.int32,
                                  device=self.device)
        self.print_every = print_every
        self.has_run = False

    @classmethod
    def from_tiles(cls, tiles, *args, **kwargs):
        """Chains for a pre-tiled [numH, numW, tile, tile] stack -- e.g. a batch
        of independent cutouts [1, B, 8, 8] (run_mcmc.py's loop over images)."""
        if tiles.dim() != 4 or tiles.shape[2] != tiles.shape[3]:
            raise ValueError("tiles must be [numH, numW, tile, tile]")
        return cls(tiles, tiles.shape[2], *args, **kwargs)

    def log_target(self, data, counts, locs, fluxes):
        """sampler.py:390-394."""
        logprior = self.Prior.log_prob(counts, locs, fluxes)
        loglik = self.ImageModel.loglikelihood(data, locs, fluxes)
        return logprior + loglik

    def prune(self, locs, fluxes):
        """sampler.py:396-418 (the SMC sampler's rule, samples on axis 2)."""
        return SMCsampler.prune(self, locs, fluxes)

    def _cmh(self):
        c = _hip.MHC()
        c.num_iters = 1
        c.locs_stdev = float(self.locs_stdev)
        c.fluxes_stdev = float(self.fluxes_stdev)
        c.fluxes_min = float(self.fluxes_min)
        c.fluxes_max = float(self.fluxes_max)
        lo = torch.as_tensor(self.locs_min).reshape(-1).cpu().float()
        hi = torch.as_tensor(self.locs_max).reshape(-1).cpu().float()
        c.locs_min_h, c.locs_min_w = float(lo[0]), float(lo[-1])
        c.locs_max_h, c.locs_max_w = float(hi[0]), float(hi[-1])
        return c

    def run(self, *, replay=None):
        """sampler.py:420-493.  replay = dict(comp [K,nH,nW(,C)], uloc
        [K,nH,nW(,C),2], uflux / uacc [K,nH,nW(,C)]) replays recorded draws
        (K = num_samples_total - 1)."""
        nH, nW = self.tiles_shape
        T, C, S = nH * nW, self.num_chains, self.Prior.max_objects
        total, burnin, keep = self.num_samples_total, self.num_samples_burnin, self.keep_every_k
        K = total - 1
        M = (total - burnin + keep - 1) // keep
        dev = self.device
        ls = _hip.dev_f32(self.locs.reshape(nH, nW, C, S, 2).clone(), "locs")
        fs = _hip.dev_f32(self.fluxes.reshape(nH, nW, C, S).clone(), "fluxes")
        counts = _hip.dev_f32(self.counts.reshape(nH, nW, C), "counts")
        lo = torch.empty(nH, nW, C, M, S, 2, device=dev)
        fo = torch.empty(nH, nW, C, M, S, device=dev)
        acc = torch.zeros(nH, nW, C, max(K, 1), dtype=torch.int32, device=dev)
        rp, keepalive = None, []
        if replay is not None:
            rc = replay["comp"].to(device=dev, dtype=torch.int32).contiguous()
            ru = [_hip.dev_f32(replay[k].to(dev), k) for k in ("uloc", "uflux", "uacc")]
            keepalive = [rc] + ru
            rp = _hip.ReplayC(_hip.ptr(rc).value, _hip.ptr(ru[0]).value, _hip.ptr(ru[1]).value,
                              _hip.ptr(ru[2]).value)
        off = self.rng.take(max(K, 1))
        cm, cp, ch = self.ImageModel._cmodel(), self.Prior._cprior(), self._cmh()
        chunk = max(1, int(self.print_every))
        # chains stopped by an upper-edge proposal (the reference's NaN cache)
        frozen = torch.zeros(T * C, device=dev, dtype=torch.int32)
        k0 = 0
        while True:
            k1 = min(K, k0 + chunk)
            _hip.check(_hip.lib().smcdet_mh_chain(
                _hip.ref(cm), _hip.ref(cp), _hip.ref(ch), _hip.ptr(self.tiled_image), T, C, S,
                _hip.ptr(counts), _hip.ptr(ls), _hip.ptr(fs), total, burnin, keep, k0, k1,
                self.rng.seed, off, _hip.ref(rp) if rp is not None else None, _hip.ptr(lo),
                _hip.ptr(fo), _hip.ptr(acc), _hip.ptr(frozen), _hip.stream_of(ls)),
                "smcdet_mh_chain")
            if k1 >= K:
                break
            k0 = k1
            if k0 % chunk == 0:
                mean_acc = acc[..., k0 - chunk:k0].float().mean().item()
                print(f"iteration {k0}, acceptance rate in past {chunk} iters = {mean_acc:.2f}\n")
        del keepalive
        self.accept = acc[..., :K][:, :, 0] if C == 1 else acc[..., :K]
        self.frozen = frozen.reshape(nH, nW, C)
        self.locs = lo.reshape(nH, nW, C * M, S, 2)
        self.fluxes = fo.reshape(nH, nW, C * M, S)
        self.counts = torch.full((nH, nW, C * M), float(S), device=dev)
        self.pruned_counts, self.pruned_locs, self.pruned_fluxes = self.prune(self.locs,
                                                                              self.fluxes)
        self.has_run = True

    def posterior_mean_count(self, counts):
        return counts.float().mean(-1)

    def posterior_mean_total_flux(self, fluxes):
        return fluxes.sum(-1).mean()

    @property
    def posterior_predictive_total_observed_flux(self):
        return self.ImageModel.sample(self.locs, self.fluxes).sum([-2, -3]).squeeze()

    def summarize(self):
        if self.has_run is False:
            raise ValueError("Sampler hasn't been run yet.")
        vals, cnts = self.pruned_counts.unique(return_counts=True)
        print("posterior distribution of number of detectable stars within image boundary:")
        print(vals.cpu())
        print((cnts / self.pruned_counts.shape[-1]).round(decimals=3).cpu(), "\n")
        print("posterior mean total intrinsic flux (including undetectable and/or in padding) =",
              f"{self.posterior_mean_total_flux(self.fluxes).item()}\n")
        print("posterior mean total intrinsic flux of detectable stars within image boundary =",
              f"{self.posterior_mean_total_flux(self.pruned_fluxes).item()}\n")
