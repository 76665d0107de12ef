"""Count-stratified SMC (CS-SMC; manuscript/manuscript.tex:312-356, Algorithm 2).

For every candidate count s in {s_min..s_max} a fixed-count SMC sampler (the
reference's SMCsampler with Prior.min_objects == Prior.max_objects == s,
smcdet/sampler.py:9-256) approximates p(z | x, s) and estimates the evidence
Z_s = p(x | s).  Bayes' rule gives p(s | x) ∝ p(s) Z_s, and the output holds N
catalogs drawn as s^n ~ p(s | x), z^n ~ p(z | x, s^n) (manuscript.tex:344-354).
The reference's experiments use this algorithm (counts 0..6,
manuscript.tex:566), but HEAD has no code for it: one SMCsampler over
min < max mixes the counts in a single population and crashes with systematic
resampling (smcdet/sampler.py:136-150).

MI355X layout: the strata are extra tiles.  Image tile (h, w) becomes NS
"stratum tiles" (h, w*NS + k), k = s - s_min, all in one [numH, numW*NS] batch
padded to S = s_max sources; the sources past a stratum's count have flux 0
and add nothing to the rate image.  The batch runs the ordinary fused SMC loop
(one MH launch and one per-tile temper/reweight/resample launch per
iteration, smcdet_amd/sampler.py).  The MH kernel draws the moved component
from 0..count-1 (SMCDET_MH_COMPONENT_BY_COUNT), which is the fixed-count
kernel with S = s exactly; the count-0 stratum has a constant likelihood,
tempers to 1 in one step and its log Z is log p(x | no sources).  One more
launch (smcdet_count_posterior, one workgroup per image tile) forms p(s | x)
and gathers the output catalogs.
"""
from __future__ import annotations

import copy
import math

import torch

from . import _hip
from .prior import PoissonProcessPrior
from .sampler import SMCsampler


def log_count_prior(Prior, dtype=torch.float32):
    """log p(s) for s = min..max: Poisson(counts_rate*(H+2pad)(W+2pad)) for
    Poisson-count priors (prior.py:91-97), DiscreteUniform(min, max) otherwise
    (prior.py:17-19, distributions.py:14-19)."""
    s = torch.arange(Prior.min_objects, Prior.max_objects + 1, dtype=torch.float64)
    if isinstance(Prior, PoissonProcessPrior):
        mu = float(Prior.poisson_mean)
        lp = s * math.log(mu) - mu - torch.lgamma(s + 1)
    else:
        lp = torch.full_like(s, -math.log(s.numel()))
    return lp.to(dtype)


class _StrataSampler(SMCsampler):
    """SMCsampler over the [numH, numW*NS] stratum tiles: the initial draw is
    the stratified prior draw of each image tile, split by count."""

    def __init__(self, *args, image_tiles_shape, num_strata, image_tile_boxes=None, **kwargs):
        # the strata of image tile t are stratum tiles t*NS .. t*NS+NS-1: they
        # share the image tile's location box
        if image_tile_boxes is not None:
            kwargs["tile_boxes"] = image_tile_boxes.repeat_interleave(num_strata, dim=0)
        super().__init__(*args, **kwargs)
        self._image_tiles_shape = image_tiles_shape
        self._num_strata = num_strata
        self._image_tile_boxes = image_tile_boxes

    @staticmethod
    def _particles_per_tile(Prior, num_catalogs):
        return num_catalogs  # one stratum (count) per stratum tile

    def _initial_particles(self):
        nH, nW = self._image_tiles_shape
        N = self.num_catalogs
        c, l, f = self.Prior.sample_stratified(nH, N, device=self.device, rng=self.rng,
                                               tiles_shape=(nH, nW),
                                               tile_boxes=self._image_tile_boxes)
        # [nH, nW, NS*N, ...] (counts in blocks of N, prior.py:47-54) -> stratum tiles
        S = l.shape[-2]
        T2 = nW * self._num_strata
        return c.reshape(nH, T2, N), l.reshape(nH, T2, N, S, 2), f.reshape(nH, T2, N, S)


class CountStratifiedSMC(object):
    """CS-SMC over the tiles of `image`, with counts Prior.min_objects ..
    Prior.max_objects.  Arguments as SMCsampler (num_catalogs_per_count = N
    particles per count stratum); `num_catalogs` output catalogs per tile
    (default N).  After run(): counts/locs/fluxes [numH,numW,num_catalogs,...]
    (equally weighted draws from the CS-SMC posterior), count_posterior
    [numH,numW,NS] = p(s|x), log_normalizing_constant_per_count [numH,numW,NS]
    = log Z_s, log_normalizing_constant [numH,numW] = log sum_s p(s) Z_s, the
    pruned catalogs, and the stratum populations strata_counts/locs/fluxes
    [numH,numW,NS*N,...] with weights_intercount = p(s|x)/N per particle."""

    def __init__(self, image, tile_dim, Prior, ImageModel, MutationKernel,
                 num_catalogs_per_count, ess_threshold_prop, resample_method,
                 flux_detection_threshold, max_smc_iters, print_every=5, *, num_catalogs=None,
                 seed=None, device=None, **sampler_kwargs):
        if Prior.max_objects < 1:
            raise ValueError("CS-SMC needs Prior.max_objects >= 1")
        if device is None:
            device = image.device if image.is_cuda else torch.device(
                "cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        image = image.to(self.device, torch.float32)
        if image.dim() == 4:
            tiles = image
        else:
            tiles = image.unfold(0, tile_dim, tile_dim).unfold(1, tile_dim, tile_dim)
        nH, nW = tiles.shape[:2]
        self.tiles_shape = (nH, nW)
        self.tile_dim = tile_dim
        self.tiled_image = tiles.contiguous()
        self.Prior = Prior
        self.ImageModel = ImageModel
        self.num_strata = Prior.max_objects - Prior.min_objects + 1
        self.counts_range = torch.arange(Prior.min_objects, Prior.max_objects + 1)
        self.num_catalogs_per_count = num_catalogs_per_count
        self.num_catalogs = num_catalogs or num_catalogs_per_count
        self.resample_method = resample_method
        self.flux_detection_threshold = flux_detection_threshold
        mh = copy.copy(MutationKernel)
        mh._acc_ws = {}
        mh.component_by_count = True
        self.MutationKernel = mh
        NS = self.num_strata
        strata_tiles = (self.tiled_image.unsqueeze(2).expand(nH, nW, NS, tile_dim, tile_dim)
                        .reshape(nH, nW * NS, tile_dim, tile_dim).contiguous())
        # Prior pad_mode "partition": each image tile its own location box
        boxes = sampler_kwargs.pop("tile_boxes", None)
        if boxes is None and hasattr(Prior, "tile_boxes"):
            boxes = Prior.tile_boxes((nH, nW), self.device)
        self.tile_boxes = boxes
        self.sampler = _StrataSampler(
            strata_tiles, tile_dim, Prior, ImageModel, mh, num_catalogs_per_count,
            ess_threshold_prop, resample_method, flux_detection_threshold, max_smc_iters,
            print_every, seed=seed, device=self.device, image_tiles_shape=(nH, nW),
            num_strata=NS, image_tile_boxes=boxes, **sampler_kwargs)
        if boxes is None:
            self.log_count_prior = log_count_prior(Prior).to(self.device)
        else:  # [T, NS]: a Poisson count mean scales with the tile's box area
            self.log_count_prior = Prior.log_count_prior_per_tile(boxes).to(
                device=self.device, dtype=torch.float32).contiguous()
        self.has_run = False

    def _per_tile(self, x, *rest):
        nH, nW = self.tiles_shape
        return x.reshape(nH, nW, self.num_strata, *rest)

    def combine(self, u_strata=None, u_pick=None):
        """p(s|x) and the output catalogs from the finished strata
        (manuscript.tex:344-354); u_strata / u_pick replay the uniforms."""
        s = self.sampler
        nH, nW = self.tiles_shape
        T, NS, N = nH * nW, self.num_strata, s.num_catalogs
        S = s.locs.shape[-2]
        n_out = self.num_catalogs
        logZ = s.log_normalizing_constant.reshape(T, NS).contiguous()
        probs = torch.empty(nH, nW, NS, device=self.device)
        idx = torch.empty(nH, nW, n_out, device=self.device, dtype=torch.int64)
        counts = torch.empty(nH, nW, n_out, device=self.device)
        locs = torch.empty(nH, nW, n_out, S, 2, device=self.device)
        fluxes = torch.empty(nH, nW, n_out, S, device=self.device)
        method = (_hip.SMCDET_RESAMPLE_SYSTEMATIC if self.resample_method == "systematic"
                  else _hip.SMCDET_RESAMPLE_MULTINOMIAL)
        off = s.rng.take(n_out)
        if u_strata is not None:
            u_strata = _hip.dev_f32(u_strata.to(self.device), "u_strata")
            u_pick = _hip.dev_f32(u_pick.to(self.device), "u_pick")
        _hip.check(_hip.lib().smcdet_count_posterior(
            _hip.ptr(logZ), _hip.ptr(self.log_count_prior), int(self.log_count_prior.dim() == 2),
            T, NS, N, S, n_out, method,
            s.rng.seed, off, _hip.ptr(u_strata), _hip.ptr(u_pick), _hip.ptr(s.counts),
            _hip.ptr(s.locs), _hip.ptr(s.fluxes), _hip.ptr(probs), _hip.ptr(idx),
            _hip.ptr(counts), _hip.ptr(locs), _hip.ptr(fluxes), _hip.stream_of(probs)),
            "smcdet_count_posterior")
        self.count_posterior = probs
        self.sample_index = idx
        self.counts, self.locs, self.fluxes = counts, locs, fluxes
        self.weights = torch.full((nH, nW, n_out), 1.0 / n_out, device=self.device)
        lz = logZ.reshape(nH, nW, NS)
        self.log_normalizing_constant_per_count = lz
        lcp = self.log_count_prior.reshape(nH, nW, NS) if self.log_count_prior.dim() == 2 \
            else self.log_count_prior
        self.log_normalizing_constant = torch.logsumexp(lz + lcp, -1)
        self.pruned_counts, self.pruned_locs, self.pruned_fluxes = s.prune(locs, fluxes)

    def run(self):
        s = self.sampler
        s.run()
        nH, nW = self.tiles_shape
        NS, N = self.num_strata, s.num_catalogs
        self.iter = s.iter
        self.temperature = self._per_tile(s.temperature)
        self.ess = self._per_tile(s.ess)
        self.mutation_acc_rates = self._per_tile(s.mutation_acc_rates) if hasattr(
            s, "mutation_acc_rates") else None
        S = s.locs.shape[-2]
        self.strata_counts = s.counts.reshape(nH, nW, NS * N)
        self.strata_locs = s.locs.reshape(nH, nW, NS * N, S, 2)
        self.strata_fluxes = s.fluxes.reshape(nH, nW, NS * N, S)
        self.combine()
        self.has_run = True
        return self

    @property
    def weights_intercount(self):
        """Weight of every stratum particle in the combined posterior:
        p(s|x)/N for each of the N equally weighted particles of stratum s."""
        N = self.sampler.num_catalogs
        return (self.count_posterior / N).repeat_interleave(N, dim=-1)

    def posterior_mean_count(self, counts):
        return (self.weights * counts).sum(-1)

    def posterior_mean_total_flux(self, fluxes):
        return (self.weights * fluxes.sum(-1)).sum(-1)

    def summarize(self):
        if self.has_run is False:
            raise ValueError("Sampler hasn't been run yet.")
        print("posterior distribution of the number of stars (including padding):")
        print(self.counts_range)
        print(self.count_posterior.reshape(-1, self.num_strata).cpu().round(decimals=3), "\n")
        vals, cnts = self.pruned_counts.unique(return_counts=True)
        print("posterior distribution of number of detectable stars within image boundary:")
        print(vals.cpu())
        print((cnts / self.pruned_counts.numel()).round(decimals=3).cpu(), "\n")
        print("posterior mean total intrinsic flux (including undetectable and/or in padding) =",
              f"{self.posterior_mean_total_flux(self.fluxes).flatten().tolist()}\n")
        print("posterior mean total intrinsic flux of detectable stars within image boundary =",
              f"{self.posterior_mean_total_flux(self.pruned_fluxes).flatten().tolist()}\n")
