"""Batched independent images.

The reference's drivers process their 332-1000 independent 8x8 images one at
a time, one SMCsampler per image (experiments/m71/run_smc.py:105-171,
experiments/m71synthetic/run_smc.py:129-162), which leaves a GPU almost idle:
an 8x8 image with 10,000 particles is 2.5 % of one MH launch's capacity.
`BatchSMC` runs B images as one [1, B] grid of tiles through the fused SMC
loop -- one MH launch and one per-tile temper/reweight/resample launch per
SMC iteration for the whole batch -- and writes the per-batch result files
the drivers write (run_smc.py:173-181).

Stopping: "independent" (default) freezes each image once it reaches
temperature 1, which is exactly a single-image run of the reference for that
image; "lockstep" keeps mutating finished images until the whole batch is
done, which is what the reference's SMCsampler does for the tiles of one
image (smcdet/sampler.py:230).
"""
from __future__ import annotations

import os
import time

import torch

from .sampler import SMCsampler

RESULT_FIELDS = ("runtime", "num_iters", "counts", "locs", "fluxes",
                 "posterior_predictive_total_flux")


class BatchSMC(object):
    """SMC over B independent images [B, H, W] (H = W = the tile size)."""

    def __init__(self, images, Prior, ImageModel, MutationKernel, num_catalogs,
                 ess_threshold_prop, resample_method, flux_detection_threshold, max_smc_iters,
                 *, stopping="independent", seed=None, device=None, **sampler_kwargs):
        if images.dim() != 3 or images.shape[1] != images.shape[2]:
            raise ValueError("images must be [B, H, H]")
        self.num_images = images.shape[0]
        B, H, _ = images.shape
        # every image is a whole image: with pad_mode "partition" each gets the
        # box of a 1x1 grid (padded on all four sides), not the box of its
        # column in the [1, B] launch grid
        if "tile_boxes" not in sampler_kwargs and hasattr(Prior, "tile_boxes"):
            box = Prior.tile_boxes((1, 1))
            if box is not None:
                sampler_kwargs["tile_boxes"] = box.repeat(B, 1)
        self.sampler = SMCsampler.from_tiles(
            images.reshape(1, B, H, H), Prior, ImageModel, MutationKernel, num_catalogs,
            ess_threshold_prop, resample_method, flux_detection_threshold, max_smc_iters,
            10 ** 9, stopping=stopping, seed=seed, device=device, **sampler_kwargs)
        self.ImageModel = ImageModel
        self.has_run = False

    def run(self):
        s = self.sampler
        torch.cuda.synchronize(s.device)
        t0 = time.perf_counter()
        s.run()
        torch.cuda.synchronize(s.device)
        self.runtime = time.perf_counter() - t0
        self.has_run = True
        return self

    def _flat(self, x):
        return x.reshape(self.num_images, *x.shape[2:])

    def results(self):
        """Per-image results in the drivers' layout (run_smc.py:106-111,
        160-168): counts [B,N], locs [B,N,S,2], fluxes [B,N,S],
        posterior_predictive_total_flux [B,N], num_iters [B] (SMC iterations
        until the image reached temperature 1; an image that never did, within
        max_smc_iters, gets the sampler's final `iter` = max_smc_iters + 1, what
        the reference drivers save as sampler.iter), runtime [B] (the batch's wall
        time shared equally: the images ran together), plus log Z, final ESS
        and the pruned catalogs."""
        if not self.has_run:
            raise ValueError("Sampler hasn't been run yet.")
        s = self.sampler
        B = self.num_images
        pp = self.ImageModel.sample(s.locs, s.fluxes).sum([2, 3])   # [1,B,N]
        return {
            "runtime": torch.full((B,), self.runtime / B),
            "num_iters": self._flat(torch.where(s.iters_per_tile < 0, int(s.iter),
                                                s.iters_per_tile)).to(torch.float32),
            "counts": self._flat(s.counts),
            "locs": self._flat(s.locs),
            "fluxes": self._flat(s.fluxes),
            "posterior_predictive_total_flux": self._flat(pp),
            "log_normalizing_constant": self._flat(s.log_normalizing_constant),
            "ess": self._flat(s.ess),
            "pruned_counts": self._flat(s.pruned_counts),
            "pruned_locs": self._flat(s.pruned_locs),
            "pruned_fluxes": self._flat(s.pruned_fluxes),
        }

    def save(self, directory, batch_index):
        return save_batch_results(self.results(), directory, batch_index)


def save_batch_results(results, directory, batch_index):
    """torch.save of each field as `{field}_{batch_index}.pt` on the CPU, the
    file layout of experiments/m71/run_smc.py:173-181 (results/smc/...)."""
    os.makedirs(directory, exist_ok=True)
    paths = []
    for k, v in results.items():
        p = os.path.join(directory, f"{k}_{batch_index}.pt")
        torch.save(v.detach().cpu(), p)
        paths.append(p)
    return paths


def load_batch_results(directory, batch_index, fields=RESULT_FIELDS):
    """Reads a batch back (tensor-only files: weights_only loading)."""
    return {k: torch.load(os.path.join(directory, f"{k}_{batch_index}.pt"), weights_only=True)
            for k in fields}
