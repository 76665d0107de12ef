"""Multi-GPU tile sharding.

Independent image tiles shard embarrassingly: every tensor of the sampler
leads with the tile dimensions and no operation mixes tiles except the
reference's global stopping rule (`torch.any(temperature < 1)`,
smcdet/sampler.py:230).  One process per GPU (torchrun / torch.distributed,
backend "nccl" = RCCL on ROCm) owns a contiguous block of the row-major tile
list and runs its own fused SMC loop on it; there is no collective on the
data path.  Collectives:

* end of run: `gather_catalogs` assembles every rank's per-tile posterior
  (counts, locs, fluxes, weights, log Z, ESS, iterations, pruned catalogs) on
  the destination rank (one gather to `dst` per field, in its own dtype;
  ~31 MB for 64 tiles x 4096 particles x 10 sources, well under 1 ms on xGMI);
* optional lockstep (`lockstep=True`): one 4-byte all_reduce(MAX) per SMC
  iteration, reproducing the reference's rule that finished tiles keep
  mutating at temperature 1 until every tile of the image is done.

The default (independent stop per rank) does strictly less work and gives
each tile the same posterior target.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ._rng import rank_seed
from .sampler import SMCsampler


def _initialized():
    return dist.is_available() and dist.is_initialized()


def world():
    if _initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_tiles(num_tiles: int, world_size: int, rank: int):
    """Contiguous block [start, stop) of the row-major tile list for `rank`;
    the first num_tiles % world_size ranks get one extra tile."""
    base, extra = divmod(num_tiles, world_size)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def split_tiles(image: torch.Tensor, tile_dim: int) -> torch.Tensor:
    """[H, W] image -> [numH*numW, tile, tile] row-major tiles (sampler.py:28-31)."""
    t = image.unfold(0, tile_dim, tile_dim).unfold(1, tile_dim, tile_dim)
    return t.reshape(-1, tile_dim, tile_dim)


class TileShardedSMC:
    """SMCsampler over this rank's shard of an image's tiles."""

    def __init__(self, image, tile_dim, Prior, ImageModel, MutationKernel, num_catalogs,
                 ess_threshold_prop, resample_method, flux_detection_threshold, max_smc_iters,
                 print_every=10 ** 9, *, lockstep=False, seed=None, device=None, group=None,
                 rank=None, world_size=None, **sampler_kwargs):
        # rank / world_size default to the process group's (explicit values let
        # one process build any rank's shard, e.g. to check sharded == unsharded)
        r, w = world()
        self.rank = r if rank is None else int(rank)
        self.world_size = w if world_size is None else int(world_size)
        self.group = group
        self.lockstep = lockstep
        tiles = split_tiles(image, tile_dim)
        self.num_tiles = tiles.shape[0]
        self.tiles_per_side = image.shape[0] // tile_dim
        self.start, self.stop = shard_tiles(self.num_tiles, self.world_size, self.rank)
        local = tiles[self.start:self.stop]
        if local.shape[0] == 0:
            raise ValueError(f"rank {self.rank} has no tiles ({self.num_tiles} tiles, "
                             f"{self.world_size} ranks)")
        seed = rank_seed(seed, self.rank)
        # pad_mode "partition": each local tile keeps the box of its place in
        # the whole image's grid (SMCsampler would derive the boxes from the
        # flat 1 x T_local launch grid otherwise)
        if "tile_boxes" not in sampler_kwargs and hasattr(Prior, "tile_boxes"):
            tps = self.tiles_per_side
            boxes = Prior.tile_boxes((tps, tps))
            if boxes is not None:
                sampler_kwargs["tile_boxes"] = boxes[self.start:self.stop]
        self.sampler = SMCsampler.from_tiles(
            local.reshape(1, -1, tile_dim, tile_dim), Prior, ImageModel, MutationKernel,
            num_catalogs, ess_threshold_prop, resample_method, flux_detection_threshold,
            max_smc_iters, print_every, seed=seed, device=device, **sampler_kwargs)
        # lockstep: the reference's global stop through one 4-byte all_reduce
        # per SMC iteration (also at world size 1 when a process group exists,
        # so a single-rank job runs the same collective path)
        if lockstep and (self.world_size > 1 or _initialized()):
            self.sampler._keep_going = self._keep_going_global

    def _keep_going_global(self):
        s = self.sampler
        flag = (s.temperature < 1).any().to(torch.int32).reshape(1)
        if dist.get_backend(self.group) == "gloo":
            flag = flag.cpu()  # gloo reduces host tensors; RCCL the device flag
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
        return bool(flag.item())

    def run(self):
        self.sampler.run()
        return self

    def local_results(self):
        s = self.sampler
        T = s._T
        out = {
            "counts": s.counts.reshape(T, -1),
            "locs": s.locs.reshape(T, *s.locs.shape[2:]),
            "fluxes": s.fluxes.reshape(T, *s.fluxes.shape[2:]),
            "weights": s.weights.reshape(T, -1),
            "log_normalizing_constant": s.log_normalizing_constant.reshape(T),
            "ess": s.ess.reshape(T),
            "temperature": s.temperature.reshape(T),
            "pruned_counts": s.pruned_counts.reshape(T, -1),
            "pruned_locs": s.pruned_locs.reshape(T, *s.pruned_locs.shape[2:]),
            "pruned_fluxes": s.pruned_fluxes.reshape(T, *s.pruned_fluxes.shape[2:]),
            "iter": torch.full((T,), float(s.iter), device=s.device),
        }
        return out

    def gather_catalogs(self, dst=0):
        """All ranks' per-tile results on `dst`, shaped [numH, numW, ...] like
        the reference's single-process sampler attributes (None elsewhere)."""
        return gather_tile_results(self.local_results(), self.num_tiles, self.tiles_per_side,
                                   self.rank, self.world_size, dst=dst, group=self.group)


def gather_tile_results(local: dict, num_tiles: int, tiles_per_side, rank: int,
                        world_size: int, dst: int = 0, group=None):
    """Gathers dicts of [T_local, ...] tensors from every rank into
    [tiles_per_side, tiles_per_side, ...] tensors on `dst` ([num_tiles, ...]
    when tiles_per_side is None: independent images).  One `gather` to `dst`
    per field, in the field's own dtype (int64 counts stay exact), on the
    group's backend: RCCL moves device tensors over xGMI, gloo host tensors.
    Only `dst` receives (and allocates) the assembled catalog."""
    lead = (num_tiles,) if tiles_per_side is None else (tiles_per_side, tiles_per_side)
    if world_size == 1 and not _initialized():
        return {k: v.reshape(*lead, *v.shape[1:]) for k, v in local.items()}
    sizes = [shard_tiles(num_tiles, world_size, r) for r in range(world_size)]
    counts = [b - a for a, b in sizes]
    tmax = max(counts)
    # gloo gathers host tensors: device results are staged through the host
    host = dist.get_backend(group) == "gloo"
    out = {}
    for k in sorted(local):
        v = local[k]
        flat = v.reshape(v.shape[0], -1).contiguous()
        if host:
            flat = flat.cpu()
        # ranks hold T or T+1 tiles (shard_tiles): pad to a common shape
        pad = torch.zeros(tmax, flat.shape[1], dtype=flat.dtype, device=flat.device)
        pad[: flat.shape[0]] = flat
        bufs = [torch.empty_like(pad) for _ in range(world_size)] if rank == dst else None
        dist.gather(pad, gather_list=bufs, dst=dst, group=group)
        if rank == dst:
            full = torch.cat([b[:c] for b, c in zip(bufs, counts)], dim=0)
            full = full.reshape(num_tiles, *v.shape[1:]).to(v.device)
            out[k] = full.reshape(*lead, *v.shape[1:])
    return out if rank == dst else None


class ShardedBatchSMC:
    """BatchSMC (smcdet_amd.batch) over this rank's contiguous slice of B
    independent images [B, H, W] (the m71 / m71synthetic cutouts, BASELINE
    configs C4/C5): no collective until the end-of-run gather of the per-image
    results (`gather_results`, [B, ...] on `dst`)."""

    def __init__(self, images, Prior, ImageModel, MutationKernel, num_catalogs,
                 ess_threshold_prop, resample_method, flux_detection_threshold, max_smc_iters,
                 *, seed=None, device=None, group=None, **batch_kwargs):
        from .batch import BatchSMC
        self.rank, self.world_size = world()
        self.group = group
        self.num_images = images.shape[0]
        self.start, self.stop = shard_tiles(self.num_images, self.world_size, self.rank)
        if self.stop <= self.start:
            raise ValueError(f"rank {self.rank} has no images ({self.num_images} images, "
                             f"{self.world_size} ranks)")
        seed = rank_seed(seed, self.rank)
        self.batch = BatchSMC(images[self.start:self.stop], Prior, ImageModel, MutationKernel,
                              num_catalogs, ess_threshold_prop, resample_method,
                              flux_detection_threshold, max_smc_iters, seed=seed, device=device,
                              **batch_kwargs)

    def run(self):
        self.batch.run()
        return self

    def gather_results(self, dst=0):
        return gather_tile_results(self.batch.results(), self.num_images, None, self.rank,
                                   self.world_size, dst=dst, group=self.group)


class ShardedMCMC:
    """MHsampler (the reference's MCMC baseline, experiments/m71/run_mcmc.py)
    over this rank's contiguous slice of B independent cutouts [B, H, W]: one
    chain launch per rank (MHsampler.from_tiles), no collective until the
    end-of-run gather of the kept samples ([B, M, ...] on `dst`)."""

    def __init__(self, images, Prior, ImageModel, locs_stdev, fluxes_stdev,
                 flux_detection_threshold, num_samples_total, num_samples_burnin,
                 keep_every_k=1, *, seed=None, device=None, group=None, **mh_kwargs):
        from .sampler import MHsampler
        self.rank, self.world_size = world()
        self.group = group
        self.num_images = images.shape[0]
        self.start, self.stop = shard_tiles(self.num_images, self.world_size, self.rank)
        if self.stop <= self.start:
            raise ValueError(f"rank {self.rank} has no images ({self.num_images} images, "
                             f"{self.world_size} ranks)")
        seed = rank_seed(seed, self.rank)
        b = self.stop - self.start
        H = images.shape[-1]
        tiles = images[self.start:self.stop].reshape(1, b, H, H)
        self.sampler = MHsampler.from_tiles(
            tiles, Prior, ImageModel, locs_stdev, fluxes_stdev, flux_detection_threshold,
            num_samples_total, num_samples_burnin, keep_every_k, seed=seed, device=device,
            **mh_kwargs)

    def run(self):
        self.sampler.run()
        return self

    def local_results(self):
        """Per-image kept samples in the run_mcmc.py layout: counts [b, M],
        locs [b, M, S, 2], fluxes [b, M, S], acc_rate [b]."""
        s = self.sampler
        acc = s.accept.float().reshape(s.accept.shape[1], -1).mean(-1)
        return {"counts": s.counts[0], "locs": s.locs[0], "fluxes": s.fluxes[0],
                "pruned_counts": s.pruned_counts[0], "acc_rate": acc}

    def gather_results(self, dst=0):
        return gather_tile_results(self.local_results(), self.num_images, None, self.rank,
                                   self.world_size, dst=dst, group=self.group)
