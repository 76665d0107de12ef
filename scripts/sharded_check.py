#!/usr/bin/env python
"""Multi-process check of the tile-sharded path on one GPU box, run by
tests/test_gpu_sharded.py under torchrun.  Every rank samples its contiguous
shard of a grid of 32x32 tiles (tests' grid_image(tps, seed)); rank 0 gathers
the catalogs and saves them to $SMCDET_SHARD_OUT.

Environment:
  SMCDET_SHARD_BACKEND  gloo (default; ranks may share cuda:0) or nccl (RCCL:
                        one rank per device -- a world of 1 on a one-GPU box)
  SMCDET_SHARD_TPS      tiles per side (default 2)
  SMCDET_SHARD_IMG_SEED grid_image seed (default 7)
  SMCDET_SHARD_N / _K   particles per tile / MH iterations (default 256 / 10)
  SMCDET_SHARD_STOP     independent (default) or lockstep (one all_reduce per
                        SMC iteration)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    backend = os.environ.get("SMCDET_SHARD_BACKEND", "gloo")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo")
        torch.cuda.set_device(0)
    try:
        from smcdet_amd.distributed import TileShardedSMC
        from tests._params import M71, p_m71_mh, p_m71_model, p_m71_prior
        from tests.test_gpu_sharded import H, S, grid_image
        tps = int(os.environ.get("SMCDET_SHARD_TPS", "2"))
        n = int(os.environ.get("SMCDET_SHARD_N", "256"))
        k = int(os.environ.get("SMCDET_SHARD_K", "10"))
        stop = os.environ.get("SMCDET_SHARD_STOP", "independent")
        img = grid_image(tps, seed=int(os.environ.get("SMCDET_SHARD_IMG_SEED", "7")))
        sh = TileShardedSMC(img, H, p_m71_prior(H, S, S, counts_rate=0.003125),
                            p_m71_model(H), p_m71_mh(k), n, 0.5, "systematic",
                            M71["flux_detection_threshold"], 300, seed=31,
                            stopping="independent" if stop == "independent" else "lockstep",
                            lockstep=stop == "lockstep")
        sh.run()
        out = sh.gather_catalogs(dst=0)
        if sh.rank == 0:
            dev = {k: str(v.device) for k, v in out.items()}
            torch.save({k: v.cpu() for k, v in out.items()}, os.environ["SMCDET_SHARD_OUT"])
            print("rank 0 gathered", backend, {k: tuple(v.shape) for k, v in out.items()},
                  "on", sorted(set(dev.values())))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
