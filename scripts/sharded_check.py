#!/usr/bin/env python
"""Two-rank check of the tile-sharded path on one GPU box (run by
tests/test_gpu_sharded.py under torchrun --nproc-per-node 2): gloo process
group, both ranks on cuda:0, a 2x2 grid of 32x32 tiles (tests'
grid_image(2, seed=7)), independent stopping, seed 31; rank 0 gathers the
catalogs and saves them to $SMCDET_SHARD_OUT."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    dist.init_process_group("gloo")
    try:
        torch.cuda.set_device(0)
        from smcdet_amd.distributed import TileShardedSMC
        from tests._params import M71, p_m71_mh, p_m71_model, p_m71_prior
        from tests.test_gpu_sharded import H, K, N, S, grid_image
        img = grid_image(2, seed=7)
        sh = TileShardedSMC(img, H, p_m71_prior(H, S, S, counts_rate=0.003125),
                            p_m71_model(H), p_m71_mh(K), N, 0.5, "systematic",
                            M71["flux_detection_threshold"], 300, seed=31,
                            stopping="independent")
        assert sh.world_size == 2 and sh.stop - sh.start == 2
        sh.run()
        out = sh.gather_catalogs(dst=0)
        if sh.rank == 0:
            torch.save({k: v.cpu() for k, v in out.items()}, os.environ["SMCDET_SHARD_OUT"])
            print("rank 0 gathered", {k: tuple(v.shape) for k, v in out.items()})
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
