"""Host-side pieces of bench.py (no GPU): the C3 strong-scaling split that the
default run's c3_strong leg and --total-tiles use must partition the 64 tiles
exactly as the library's TileShardedSMC does (smcdet_amd.distributed), so the
union of the ranks' work at N = 2, 4, 8 is the one-GPU workload."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from smcdet_amd.distributed import shard_tiles  # noqa: E402


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 8, 64])
def test_c3_split_partitions_tiles_like_the_library(world):
    total = bench.C3_TILES
    seen = []
    for rank in range(world):
        ids = bench.shard(total, world, rank)
        a, b = shard_tiles(total, world, rank)
        assert ids == list(range(a, b))
        assert ids, "every rank owns at least one tile"
        seen += ids
    assert seen == list(range(total))


def test_c3_leg_is_part_of_the_default_run():
    old = sys.argv
    try:
        sys.argv = ["bench.py"]
        args = bench.parse()
    finally:
        sys.argv = old
    # the leg runs for the default C2 command (c3_leg's guard in main)
    assert (args.workload, args.kernel, args.total_tiles, args.tiles_per_gpu,
            args.no_c3) == ("c2", "mh", 0, 1, False)
