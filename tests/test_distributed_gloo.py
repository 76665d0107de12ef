"""Multi-process (gloo, world_size 2 and 3, CPU) tests of the tile-sharded
path: shard arithmetic, tile splitting, the end-of-run catalog gather and the
lockstep stopping collective.  The HIP kernels are not called (no GPU here);
the per-rank sampler state is synthetic."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from smcdet_amd.distributed import (TileShardedSMC, gather_tile_results, shard_tiles,
                                    split_tiles)


def test_shard_tiles_cover_exactly():
    for n in (1, 7, 64, 100):
        for w in (1, 2, 3, 8):
            if w > n:
                continue
            spans = [shard_tiles(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_split_tiles_row_major():
    img = torch.arange(16 * 16, dtype=torch.float32).reshape(16, 16)
    t = split_tiles(img, 8)
    assert t.shape == (4, 8, 8)
    assert torch.equal(t[1], img[0:8, 8:16])
    assert torch.equal(t[2], img[8:16, 0:8])


def _free_port():
    """A fresh file:// rendezvous for one process group (no TCP port to race
    for between picking it and binding it)."""
    import tempfile
    fd, path = tempfile.mkstemp(prefix="smcdet_gloo_")
    os.close(fd)
    os.unlink(path)
    return path


def _worker(rank, world, port, num_tiles, tps, q):
    dist.init_process_group("gloo", init_method=f"file://{port}", rank=rank, world_size=world)
    try:
        a, b = shard_tiles(num_tiles, world, rank)
        T = b - a
        tiles = torch.arange(a, b, dtype=torch.float32)
        local = {
            "counts": tiles[:, None].repeat(1, 5),                         # [T, N]
            "locs": tiles[:, None, None, None].repeat(1, 5, 3, 2) + 0.5,    # [T, N, S, 2]
            "log_normalizing_constant": -tiles,                            # [T]
            "pruned_counts": tiles[:, None].repeat(1, 5).to(torch.int64),  # int field
            # int64 beyond float32's 2^24: gathered in its own dtype, exact
            "big": tiles.to(torch.int64) + (1 << 40),
        }
        out = gather_tile_results(local, num_tiles, tps, rank, world, dst=0)
        if rank == 0:
            # numpy, not tensors: a tensor sent through a torch.multiprocessing
            # queue is fetched from the sender's process, which may have exited
            q.put({k: v.numpy().copy() for k, v in out.items()})
        else:
            assert out is None

        # lockstep stopping rule: any rank with a tile below temperature 1 keeps
        # every rank going (one 4-byte all_reduce per SMC iteration)
        class FakeSampler:
            temperature = torch.tensor([[1.0, 1.0 if rank == 0 else 0.5]])

        sh = TileShardedSMC.__new__(TileShardedSMC)
        sh.sampler, sh.group = FakeSampler(), None
        keep = sh._keep_going_global()
        q.put(("keep", rank, keep))
    finally:
        dist.destroy_process_group()


def _worker_images(rank, world, port, num_images, q):
    dist.init_process_group("gloo", init_method=f"file://{port}", rank=rank, world_size=world)
    try:
        a, b = shard_tiles(num_images, world, rank)
        ids = torch.arange(a, b, dtype=torch.float32)
        local = {"log_normalizing_constant": -ids, "counts": ids[:, None].repeat(1, 4),
                 "num_iters": ids + 1}
        out = gather_tile_results(local, num_images, None, rank, world, dst=0)
        q.put({k: v.numpy().copy() for k, v in out.items()} if rank == 0 else None)
    finally:
        dist.destroy_process_group()


def test_gather_independent_images_gloo():
    world, num_images = 3, 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_images, args=(r, world, port, num_images, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full = {k: torch.as_tensor(v) for k, v in next(g for g in got if g is not None).items()}
    ids = torch.arange(num_images, dtype=torch.float32)
    assert torch.equal(full["log_normalizing_constant"], -ids)
    assert full["counts"].shape == (num_images, 4)
    assert torch.equal(full["num_iters"], ids + 1)


@pytest.mark.parametrize("world", [2, 3])
def test_gather_and_lockstep_gloo(world):
    num_tiles, tps = 9, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, num_tiles, tps, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world + 1)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full = {k: torch.as_tensor(v) for k, v in next(g for g in got if isinstance(g, dict)).items()}
    keeps = [g for g in got if isinstance(g, tuple)]
    idx = torch.arange(num_tiles, dtype=torch.float32).reshape(tps, tps)
    assert torch.equal(full["counts"][..., 0], idx)
    assert full["locs"].shape == (tps, tps, 5, 3, 2)
    assert torch.equal(full["locs"][..., 0, 0, 0], idx + 0.5)
    assert torch.equal(full["log_normalizing_constant"], -idx)
    assert full["pruned_counts"].dtype == torch.int64
    assert full["big"].dtype == torch.int64
    assert torch.equal(full["big"], idx.to(torch.int64) + (1 << 40))
    assert all(k[2] is True for k in keeps)  # rank 1 (and 2) still below 1


def test_rank_seeds_distinct_and_rank0_identity():
    """under torchrun every rank's torch.manual_seed is the same;
    the kernels key draws by rank-local tile index, so the ranks' stream seeds
    must differ.  Rank 0 keeps the base seed (a one-rank shard reproduces the
    single-process sampler)."""
    from smcdet_amd._rng import rank_seed
    seeds = [rank_seed(12345, r) for r in range(64)]
    assert seeds[0] == 12345 and len(set(seeds)) == 64
    torch.manual_seed(0)
    a = [rank_seed(None, r) for r in range(2)]
    torch.manual_seed(0)
    b = [rank_seed(None, r) for r in range(2)]
    assert a[0] != a[1] and a == b  # each rank: same base from the same manual_seed
