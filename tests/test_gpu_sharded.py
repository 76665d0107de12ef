"""The tile-sharded multi-GPU path (smcdet_amd/distributed.py) on
a device, and the C3 shape (a grid of 32x32 tiles through one SMCsampler).

* A rank's shard keys its draws by rank-local tile index and rank 0 keeps the
  base seed, so with independent stopping (each tile stops at temperature 1)
  rank 0's shard reproduces the single-process run's first tiles bit for
  bit, and rank r's shard reproduces a single-process run of its own tiles
  with rank_seed(seed, r).
* world_size 1 with a real gloo process group: gather_catalogs equals the
  single-process sampler's attributes.
* two processes (torchrun, gloo, both on cuda:0): the gathered catalogs equal
  the two single-process runs of the shards' tiles.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from tests._params import M71, p_m71_mh, p_m71_model, p_m71_prior

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H, N, K, S = 32, 256, 10, 10
FIELDS = ("counts", "locs", "fluxes", "weights", "log_normalizing_constant", "ess",
          "pruned_counts", "pruned_locs", "pruned_fluxes")


def grid_image(tps, seed=5):
    """tps x tps synthetic 32x32 M71 tiles (counts_rate 5/40^2, <= 10 sources)."""
    from smcdet_amd.prior import M71Prior
    model = p_m71_model(H)
    truth = M71Prior(min_objects=0, max_objects=100, counts_rate=0.003125, image_height=H,
                     image_width=H, flux_alpha=M71["flux_alpha"],
                     flux_lower=M71["flux_detection_threshold"], flux_upper=M71["flux_upper"],
                     pad=4)
    torch.manual_seed(seed)
    img = torch.empty(tps * H, tps * H, device="cuda")
    for a in range(tps):
        for b in range(tps):
            while True:
                c, l, f = truth.sample(num_catalogs=1, device="cuda")
                if int(c.max()) <= S:
                    break
            img[a * H:(a + 1) * H, b * H:(b + 1) * H] = model.sample(l, f)[0, 0, :, :, 0]
    return img


def sampler(image_or_tiles, seed, stopping="independent", tiles=False, n=N, k=K):
    from smcdet_amd.sampler import SMCsampler
    args = (p_m71_prior(H, S, S, counts_rate=0.003125), p_m71_model(H), p_m71_mh(k), n, 0.5,
            "systematic", M71["flux_detection_threshold"], 300)
    kw = dict(print_every=10 ** 9, seed=seed, stopping=stopping)
    if tiles:
        return SMCsampler.from_tiles(image_or_tiles, *args, **kw)
    return SMCsampler(image_or_tiles, H, *args, **kw)


def shard(image, seed, rank, world, **kw):
    from smcdet_amd.distributed import TileShardedSMC
    return TileShardedSMC(image, H, p_m71_prior(H, S, S, counts_rate=0.003125), p_m71_model(H),
                          p_m71_mh(K), N, 0.5, "systematic", M71["flux_detection_threshold"],
                          300, seed=seed, rank=rank, world_size=world, **kw)


def flat_tiles(s, f):
    v = getattr(s, f)
    return v.reshape(-1, *v.shape[2:]) if v.dim() >= 3 else v.reshape(-1)


def test_rank_shards_reproduce_single_process_tiles():
    from smcdet_amd._rng import rank_seed
    img = grid_image(2)
    single = sampler(img, 11)
    single.run()
    r0 = shard(img, 11, 0, 2, stopping="independent")
    r0.run()
    # rank 0 owns tiles 0, 1 (the top row): bit-equal to the single-process run
    for f in FIELDS:
        a, b = flat_tiles(r0.sampler, f), flat_tiles(single, f)[:2]
        assert torch.equal(a, b), f
    assert torch.equal(r0.sampler.iters_per_tile.flatten(), single.iters_per_tile.flatten()[:2])
    # rank 1 (tiles 2, 3) runs with its own seed: equal to a single-process
    # run of those tiles with that seed
    r1 = shard(img, 11, 1, 2, stopping="independent")
    r1.run()
    tiles = img.unfold(0, H, H).unfold(1, H, H).reshape(1, 4, H, H)[:, 2:4].contiguous()
    alone = sampler(tiles, rank_seed(11, 1), tiles=True)
    alone.run()
    for f in FIELDS:
        assert torch.equal(flat_tiles(r1.sampler, f), flat_tiles(alone, f)), f
    assert float(r1.sampler.temperature.min()) == 1.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_world1_gloo_gather_equals_single_process():
    import torch.distributed as dist
    img = grid_image(2, seed=6)
    single = sampler(img, 21, stopping="lockstep")
    single.run()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        from smcdet_amd.distributed import TileShardedSMC
        sh = TileShardedSMC(img, H, p_m71_prior(H, S, S, counts_rate=0.003125), p_m71_model(H),
                            p_m71_mh(K), N, 0.5, "systematic", M71["flux_detection_threshold"],
                            300, seed=21, lockstep=True)
        assert (sh.rank, sh.world_size) == (0, 1)
        sh.run()
        out = sh.gather_catalogs()
    finally:
        dist.destroy_process_group()
    for f in FIELDS:
        assert torch.equal(out[f].to(getattr(single, f).device), getattr(single, f)), f
    assert int(out["iter"].flatten()[0]) == single.iter


def _torchrun(tmp_path, nproc, **env_extra):
    """scripts/sharded_check.py under torchrun: every rank samples its shard,
    rank 0 gathers the catalogs (one gather per field) and saves them."""
    out = tmp_path / "gathered.pt"
    env = dict(os.environ, SMCDET_SHARD_OUT=str(out), PYTHONPATH=ROOT,
               **{k: str(v) for k, v in env_extra.items()})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.join(ROOT, "scripts", "sharded_check.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return torch.load(out, weights_only=True), r.stdout


def _check_gathered(got, img, shards, n=N, k=K, stopping="independent"):
    """The gathered catalogs equal single-process runs of each rank's tiles
    (with that rank's seed), field by field and bit for bit, in the
    single-process dtypes."""
    from smcdet_amd._rng import rank_seed
    nt = (img.shape[0] // H) ** 2
    tiles = img.unfold(0, H, H).unfold(1, H, H).reshape(1, nt, H, H)
    for rank, (a, b) in enumerate(shards):
        alone = sampler(tiles[:, a:b].contiguous(), rank_seed(31, rank), tiles=True, n=n, k=k,
                        stopping=stopping)
        alone.run()
        for f in FIELDS:
            want = flat_tiles(alone, f).cpu()
            have = got[f].reshape(nt, *got[f].shape[2:])[a:b] if got[f].dim() > 2 else \
                got[f].reshape(nt)[a:b]
            assert have.dtype == want.dtype, (f, have.dtype, want.dtype)
            assert torch.equal(have, want), (rank, f)


def test_two_process_gloo_gather_on_device(tmp_path):
    """torchrun --nproc-per-node 2 (gloo; both ranks on cuda:0): the gathered
    catalogs equal the single-process runs of the two shards' tiles."""
    got, _ = _torchrun(tmp_path, 2)
    _check_gathered(got, grid_image(2, seed=7), ((0, 2), (2, 4)))


def test_rccl_world1_lockstep_gather(tmp_path):
    """The RCCL code path on one GPU: a world-size-1
    "nccl" process group (device_id cuda:0) in a fresh torchrun process runs
    TileShardedSMC with the reference's lockstep stop (one RCCL all_reduce
    per SMC iteration) and gathers the catalogs with RCCL gathers of device
    tensors; they equal the single-process lockstep sampler's attributes."""
    got, log = _torchrun(tmp_path, 1, SMCDET_SHARD_BACKEND="nccl", SMCDET_SHARD_STOP="lockstep")
    assert "cuda:0" in log, log
    img = grid_image(2, seed=7)
    single = sampler(img, 31, stopping="lockstep")
    single.run()
    for f in FIELDS:
        have, want = got[f], getattr(single, f).cpu()
        assert have.dtype == want.dtype, (f, have.dtype, want.dtype)
        assert torch.equal(have, want), f
    assert int(got["iter"].flatten()[0]) == single.iter


def test_c3_two_process_gloo_full_size(tmp_path):
    """BASELINE configs[2] at full size over two ranks (torchrun, gloo, both
    on cuda:0): 64 32x32 tiles, N=4096, K=100, 32 tiles per rank; the
    gathered catalogs equal single-process runs of each rank's 32 tiles."""
    got, _ = _torchrun(tmp_path, 2, SMCDET_SHARD_TPS=8, SMCDET_SHARD_IMG_SEED=9,
                       SMCDET_SHARD_N=4096, SMCDET_SHARD_K=100)
    _check_gathered(got, grid_image(8, seed=9), ((0, 32), (32, 64)), n=4096, k=100)


def test_c3_shape_grid_of_32x32_tiles():
    """(Property checks only; the full-size C3 run is
    test_c3_full_size_lockstep.)  A 4x4 grid of 32x32 tiles (the C3 geometry
    at reduced N) through one SMCsampler with the reference's lockstep stop:
    every tile reaches
    temperature 1, log Z and ESS are finite, non-final ESS = rho*N, and each
    tile's result is independent of its neighbours (equal to the same tile
    sampled alone, independent stopping)."""
    img = grid_image(4, seed=8)
    s = sampler(img, 41, stopping="lockstep")
    esses, taus = [], []
    orig = s._temper_reweight

    def tr(with_resample, orig=orig):
        orig(with_resample)
        esses.append(s.ess.detach().clone())
        taus.append(s.temperature.detach().clone())

    s._temper_reweight = tr
    s.run()
    assert s.log_normalizing_constant.shape == (4, 4)
    assert float(s.temperature.min()) == 1.0
    assert torch.isfinite(s.log_normalizing_constant).all()
    it = s.iters_per_tile.cpu().numpy()
    assert (it > 0).all()
    E = torch.stack(esses).cpu().numpy()  # [iters+1, 4, 4]
    Tt = torch.stack(taus).cpu().numpy()
    for t in range(16):
        h, w = divmod(t, 4)
        # steps before the tile reached temperature 1 whose increment is
        # >= 1e-3 (below that brentq's xtol = 1e-6, reproduced on device, is
        # not small against the increment: the first step's ESS is ~10)
        inner = E[: it[h, w], h, w]
        delta = np.diff(np.concatenate([[0.0], Tt[: it[h, w], h, w]]))
        np.testing.assert_allclose(inner[delta >= 1e-3], 0.5 * N, rtol=0.01)
    # independent stopping, same seed: the first tile's stream is the same
    ind = sampler(img, 41, stopping="independent")
    ind.run()
    assert torch.equal(ind.iters_per_tile, s.iters_per_tile)
    # log Z is fixed once a tile reaches temperature 1 (delta = 0), so the two
    # modes agree on it even though lockstep keeps mutating finished tiles
    assert torch.equal(ind.log_normalizing_constant, s.log_normalizing_constant)


def test_c3_full_size_lockstep():
    """BASELINE configs[2] (C3) at its configured size through one
    SMCsampler, the reference's tiling (smcdet/sampler.py:28-31) and lockstep
    stop (:230): an 8x8 grid of 32x32 tiles (a 256x256 image), N=4096, K=100.
    Every tile reaches temperature 1 with a finite log Z; every non-final step
    whose increment is >= 1e-3 has ESS = rho*N within 1%; the independent-stop
    run of the same image and seed finishes every tile at the same iteration
    with the same log Z; and a sampler over the first two tiles alone
    reproduces them bit for bit (draws are keyed by tile-local particle)."""
    Nc, Kc = 4096, 100
    img = grid_image(8, seed=10)
    s = sampler(img, 51, stopping="lockstep", n=Nc, k=Kc)
    esses, taus = [], []
    orig = s._temper_reweight

    def tr(with_resample, orig=orig):
        orig(with_resample)
        esses.append(s.ess.detach().clone())
        taus.append(s.temperature.detach().clone())

    s._temper_reweight = tr
    s.run()
    assert s.locs.shape == (8, 8, Nc, S, 2)
    assert float(s.temperature.min()) == 1.0
    assert torch.isfinite(s.log_normalizing_constant).all()
    assert torch.isfinite(s.ess).all() and float(s.ess.min()) > 0
    it = s.iters_per_tile.cpu().numpy()
    assert (it > 0).all() and s.iter == it.max()
    E = torch.stack(esses).cpu().numpy()
    Tt = torch.stack(taus).cpu().numpy()
    checked = 0
    for t in range(64):
        h, w = divmod(t, 8)
        inner = E[: it[h, w], h, w]
        delta = np.diff(np.concatenate([[0.0], Tt[: it[h, w], h, w]]))
        np.testing.assert_allclose(inner[delta >= 1e-3], 0.5 * Nc, rtol=0.01)
        checked += int((delta >= 1e-3).sum())
    assert checked >= 64 * 5
    ind = sampler(img, 51, stopping="independent", n=Nc, k=Kc)
    ind.run()
    assert torch.equal(ind.iters_per_tile, s.iters_per_tile)
    assert torch.equal(ind.log_normalizing_constant, s.log_normalizing_constant)
    tiles = img.unfold(0, H, H).unfold(1, H, H).reshape(1, 64, H, H)[:, :2].contiguous()
    two = sampler(tiles, 51, stopping="independent", tiles=True, n=Nc, k=Kc)
    two.run()
    for f in FIELDS:
        assert torch.equal(flat_tiles(two, f), flat_tiles(ind, f)[:2]), f


def test_partition_boxes_follow_the_grid_in_shards_and_batches():
    """with pad_mode="partition" a rank's tiles keep the
    location boxes of their places in the whole image's grid (not of the flat
    1 x T_local launch grid), so a sharded run equals the single-process run
    tile for tile; BatchSMC gives every independent image the full padded box
    (a 1x1 grid's partition)."""
    from smcdet_amd._rng import rank_seed
    from smcdet_amd.batch import BatchSMC
    from smcdet_amd.prior import M71Prior, partition_boxes
    from smcdet_amd.sampler import SMCsampler

    def prior():
        return M71Prior(min_objects=S, max_objects=S, counts_rate=0.003125, image_height=H,
                        image_width=H, flux_alpha=M71["flux_alpha"], flux_lower=M71["flux_lower"],
                        flux_upper=M71["flux_upper"], pad=4, pad_mode="partition")

    img = grid_image(3, seed=12)            # 3x3 tiles: middle tiles have no padding
    args = (p_m71_model(H), p_m71_mh(K), N, 0.5, "systematic", M71["flux_detection_threshold"],
            300)
    single = SMCsampler(img, H, prior(), *args, print_every=10 ** 9, seed=61,
                        stopping="independent")
    single.run()
    boxes = partition_boxes((3, 3), H, H, 4, "cuda")
    assert torch.equal(single.tile_boxes, boxes)
    for rank in range(2):
        from smcdet_amd.distributed import TileShardedSMC
        sh = TileShardedSMC(img, H, prior(), *args, seed=61, rank=rank, world_size=2,
                            stopping="independent")
        assert torch.equal(sh.sampler.tile_boxes, boxes[sh.start:sh.stop]), rank
        sh.run()
        if rank == 0:
            for f in FIELDS:
                assert torch.equal(flat_tiles(sh.sampler, f),
                                   flat_tiles(single, f)[sh.start:sh.stop]), f
        else:
            tiles = img.unfold(0, H, H).unfold(1, H, H).reshape(1, 9, H, H)
            alone = SMCsampler.from_tiles(tiles[:, sh.start:sh.stop].contiguous(), prior(), *args,
                                          print_every=10 ** 9, seed=rank_seed(61, 1),
                                          stopping="independent",
                                          tile_boxes=boxes[sh.start:sh.stop])
            alone.run()
            for f in FIELDS:
                assert torch.equal(flat_tiles(sh.sampler, f), flat_tiles(alone, f)), f
    b = BatchSMC(img.unfold(0, H, H).unfold(1, H, H).reshape(9, H, H)[:3].contiguous(), prior(),
                 *args)
    full = partition_boxes((1, 1), H, H, 4, "cuda")
    assert torch.equal(b.sampler.tile_boxes, full.repeat(3, 1))
