"""GPU parity of MHsampler (smcdet/sampler.py:301-576; smcdet_amd/csrc/
chain_kernel.hip through smcdet_mh_chain): replays of the reference's
recorded chains (tests/golden/mcmc_*.npz, make_golden.py gen_mcmc) must keep
the same samples with every accept decision equal; a C2-geometry chain under
synthetic replayed draws must match the C oracle; chunked launches continue
the chains."""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from tests._params import (M71, golden, o_m71_mh, o_m71_model, o_m71_prior, p_m71_model,
                           p_m71_prior, tiles_of)

pytestmark = pytest.mark.gpu
DEV = "cuda"


def N(t):
    return t.detach().cpu().numpy()


def _sampler(image, td, S, d, **kw):
    from smcdet_amd.sampler import MHsampler
    s = MHsampler(torch.as_tensor(image, device=DEV), td, p_m71_prior(td, S, S), p_m71_model(td),
                  0.1, 2.5, M71["flux_detection_threshold"], int(d["total"]), int(d["burnin"]),
                  int(d["keep"]), **kw)
    return s


def _replay(d):
    return {k: torch.as_tensor(d[k]) for k in ("comp", "uloc", "uflux", "uacc")}


@pytest.mark.parametrize("name,td,S", [("mcmc_m71_8x8", 8, 4), ("mcmc_m71_tiles", 8, 3)])
def test_mh_chain_replay_vs_reference(name, td, S):
    d = golden(name + ".npz")
    s = _sampler(d["image"], td, S, d, print_every=10 ** 9)
    s.locs = torch.as_tensor(d["init_locs"][:, :, None], device=DEV)
    s.fluxes = torch.as_tensor(d["init_fluxes"][:, :, None], device=DEV)
    s.run(replay=_replay(d))
    np.testing.assert_array_equal(N(s.accept), d["accept"])
    np.testing.assert_allclose(N(s.locs), d["locs"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(N(s.fluxes), d["fluxes"], rtol=2e-6, atol=1e-3)
    np.testing.assert_array_equal(N(s.counts), d["counts"])
    np.testing.assert_array_equal(N(s.pruned_counts), d["pruned_counts"])
    np.testing.assert_allclose(N(s.pruned_locs), d["pruned_locs"], rtol=0, atol=2e-5)
    assert s.has_run


def test_mh_chain_chunked_equals_single_launch():
    """print_every chunks relaunch the kernel (re-rendered rate image, same
    Philox streams): the same chain up to float32 near-ties."""
    d = golden("mcmc_m71_8x8.npz")
    outs = []
    for pe in (10 ** 9, 37):
        s = _sampler(d["image"], 8, 4, d, print_every=pe, seed=5)
        s.run()
        outs.append((N(s.locs), N(s.accept)))
    assert (outs[0][1] == outs[1][1]).mean() > 0.97
    np.testing.assert_allclose(outs[0][0][:, :, :20], outs[1][0][:, :, :20], rtol=0, atol=1e-3)


def test_mh_chain_c2_vs_oracle():
    """32x32 tile, S=10, 400 iterations under synthetic replayed draws: the
    kernel's chain against the C restatement's (bench C2 geometry)."""
    H, S, total, burnin, keep = 32, 10, 401, 1, 4
    d = golden("mh_m71_32x32.npz")
    img = tiles_of(d["image"], H)
    rng = np.random.default_rng(7)
    K = total - 1
    rp = dict(comp=rng.integers(0, S, (K, 1, 1)).astype(np.int32),
              uloc=rng.random((K, 1, 1, 2)).astype(np.float32),
              uflux=rng.random((K, 1, 1)).astype(np.float32),
              uacc=rng.random((K, 1, 1)).astype(np.float32))
    init_l, init_f = d["locs0"][:, :, :1], d["fluxes0"][:, :, :1]
    oprior = o_m71_prior(H, S, S)
    ol, of_, oacc = c_oracle.mh_chain(img, np.full((1, 1), S, np.float32), init_l[:, :, 0],
                                      init_f[:, :, 0], oprior, o_m71_model(H), o_m71_mh(1), total,
                                      burnin, keep, rp)
    from smcdet_amd.sampler import MHsampler
    s = MHsampler(torch.as_tensor(d["image"], device=DEV), H, p_m71_prior(H, S, S),
                  p_m71_model(H), 0.1, 2.5, M71["flux_detection_threshold"], total, burnin, keep,
                  print_every=10 ** 9)
    s.locs = torch.as_tensor(init_l, device=DEV)
    s.fluxes = torch.as_tensor(init_f, device=DEV)
    s.run(replay={k: torch.as_tensor(v) for k, v in rp.items()})
    same = (N(s.accept) == oacc).mean()
    assert same > 0.99, same
    first = int(np.argmax(N(s.accept)[0, 0] != oacc[0, 0])) if same < 1 else K
    m = max(0, (first - burnin) // keep)
    np.testing.assert_allclose(N(s.locs)[:, :, :m], ol[:, :, :m], rtol=0, atol=1e-4)


def test_mh_chain_many_chains_and_images():
    """C chains x a batch of images in one launch: shapes, bounds, pooled
    samples, and independent streams per chain."""
    from smcdet_amd.sampler import MHsampler
    d = golden("mcmc_m71_tiles.npz")
    tiles = torch.as_tensor(tiles_of(d["image"], 8), device=DEV).reshape(1, 4, 8, 8)
    s = MHsampler.from_tiles(tiles, p_m71_prior(8, 3, 3), p_m71_model(8), 0.1, 2.5,
                             M71["flux_detection_threshold"], 1000, 500, 5, print_every=10 ** 9,
                             num_chains=8, seed=3)
    s.run()
    assert tuple(s.locs.shape) == (1, 4, 8 * 100, 3, 2)
    assert tuple(s.accept.shape) == (1, 4, 8, 999)
    lc = N(s.locs)
    assert lc.min() >= -4 and lc.max() < 12
    per_chain = lc.reshape(1, 4, 8, 100, 3, 2)
    assert not np.allclose(per_chain[:, :, 0], per_chain[:, :, 1])
    assert 0.05 < float(s.accept.float().mean()) < 0.99
    assert s.posterior_mean_count(s.pruned_counts).shape == (1, 4)


def test_mh_chain_poisson_many_chains_vs_oracle():
    """Poisson ImageModel + ParetoStarPrior (the basic family) chains, C=5 per
    tile (not a multiple of 4) on 2x2 tiles, replayed synthetic draws: every
    chain against the C restatement."""
    from oracle.smc_oracle import MHParams
    from smcdet_amd.sampler import MHsampler
    from tests._params import BASIC_FLUX_SCALE, o_basic_model, o_basic_prior, p_basic_model, \
        p_basic_prior
    H, S, C, total, burnin, keep = 8, 3, 5, 121, 20, 5
    K = total - 1
    d = golden("mh_basic_16x16.npz")
    img = tiles_of(d["image"], H)                                        # [2,2,8,8]
    rng = np.random.default_rng(3)
    init_l = (rng.random((2, 2, C, S, 2)) * 10 - 1).astype(np.float32)
    init_f = (BASIC_FLUX_SCALE * 0.9 * (1 + 3 * rng.random((2, 2, C, S)))).astype(np.float32)
    rp = dict(comp=rng.integers(0, S, (K, 2, 2, C)).astype(np.int32),
              uloc=rng.random((K, 2, 2, C, 2)).astype(np.float32),
              uflux=rng.random((K, 2, 2, C)).astype(np.float32),
              uacc=rng.random((K, 2, 2, C)).astype(np.float32))
    prior = p_basic_prior(H, S, S)
    prior.flux_lower, prior.flux_upper = BASIC_FLUX_SCALE * 0.9, 1e6
    s = MHsampler(torch.as_tensor(d["image"], device=DEV), H, prior, p_basic_model(H), 0.1, 100,
                  0.0, total, burnin, keep, print_every=10 ** 9, num_chains=C)
    s.locs = torch.as_tensor(init_l, device=DEV)
    s.fluxes = torch.as_tensor(init_f, device=DEV)
    s.run(replay={k: torch.as_tensor(v) for k, v in rp.items()})
    M = (total - burnin + keep - 1) // keep
    gl = N(s.locs).reshape(2, 2, C, M, S, 2)
    ga = N(s.accept)
    ok = 0
    for c in range(C):
        sub = {k: np.ascontiguousarray(v[:, :, :, c]) for k, v in rp.items()}
        ol, of_, oacc = c_oracle.mh_chain(img, np.full((2, 2), S, np.float32), init_l[:, :, c],
                                          init_f[:, :, c], o_basic_prior(H, S, S), o_basic_model(H),
                                          MHParams(1, 0.1, 100, BASIC_FLUX_SCALE * 0.9, 1e6),
                                          total, burnin, keep, sub)
        ok += (ga[:, :, c] == oacc).mean()
        same = (ga[:, :, c] == oacc).all(-1)
        np.testing.assert_allclose(gl[:, :, c][same], ol[same], rtol=0, atol=1e-3)
    assert ok / C > 0.99


def test_sharded_mcmc_single_rank_equals_mhsampler():
    """ShardedMCMC (smcdet_amd.distributed) on one rank is MHsampler.from_tiles
    over all cutouts, with the per-image results in run_mcmc.py's layout."""
    from smcdet_amd.distributed import ShardedMCMC
    from smcdet_amd.sampler import MHsampler
    d = golden("mcmc_m71_tiles.npz")
    imgs = torch.as_tensor(tiles_of(d["image"], 8), device=DEV).reshape(4, 8, 8)
    args = (p_m71_prior(8, 3, 3), p_m71_model(8), 0.1, 2.5, M71["flux_detection_threshold"],
            400, 100, 3)
    sh = ShardedMCMC(imgs, *args, seed=7, print_every=10 ** 9).run()
    res = sh.gather_results()
    ref = MHsampler.from_tiles(imgs.reshape(1, 4, 8, 8), *args, seed=7,  # rank 0 keeps the seed
                               print_every=10 ** 9)
    ref.run()
    M = (400 - 100 + 2) // 3
    assert tuple(res["locs"].shape) == (4, M, 3, 2)
    assert torch.equal(res["locs"], ref.locs[0]) and torch.equal(res["fluxes"], ref.fluxes[0])
    assert tuple(res["acc_rate"].shape) == (4,)


@pytest.mark.parametrize("print_every", [10 ** 9, 37], ids=["one-launch", "chunked"])
def test_mh_chain_edge_freeze_vs_reference(print_every):
    """The reference's MHsampler chains whose proposal landed on the prior
    box's upper edge (make_golden.py gen_mcmc_edge): rejected, then frozen for
    the rest of the run -- every accept flag and kept sample equal to the
    reference's, also when the run is chunked into launches of 37 iterations
    (the freeze is carried in the chains' `frozen` flags)."""
    d = golden("mcmc_m71_edge_tiles.npz")
    s = _sampler(d["image"], 8, 3, d, print_every=print_every)
    s.locs = torch.as_tensor(d["init_locs"][:, :, None], device=DEV)
    s.fluxes = torch.as_tensor(d["init_fluxes"][:, :, None], device=DEV)
    with __import__("contextlib").redirect_stdout(__import__("io").StringIO()):
        s.run(replay=_replay(d))
    np.testing.assert_array_equal(N(s.accept), d["accept"])
    np.testing.assert_allclose(N(s.locs), d["locs"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(N(s.fluxes), d["fluxes"], rtol=2e-6, atol=1e-3)
    np.testing.assert_array_equal(N(s.frozen)[..., 0], [[1, 0], [0, 1]])
