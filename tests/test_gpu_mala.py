"""GPU parity of the fused MALA sweep (smcdet/kernel.py:133-275,
smcdet_amd/csrc/mala_kernel.hip) through the C ABI.

Against the reference: replays of its recorded draws (tests/golden/mala_*.npz,
make_golden.py gen_mala) must reproduce every accept decision and the final
states.  MALA moves by step^2/2 x gradient, so the float32 rounding of the
reference's autograd sums is amplified into the proposals (<= ~1e-3 relative
in the fixtures, see test_oracle_golden.py); state tolerances are set to that.
Against the C oracle at C2 geometry (replayed synthetic draws): the same
moves except for rare near-tie decisions.
"""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from oracle import smc_oracle as O
from tests._params import (M71, MALA_FIXTURES, golden, o_m71_model,
                           o_m71_prior, p_m71_model, p_m71_prior, p_mala_fixture_setup,
                           tiles_of)

pytestmark = pytest.mark.gpu
DEV = "cuda"


def T(x, dtype=torch.float32):
    return torch.as_tensor(np.asarray(x)).to(DEV, dtype)


def N(t):
    return t.detach().cpu().numpy()


def _replay(d):
    return dict(comp=torch.as_tensor(d["comp"]), uloc=torch.as_tensor(d["uloc"]),
                uflux=torch.as_tensor(d["uflux"]), uacc=torch.as_tensor(d["uacc"]))


@pytest.mark.parametrize("name", MALA_FIXTURES)
def test_mala_replay_vs_reference(name):
    d = golden(name + ".npz")
    td, model, prior, mala = p_mala_fixture_setup(name)
    t = T(tiles_of(d["image"], td))
    tau = T(np.full(t.shape[:2], float(d["tau"])))
    mala.locs_min, mala.locs_max = torch.tensor(d["locs_min"]), torch.tensor(d["locs_max"])
    l, f, acc = mala.run(t, T(d["counts"]), T(d["locs0"]), T(d["fluxes0"]), tau, prior=prior,
                         image_model=model, replay=_replay(d))
    np.testing.assert_array_equal(N(acc), d["acc"])
    np.testing.assert_allclose(N(l), d["locs1"], rtol=0, atol=2e-4)
    np.testing.assert_allclose(N(f), d["fluxes1"], rtol=1e-4, atol=2e-3)
    # the returned log-likelihood is that of the returned state (rate image
    # maintained incrementally: float32 update rounding)
    ll = model.loglikelihood(t, l, f)
    np.testing.assert_allclose(N(mala.last_loglik), N(ll), rtol=2e-6, atol=1e-3)


def _c2_case(N_, K, tau, seed):
    H, S = 32, 10
    d = golden("mh_m71_32x32.npz")
    oprior = o_m71_prior(H, S, S, counts_rate=0.003125)
    rng = np.random.default_rng(seed)
    counts, locs, fluxes = O.prior_sample_stratified(
        oprior, 1, N_, rng.random((1, 1, N_, S, 2)), rng.random((1, 1, N_, S)), np.float32)
    replay = dict(comp=rng.integers(0, S, (K, 1, 1, N_)).astype(np.int32),
                  uloc=rng.random((K, 1, 1, N_, 2)).astype(np.float32),
                  uflux=rng.random((K, 1, 1, N_)).astype(np.float32),
                  uacc=rng.random((K, 1, 1, N_)).astype(np.float32))
    img = tiles_of(d["image"], H)
    return H, S, oprior, img, counts.astype(np.float32), locs.astype(np.float32), \
        fluxes.astype(np.float32), replay


@pytest.mark.parametrize("tau", [0.05, 1.0])
def test_mala_vs_c_oracle_c2(tau):
    """C2 geometry (32x32, S=10), 256 particles x 20 iterations, the same
    replayed draws through the kernel and the C restatement."""
    Np, K = 256, 20
    H, S, oprior, img, counts, locs, fluxes, rp = _c2_case(Np, K, tau, 5)
    from oracle.smc_oracle import MHParams
    ol, of_, oacc = c_oracle.mala_sweep(img, counts, locs, fluxes, tau, oprior, o_m71_model(H),
                                        MHParams(K, 0.1, 2.5, M71["flux_lower"],
                                                 M71["flux_upper"]), replay=rp, threads=8)
    from smcdet_amd.kernel import SingleComponentMALA
    model, prior = p_m71_model(H), p_m71_prior(H, S, S, counts_rate=0.003125)
    mala = SingleComponentMALA(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    l, f, acc = mala.run(T(img), T(counts), T(locs), T(fluxes), T([[tau]]), prior=prior,
                         image_model=model, replay={k: torch.as_tensor(v) for k, v in rp.items()})
    close = (np.abs(N(l) - ol).max((-1, -2)) < 1e-3) & (np.abs(N(f) - of_).max(-1) <
                                                         1e-3 * (1 + np.abs(of_).max(-1)))
    assert close.mean() > 0.97, close.mean()
    assert abs(float(N(acc)[0, 0]) - float(oacc[0, 0])) < 0.05


def test_mala_rate_persistence_and_gather():
    """rate_in/rate_out and the ancestor gather: a sweep from persisted rate
    images equals a sweep that re-renders (same Philox stream), up to float32
    rate rounding, and gathers the ancestors' states."""
    from smcdet_amd._rng import PhiloxStream
    from smcdet_amd.kernel import SingleComponentMALA
    H, S, Np, K = 16, 4, 256, 20
    model, prior = p_m71_model(H), p_m71_prior(H, S, S)
    torch.manual_seed(3)
    truth = p_m71_prior(H, 0, 100)
    _, tl, tf = truth.sample(num_catalogs=1, device=DEV)
    img = model.sample(tl, tf)[:, :, :, :, 0].contiguous()
    counts, locs, fluxes = prior.sample(num_tiles_per_side=1, stratify_by_count=True,
                                        num_catalogs_per_count=Np, device=DEV)
    anc = torch.randint(0, Np, (1, 1, Np), device=DEV)
    rate = torch.empty(1, 1, Np, H * H, device=DEV)
    m0 = SingleComponentMALA(0, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    m0.run(img, counts, locs, fluxes, torch.ones(1, 1, device=DEV), prior=prior,
           image_model=model, rate_out=rate)
    outs = []
    for use_rate in (False, True):
        mala = SingleComponentMALA(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
        mala.rng = PhiloxStream(9)
        rout = torch.empty_like(rate)
        kw = dict(rate_in=rate, rate_out=rout) if use_rate else {}
        outs.append(mala.run(img, counts, locs, fluxes, torch.full((1, 1), 0.5, device=DEV),
                             prior=prior, image_model=model, ancestors=anc, **kw)
                    + [mala.last_loglik, rout])
    same = (outs[0][0] - outs[1][0]).abs().amax((-1, -2)) < 1e-4
    assert float(same.float().mean()) > 0.97
    fresh = model.loglikelihood(img, outs[1][0], outs[1][1])
    np.testing.assert_allclose(N(outs[1][3]), N(fresh), rtol=2e-6, atol=1e-2)
    # K = 0 sweeps return the gathered ancestors unchanged
    m0.rng = PhiloxStream(1)
    l0, f0, _ = m0.run(img, counts, locs, fluxes, torch.ones(1, 1, device=DEV), prior=prior,
                       image_model=model, ancestors=anc)
    torch.testing.assert_close(l0, locs[:, :, anc[0, 0]], rtol=0, atol=0)
    torch.testing.assert_close(f0, fluxes[:, :, anc[0, 0]], rtol=0, atol=0)


def test_mala_smc_end_to_end():
    """SMCsampler with the MALA kernel (the reference's jsm2024-era pairing)
    runs to temperature 1 on the GPU, with finite evidence and states in the box."""
    from smcdet_amd.kernel import SingleComponentMALA
    from smcdet_amd.sampler import SMCsampler
    d = golden("mala_m71_8x8.npz")
    model, prior = p_m71_model(8), p_m71_prior(8, 4, 4)
    mala = SingleComponentMALA(20, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    s = SMCsampler(T(d["image"]), 8, prior, model, mala, 1024, 0.5, "systematic",
                   M71["flux_detection_threshold"], 100, print_every=10 ** 9, seed=4)
    s.run()
    assert float(s.temperature.min()) == 1.0
    assert np.isfinite(N(s.log_normalizing_constant)).all()
    lc = N(s.locs)
    assert lc.min() >= -4 and lc.max() < 12
    assert s.mutation_acc_rates is not None


def test_mala_component_by_count_keeps_padding():
    """CS-SMC mode (SMCDET_MH_COMPONENT_BY_COUNT) in the MALA kernel: padded
    sources (index >= count) never move, count-0 particles never move."""
    from smcdet_amd._rng import PhiloxStream
    from smcdet_amd.kernel import SingleComponentMALA
    torch.manual_seed(3)
    H, Np = 8, 256
    model, prior = p_m71_model(H), p_m71_prior(H, 0, 4)
    img = 104.15 + 14 * torch.randn(1, 1, H, H, device=DEV)
    counts, locs, fluxes = prior.sample(num_tiles_per_side=1, stratify_by_count=True,
                                        num_catalogs_per_count=Np, device=DEV)
    mala = SingleComponentMALA(40, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    mala.component_by_count = True
    mala.rng = PhiloxStream(9)
    l1, f1, _ = mala.run(img, counts, locs, fluxes, torch.tensor([[0.5]], device=DEV),
                         prior=prior, image_model=model)
    c = N(counts)[0, 0]
    pad = np.arange(4)[None] >= c[:, None]
    moved = (N(l1)[0, 0] != N(locs)[0, 0]).any(-1) | (N(f1)[0, 0] != N(fluxes)[0, 0])
    assert not moved[pad].any()
    assert not moved[c == 0].any()
    assert moved[~pad].mean() > 0.3
    # incrementally maintained rate image: MALA's drift moves bright sources
    # by whole pixels and large flux steps, so the float32 update rounding is
    # larger than for MH's local moves
    ll = model.loglikelihood(img, l1, f1)
    np.testing.assert_allclose(N(mala.last_loglik), N(ll), rtol=2e-5, atol=1e-3)


def test_mala_batch_independent_vs_lockstep():
    """Batched images with the MALA kernel: independent stopping (tile freeze
    + SMCDET_MH_SKIP_DONE) draws the same streams as lockstep, so log Z and
    finishing iterations agree exactly for every image."""
    from smcdet_amd.batch import BatchSMC
    from smcdet_amd.kernel import SingleComponentMALA
    torch.manual_seed(5)
    H, B = 8, 4
    model = p_m71_model(H)
    truth = p_m71_prior(H, 0, 20)
    ims = []
    for b in range(B):
        c, l, f = truth.sample(num_catalogs=1, device=DEV)
        ims.append(model.sample(l, f)[0, 0, :, :, 0])
    images = torch.stack(ims)
    res = []
    for stopping in ("lockstep", "independent"):
        mala = SingleComponentMALA(10, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
        bs = BatchSMC(images, p_m71_prior(H, 4, 4), model, mala, 256, 0.5, "systematic",
                      M71["flux_detection_threshold"], 100, stopping=stopping, seed=21,
                      device=DEV).run()
        res.append(bs.results())
    np.testing.assert_array_equal(N(res[0]["num_iters"]), N(res[1]["num_iters"]))
    np.testing.assert_array_equal(N(res[0]["log_normalizing_constant"]),
                                  N(res[1]["log_normalizing_constant"]))


def test_mala_ragged_tiles_vs_oracle():
    """Ragged N (37, not a multiple of the 4 particles per workgroup) over a
    2x3 grid of tiles, replayed synthetic draws: kernel vs C restatement."""
    from oracle.smc_oracle import MHParams
    from smcdet_amd.kernel import SingleComponentMALA
    H, S, Np, K = 8, 3, 37, 15
    d = golden("mh_m71_tiles.npz")
    img = np.ascontiguousarray(np.concatenate([tiles_of(d["image"], H)] * 2, 1)[:, :3])  # [2,3,8,8]
    oprior = o_m71_prior(H, S, S)
    rng = np.random.default_rng(11)
    counts, locs, fluxes = O.prior_sample_stratified(
        oprior, 1, Np, rng.random((1, 1, Np, S, 2)), rng.random((1, 1, Np, S)), np.float32)
    rep = lambda a: np.ascontiguousarray(np.broadcast_to(a, (2, 3) + a.shape[2:]))  # noqa: E731
    counts, locs, fluxes = (rep(x).astype(np.float32) for x in (counts, locs, fluxes))
    rp = dict(comp=rng.integers(0, S, (K, 2, 3, Np)).astype(np.int32),
              uloc=rng.random((K, 2, 3, Np, 2)).astype(np.float32),
              uflux=rng.random((K, 2, 3, Np)).astype(np.float32),
              uacc=rng.random((K, 2, 3, Np)).astype(np.float32))
    tau = np.array([[0.2, 0.5, 1.0], [0.05, 0.7, 0.3]], np.float32)
    ol, of_, oacc = c_oracle.mala_sweep(img, counts, locs, fluxes, tau, oprior, o_m71_model(H),
                                        MHParams(K, 0.1, 2.5, M71["flux_lower"],
                                                 M71["flux_upper"]), replay=rp, threads=8)
    mala = SingleComponentMALA(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    l, f, acc = mala.run(T(img), T(counts), T(locs), T(fluxes), T(tau), prior=p_m71_prior(H, S, S),
                         image_model=p_m71_model(H),
                         replay={k: torch.as_tensor(v) for k, v in rp.items()})
    close = (np.abs(N(l) - ol).max((-1, -2)) < 1e-3) & (np.abs(N(f) - of_).max(-1) <
                                                         1e-3 * (1 + np.abs(of_).max(-1)))
    assert close.mean() > 0.97, close.mean()
    assert np.abs(N(acc) - oacc).max() <= 2.0 / Np + 1e-6
