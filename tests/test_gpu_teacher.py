"""Teacher-forced MH replay at the headline geometry (VERDICT r2 next #1b).

tests/golden/mh_teacher_c2.npz (make_golden.py gen_mh_teacher) holds three
consecutive SMC iterations of the reference's own run on one 32x32 M71 tile
(S=10, N=1024, K=100; smcdet/sampler.py:221-256 with smcdet/kernel.py:26-130):
for each, the state the reference mutated, its temperature, every draw, every
accept decision and the returned state, plus the resampling indices linking
the iterations.  Each sweep here starts from the reference's recorded state
(teacher forcing), so a float32 near-tie cannot propagate from one SMC
iteration to the next.  Every decision the float64 oracle makes with a margin
|log U - min(log alpha, 0)| >= 1e-4 along the reference's trajectory (all of a
particle's decisions before its first smaller margin: `pin`) must be the
reference's -- about 306,000 decisions per mode -- in three modes:

* fresh: the incremental delta-likelihood sweep from a fresh render;
* persist: the incremental sweep whose rate images persist across the SMC
  iterations (the sampler's default): iteration i+1 gathers its ancestors
  (`ancestors` = the recorded indices) from the reference's returned state of
  iteration i and starts from the rate images the kernel left for them;
* full: SMCDET_MH_FULL_RECOMPUTE (every source re-rendered every step, the
  reference's arithmetic).

Particles with every decision pinned must also end in the reference's state.
"""
import numpy as np
import pytest
import torch

from tests._params import golden, p_m71_model, p_m71_mh, p_m71_prior

pytestmark = pytest.mark.gpu
DEV = "cuda"


def T(x, dtype=torch.float32):
    return torch.as_tensor(np.asarray(x)).to(DEV, dtype)


def N(t):
    return t.detach().cpu().numpy()


@pytest.fixture(scope="module")
def fx():
    return golden("mh_teacher_c2.npz")


def _sweep(d, i, full, ancestors=None, locs_in=None, fluxes_in=None, rate_in=None,
           rate_out=None):
    K, Np = int(d["K"]), int(d["N"])
    key = f"s{i}_"
    model, prior = p_m71_model(32), p_m71_prior(32, 10, 10, counts_rate=0.003125)
    mh = p_m71_mh(K, full_recompute=full)
    mh.locs_min, mh.locs_max = torch.tensor(d["locs_min"]), torch.tensor(d["locs_max"])
    loga = torch.full((K, 1, 1, Np), float("nan"), device=DEV)
    acc = torch.full((K, 1, 1, Np), 255, device=DEV, dtype=torch.uint8)
    replay = dict(comp=torch.as_tensor(d[key + "comp"].astype(np.int32)),
                  uloc=torch.as_tensor(d[key + "uloc"]), uflux=torch.as_tensor(d[key + "uflux"]),
                  uacc=torch.as_tensor(d[key + "uacc"]), trace_loga=loga, trace_accept=acc)
    locs = T(d[key + "locs0"]) if locs_in is None else locs_in
    fluxes = T(d[key + "fluxes0"]) if fluxes_in is None else fluxes_in
    kw = {}
    if rate_out is not None:
        kw = dict(rate_in=rate_in, rate_out=rate_out)
    l1, f1, rate = mh.run(T(d["image"]).reshape(1, 1, 32, 32), T(d[key + "counts"]), locs, fluxes,
                          T(np.full((1, 1), float(d[key + "tau"]))), prior=prior,
                          image_model=model, replay=replay, ancestors=ancestors, **kw)
    return N(l1)[0, 0], N(f1)[0, 0], N(acc)[:, 0, 0], N(loga)[:, 0, 0], N(rate)


def _check(d, i, l1, f1, acc, loga, eligible):
    """Decisions pinned by the oracle's margins (and, for persisted images,
    particles whose ancestor was fully pinned) equal the reference's."""
    K = int(d["K"])
    key = f"s{i}_"
    pin = d[key + "pin"].astype(np.int64)
    ref = d[key + "accept"][:, 0, 0]
    pinned = (np.arange(K)[:, None] < pin[None, :]) & eligible[None, :]
    assert np.all(acc[pinned] <= 1), "a pinned iteration was not run"
    bad = np.nonzero(pinned & (acc.astype(bool) != ref))
    assert bad[0].size == 0, (f"step {i}: {bad[0].size} pinned decisions differ, first at "
                              f"iteration {bad[0][:5]} particle {bad[1][:5]}, "
                              f"log alpha {loga[bad][:5]}")
    full = (pin == K) & eligible
    np.testing.assert_allclose(l1[full], d[key + "locs1"][0, 0][full], rtol=0, atol=2e-5)
    np.testing.assert_allclose(f1[full], d[key + "fluxes1"][0, 0][full], rtol=2e-6, atol=1e-3)
    return int(pinned.sum()), full


@pytest.mark.parametrize("full", [False, True], ids=["fresh", "full"])
def test_teacher_forced_mh_vs_reference(fx, full):
    steps = len(fx["steps"])
    total = 0
    for i in range(steps):
        l1, f1, acc, loga, _ = _sweep(fx, i, full)
        n, _ = _check(fx, i, l1, f1, acc, loga, np.ones(int(fx["N"]), bool))
        total += n
        # the kernel's log alpha is finite wherever it decided
        assert np.isfinite(loga[acc <= 1]).all()
    assert total >= 300_000, total


def test_teacher_forced_mh_persisted_rate_images(fx):
    """The sampler's schedule: rate images persist across SMC iterations and
    each sweep gathers its ancestors from the previous sweep's output."""
    K, Np, steps = int(fx["K"]), int(fx["N"]), len(fx["steps"])
    rate = [torch.empty(1, 1, Np, 32 * 32, device=DEV) for _ in range(2)]
    total = 0
    eligible = np.ones(Np, bool)
    prev_full = None
    for i in range(steps):
        if i == 0:
            l1, f1, acc, loga, _ = _sweep(fx, 0, False, rate_out=rate[0])
        else:
            key = f"s{i}_"
            idx = fx[key + "idx"]
            # the ancestors' states: the reference's returned state of the
            # previous iteration (teacher forcing); its rate images: what this
            # kernel left for the same particles
            pk = f"s{i - 1}_"
            l1, f1, acc, loga, _ = _sweep(
                fx, i, False, ancestors=T(idx.reshape(1, 1, Np), torch.int64),
                locs_in=T(fx[pk + "locs1"]), fluxes_in=T(fx[pk + "fluxes1"]),
                rate_in=rate[(i - 1) % 2], rate_out=rate[i % 2])
            eligible = prev_full[idx]
            assert eligible.mean() > 0.95
        n, prev_full = _check(fx, i, l1, f1, acc, loga, eligible)
        total += n
    assert total >= 290_000, total
