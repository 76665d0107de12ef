"""The oracle's cached sweep (oracle/mh_oracle.c mh_oracle_sweep_cached) and
its float32 arithmetic-class build (libmh_oracle_f32.so), which make the
round-5 statistics targets (tests/golden/make_oracle_stats.py).

In float64 the cached sweep re-sums cached per-source PSF contributions in
source order and cached per-pixel terms in pixel order, so it must equal the
full re-render (the restatement of smcdet/kernel.py:26-130 pinned by the
reference's goldens) bit for bit.  The float32 build is a different
arithmetic, held to the decisions: same acceptance rates on the same draws
away from ties, log-likelihoods within float32 rounding of the float64 ones.
"""
import numpy as np
import pytest

from oracle import c_oracle as C
from oracle import smc_oracle as O
from tests._params import M71, o_m71_model, o_m71_prior


def _case(H, S, N, seed=1):
    rng = np.random.default_rng(seed)
    prior = o_m71_prior(H, S, S)
    model = o_m71_model(H)
    uloc = rng.random((1, 1, N, S, 2), dtype=np.float32)
    uflux = rng.random((1, 1, N, S), dtype=np.float32)
    counts, locs, fluxes = O.prior_sample_stratified(prior, 1, N, uloc, uflux)
    img = np.asarray(O.render_rate(locs[:, :, :1], fluxes[:, :, :1], model),
                     np.float32)[0, 0, :, :, 0] + np.float32(M71["background"])
    img = (img + rng.normal(0, 14, img.shape)).astype(np.float32).reshape(1, 1, H, H)
    return prior, model, img, counts, locs, fluxes


@pytest.mark.parametrize("H,S", [(8, 6), (32, 10), (16, 3), (8, 1)])
@pytest.mark.parametrize("tau", [0.02, 1.0])
def test_cached_sweep_equals_full_rerender(H, S, tau):
    prior, model, img, counts, locs, fluxes = _case(H, S, 96)
    mh = O.MHParams(40, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    a = C.mh_sweep(img, counts, locs, fluxes, tau, prior, model, mh, seed=77, threads=2,
                   frozen_out=True)
    b = C.mh_sweep(img, counts, locs, fluxes, tau, prior, model, mh, seed=77, threads=2,
                   frozen_out=True, cached=True)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    assert np.abs(a[0] - locs).max() > 0  # not vacuous


def test_cached_loglik_equals_full():
    prior, model, img, counts, locs, fluxes = _case(32, 10, 64)
    a = C.loglik(img, locs, fluxes, model, 2)
    out = np.empty(64)
    m, _, _ = C._pack(model, prior, O.MHParams(0, 1.0, 1.0, 0.1, 1.0))
    P = lambda v: v.ctypes.data_as(C.ctypes.c_void_p)  # noqa: E731
    lo, fl = np.ascontiguousarray(locs, np.float32), np.ascontiguousarray(fluxes, np.float32)
    C.lib().mh_oracle_loglik_cached(C.ctypes.byref(m), P(img), P(lo), P(fl), 1, 64, 10, 2, P(out))
    np.testing.assert_array_equal(a.ravel(), out)


def test_replayed_cached_sweep_edge_freeze():
    """A proposal on the box's upper edge freezes the particle (acc 2), in both
    sweeps alike."""
    prior, model, img, counts, locs, fluxes = _case(8, 3, 32)
    K = 6
    d = C.sweep_draws(5, 1, 32, K, 3)
    d["uloc"][2, 0, :4, 0] = 1.0  # clamp to the upper bound (distributions.py:44-48)
    mh = O.MHParams(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    a = C.mh_sweep(img, counts, locs, fluxes, 0.3, prior, model, mh, replay=d, threads=1,
                   frozen_out=True)
    b = C.mh_sweep(img, counts, locs, fluxes, 0.3, prior, model, mh, replay=d, threads=1,
                   frozen_out=True, cached=True)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_f32_build_close_to_f64():
    prior, model, img, counts, locs, fluxes = _case(32, 10, 128)
    # particles near the image's own catalog, so the log target has a
    # realistic magnitude (|tau * loglik| ~ 1e3, float32 ulp ~ 1e-4 nats; at
    # prior states it reaches 1e5 and decisions within its ulp flip)
    rng = np.random.default_rng(4)
    locs = (locs[:, :, :1] + rng.normal(0, 0.05, locs.shape)).astype(np.float32)
    locs = np.clip(locs, -4, 35.99).astype(np.float32)
    fluxes = (fluxes[:, :, :1] * (1 + 0.01 * rng.random(fluxes.shape))).astype(np.float32)
    img = np.asarray(O.render_rate(locs[:, :, :1], fluxes[:, :, :1], model),
                     np.float32)[0, 0].sum(-1) + np.float32(M71["background"])
    img = (img + rng.normal(0, 14, img.shape)).astype(np.float32).reshape(1, 1, 32, 32)
    l64 = C.loglik(img, locs, fluxes, model, 2)
    l32 = C.loglik(img, locs, fluxes, model, 2, arith="f32")
    np.testing.assert_allclose(l32, l64, rtol=5e-6)
    mh = O.MHParams(30, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    a = C.mh_sweep(img, counts, locs, fluxes, 0.4, prior, model, mh, seed=9, threads=2,
                   cached=True)
    b = C.mh_sweep(img, counts, locs, fluxes, 0.4, prior, model, mh, seed=9, threads=2,
                   cached=True, arith="f32")
    # same draws: the states agree to float32 proposal rounding, except for
    # the few particles where a near-tie decision went the other way
    close = (np.abs(b[0] - a[0]) <= 1e-3).all((-1, -2)) & \
        (np.abs(b[1] - a[1]) <= 1e-3 * (1 + np.abs(a[1]))).all(-1)
    assert close.mean() >= 0.95, close.mean()
    with pytest.raises(ValueError):
        C.mh_sweep(img, counts, locs, fluxes, 0.4, prior, model, mh, arith="f32")
