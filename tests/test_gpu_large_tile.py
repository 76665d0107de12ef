"""Tiles above the LDS budget: 128x128 M71 tiles run
the global-memory paths -- the tile image read from global memory (L2
resident), the rate images in HBM (smcdet_hip.h: rate rows of H*W + 64),
smcdet_loglik / smcdet_render rendering 64-pixel chunks in registers -- where
the reference tiles any image (smcdet/sampler.py:25-31).  Checked against the
float64 oracle (likelihood, render), a replayed MH sweep decision by decision
(the kernel's decision trace vs the oracle's along the same draws), the C
oracle's end states, the maintained rate image against a fresh render, and a
whole SMC run to temperature 1."""
import numpy as np
import pytest
import torch

from oracle import smc_oracle as O
from tests._params import (M71, o_m71_model, o_m71_prior, p_m71_mh, p_m71_model, p_m71_prior)

pytestmark = pytest.mark.gpu
DEV = "cuda"
H = 128
S = 10


def T(x, dtype=torch.float32):
    return torch.as_tensor(np.asarray(x)).to(DEV, dtype)


def N_(t):
    return t.detach().cpu().numpy()


def truth_image(seed=3, n_stars=12):
    """A 128x128 M71 image of a dozen stars (1-30 nmgy) from the image model."""
    g = torch.Generator().manual_seed(seed)
    locs = torch.rand(1, 1, 1, n_stars, 2, generator=g) * (H - 8) + 4
    fluxes = torch.rand(1, 1, 1, n_stars, generator=g) * 29 + 1
    torch.manual_seed(seed)
    return p_m71_model(H).sample(locs.to(DEV), fluxes.to(DEV))[0, 0, :, :, 0]


def population(n, seed=4):
    prior = p_m71_prior(H, S, S, counts_rate=0.0004)
    torch.manual_seed(seed)
    return prior, prior.sample(num_tiles_per_side=1, stratify_by_count=True,
                               num_catalogs_per_count=n, device=DEV)


def test_loglik_and_render_128_vs_oracle():
    from smcdet_amd import _hip
    img = truth_image()
    prior, (c, l, f) = population(64)
    model = p_m71_model(H)
    ll = model.loglikelihood(img[None, None].contiguous(), l, f)
    ref = O.loglikelihood(N_(img)[None, None], N_(l), N_(f), o_m71_model(H))
    # 16,384-term float32 sums against float64
    np.testing.assert_allclose(N_(ll), ref, rtol=4e-6, atol=5e-3)
    rate = torch.empty(1, H, H, 64, device=DEV)
    _hip.check(_hip.lib().smcdet_render(_hip.ref(model._cmodel()), _hip.ptr(l), _hip.ptr(f), 1, 64,
                                        S, _hip.ptr(rate), _hip.stream_of(rate)), "render")
    rr = O.render_rate(N_(l), N_(f), o_m71_model(H))            # [1,1,H,W,N]
    np.testing.assert_allclose(N_(rate)[0], np.asarray(rr)[0, 0], rtol=2e-6, atol=1e-3)


def _replay(n, K, seed):
    g = torch.Generator().manual_seed(seed)
    return dict(comp=torch.randint(0, S, (K, 1, 1, n), generator=g, dtype=torch.int32),
                uloc=torch.rand(K, 1, 1, n, 2, generator=g),
                uflux=torch.rand(K, 1, 1, n, generator=g),
                uacc=torch.rand(K, 1, 1, n, generator=g))


@pytest.mark.parametrize("full", [False, True], ids=["incremental", "full"])
def test_mh_sweep_128_decisions_vs_oracle(full):
    """A replayed sweep (N=16, K=30, tau=0.3): every decision the float64
    oracle makes with a margin >= 1e-3 (all of a particle's decisions before
    its first smaller one) is the kernel's, and fully pinned particles end in
    the oracle's state."""
    img = truth_image()
    prior, (c, l, f) = population(16)
    K = 30
    mh = p_m71_mh(K, full_recompute=full)
    rp = _replay(16, K, 5)
    loga = torch.full((K, 1, 1, 16), float("nan"), device=DEV)
    acc = torch.full((K, 1, 1, 16), 255, device=DEV, dtype=torch.uint8)
    tiled = img[None, None].contiguous()
    l1, f1, _ = mh.run(tiled, c, l, f, T([[0.3]]), prior=prior, image_model=p_m71_model(H),
                       replay=dict(rp, trace_loga=loga, trace_accept=acc))
    ol, of, _, ologa, oacc = O.mh_sweep(
        N_(tiled), N_(c), N_(l), N_(f), np.full((1, 1), 0.3), o_m71_prior(H, S, S, 0.0004),
        o_m71_model(H), O.MHParams(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"]),
        rp["comp"].numpy(), rp["uloc"].numpy(), rp["uflux"].numpy(), rp["uacc"].numpy(),
        trace=True)
    with np.errstate(all="ignore"):
        marg = np.abs(np.log(rp["uacc"].numpy().astype(np.float64)) - np.minimum(ologa, 0))
    marg = np.where(np.isnan(marg), np.inf, marg)[:, 0, 0]
    low = marg < 1e-3
    pin = np.where(low.any(0), low.argmax(0), K)
    pinned = np.arange(K)[:, None] < pin[None, :]
    assert pinned.sum() >= 0.9 * K * 16
    got = N_(acc)[:, 0, 0]
    assert np.array_equal(got[pinned].astype(bool), oacc[:, 0, 0][pinned])
    assert 0.05 < got[got <= 1].mean() < 0.95
    fullp = pin == K
    np.testing.assert_allclose(N_(l1)[0, 0][fullp], ol[0, 0][fullp], rtol=0, atol=2e-5)
    np.testing.assert_allclose(N_(f1)[0, 0][fullp], of[0, 0][fullp], rtol=2e-6, atol=1e-3)


def test_mh_sweep_128_vs_c_oracle_and_rate_images():
    """N=256, K=50 replayed: the end states match the C oracle's except for
    float32 near-ties; the rate images the sweep maintained in global memory
    (persisted, then gathered by a second sweep through `ancestors`) equal a
    fresh render of the returned states."""
    from oracle import c_oracle
    from smcdet_amd import _hip
    img = truth_image(seed=6)
    n, K = 256, 50
    prior, (c, l, f) = population(n, seed=7)
    model = p_m71_model(H)
    tiled = img[None, None].contiguous()
    mh = p_m71_mh(K)
    row = mh.rate_row(H, H)
    assert row == H * H + 64
    rate = [torch.empty(1, 1, n, row, device=DEV) for _ in range(2)]
    rp = _replay(n, K, 8)
    l1, f1, _ = mh.run(tiled, c, l, f, T([[0.5]]), prior=prior, image_model=model, replay=rp,
                       rate_out=rate[0])
    ol, of, _ = c_oracle.mh_sweep(N_(tiled), N_(c), N_(l), N_(f), 0.5,
                                  o_m71_prior(H, S, S, 0.0004), o_m71_model(H),
                                  O.MHParams(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"]),
                                  replay={k: v.numpy() for k, v in rp.items()})
    same = np.all(np.abs(N_(l1)[0, 0] - ol[0, 0]) <= 2e-5, axis=(-1, -2))
    assert same.mean() >= 0.95, same.mean()

    def fresh(locs, fluxes):
        out = torch.empty(1, H, H, n, device=DEV)
        _hip.check(_hip.lib().smcdet_render(_hip.ref(model._cmodel()), _hip.ptr(locs),
                                            _hip.ptr(fluxes), 1, n, S, _hip.ptr(out),
                                            _hip.stream_of(out)), "render")
        return N_(out)[0].reshape(H * H, n).T

    r0 = fresh(l1, f1)
    np.testing.assert_allclose(N_(rate[0])[0, 0, :, :H * H], r0, rtol=1e-5, atol=0.1)
    # the returned log-likelihood: the sum over the maintained image
    ll = model.loglikelihood(tiled, l1, f1)
    np.testing.assert_allclose(N_(mh.last_loglik), N_(ll), rtol=4e-6, atol=5e-3)
    # a second sweep from gathered ancestors, starting from the persisted images
    anc = torch.randint(0, n, (1, 1, n), device=DEV, generator=torch.Generator(DEV).manual_seed(9))
    l2, f2, _ = mh.run(tiled, c, l1, f1, T([[0.7]]), prior=prior, image_model=model,
                       replay=_replay(n, K, 10), ancestors=anc, rate_in=rate[0],
                       rate_out=rate[1])
    np.testing.assert_allclose(N_(rate[1])[0, 0, :, :H * H], fresh(l2, f2), rtol=1e-5, atol=0.1)


def test_smc_run_128_tile_to_temperature_1():
    """SMCsampler over one 128x128 tile (N=1024, K=20) runs to temperature 1
    through the global-memory sweep with persisted rate images: finite log Z,
    ESS = rho*N at every non-final step whose increment is >= 1e-3, and a
    log Z equal to a second run with the images re-rendered every sweep up to
    the Monte Carlo error."""
    from smcdet_amd.sampler import SMCsampler
    img = truth_image()
    runs = []
    for refresh in (8, 1):
        s = SMCsampler(img, H, p_m71_prior(H, S, S, counts_rate=0.0004), p_m71_model(H),
                       p_m71_mh(20), 1024, 0.5, "systematic", M71["flux_detection_threshold"],
                       400, print_every=10 ** 9, seed=12, rate_refresh_every=refresh)
        esses, taus = [], []
        orig = s._temper_reweight

        def tr(with_resample, orig=orig, s=s, esses=esses, taus=taus):
            orig(with_resample)
            esses.append(float(s.ess.flatten()[0]))
            taus.append(float(s.temperature.flatten()[0]))

        s._temper_reweight = tr
        s.run()
        assert float(s.temperature.min()) == 1.0
        assert np.isfinite(float(s.log_normalizing_constant))
        d = np.diff(np.concatenate([[0.0], taus]))[:-1]
        e = np.array(esses[:-1])
        np.testing.assert_allclose(e[d >= 1e-3], 512, rtol=0.01)
        assert s.pruned_counts.shape == (1, 1, 1024)
        runs.append(float(s.log_normalizing_constant))
    assert abs(runs[0] - runs[1]) < 0.02 * abs(runs[1])
