"""Count-stratified SMC on the GPU (manuscript.tex:314-356).

* smcdet_count_posterior against the oracle under replayed uniforms: p(s|x)
  to float rounding, stratum/particle indices and gathered catalogs exact;
* the MH kernel's SMCDET_MH_COMPONENT_BY_COUNT mode never touches the padded
  sources of a stratum (and count 0 never moves);
* statistical parity of whole CS-SMC runs against the reference's own
  fixed-count samplers (tests/golden/stats_cssmc.json: 16 seeds, one
  SMCsampler per count): mean log Z_s within 3 pooled SE and 1%, log Z_0
  equal to the empty-catalog likelihood, mean p(s|x) within 3 SE + 0.02.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import smc_oracle as O
from tests._params import GOLDEN, M71, p_m71_mh, p_m71_model, p_m71_prior

pytestmark = pytest.mark.gpu
DEV = "cuda"


def N_(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("method", ["systematic", "multinomial"])
def test_count_posterior_kernel_vs_oracle(method):
    from smcdet_amd import _hip
    rng = np.random.default_rng(1)
    T, NS, Np, S, n_out = 3, 5, 37, 4, 200
    logZ = rng.normal(-300, 3, (T, NS)).astype(np.float32)
    lcp = O.log_count_prior(O.M71PriorP(0, NS - 1, 0.03, 8, 8, 4, M71["flux_alpha"],
                                        M71["flux_lower"], M71["flux_upper"])).astype(np.float32)
    counts = np.repeat(np.arange(NS, dtype=np.float32), Np)[None].repeat(T, 0).reshape(T, NS, Np)
    locs = rng.random((T, NS, Np, S, 2)).astype(np.float32)
    fluxes = rng.random((T, NS, Np, S)).astype(np.float32)
    us = (rng.random(T) if method == "systematic" else rng.random((T, n_out))).astype(np.float32)
    up = rng.random((T, n_out)).astype(np.float32)
    d = lambda x: torch.as_tensor(x).to(DEV)  # noqa: E731
    probs = torch.empty(T, NS, device=DEV)
    idx = torch.empty(T, n_out, device=DEV, dtype=torch.int64)
    co = torch.empty(T, n_out, device=DEV)
    lo = torch.empty(T, n_out, S, 2, device=DEV)
    fo = torch.empty(T, n_out, S, device=DEV)
    m = _hip.SMCDET_RESAMPLE_SYSTEMATIC if method == "systematic" else \
        _hip.SMCDET_RESAMPLE_MULTINOMIAL
    keep = [d(logZ), d(lcp), d(us), d(up), d(counts), d(locs), d(fluxes)]
    _hip.check(_hip.lib().smcdet_count_posterior(
        *[_hip.ptr(k) for k in keep[:2]], 0, T, NS, Np, S, n_out, m, 0, 0,
        *[_hip.ptr(k) for k in keep[2:]], _hip.ptr(probs), _hip.ptr(idx), _hip.ptr(co),
        _hip.ptr(lo), _hip.ptr(fo), _hip.stream_of(probs)), "count_posterior")
    p_ref = O.count_posterior(logZ, lcp)
    np.testing.assert_allclose(N_(probs), p_ref, rtol=1e-6, atol=1e-12)
    i_ref = O.count_posterior_draw(p_ref, us, up, Np, method)
    np.testing.assert_array_equal(N_(idx), i_ref)
    flat_c = counts.reshape(T, NS * Np)
    np.testing.assert_array_equal(N_(co), np.take_along_axis(flat_c, i_ref, 1))
    np.testing.assert_array_equal(
        N_(lo), np.take_along_axis(locs.reshape(T, NS * Np, S, 2), i_ref[..., None, None], 1))
    np.testing.assert_array_equal(
        N_(fo), np.take_along_axis(fluxes.reshape(T, NS * Np, S), i_ref[..., None], 1))


def test_mh_component_by_count_keeps_padding():
    from smcdet_amd._rng import PhiloxStream
    torch.manual_seed(3)
    H, Np = 8, 256
    model, prior = p_m71_model(H), p_m71_prior(H, 0, 4)
    img = 104.15 + 14 * torch.randn(1, 1, H, H, device=DEV)
    counts, locs, fluxes = prior.sample(num_tiles_per_side=1, stratify_by_count=True,
                                        num_catalogs_per_count=Np, device=DEV)
    mh = p_m71_mh(40)
    mh.component_by_count = True
    mh.rng = PhiloxStream(9)
    l1, f1, _ = mh.run(img, counts, locs, fluxes, torch.tensor([[0.5]], device=DEV),
                       prior=prior, image_model=model)
    c = N_(counts)[0, 0]
    pad = np.arange(4)[None] >= c[:, None]                      # [N, S] padded sources
    moved = (N_(l1)[0, 0] != N_(locs)[0, 0]).any(-1) | (N_(f1)[0, 0] != N_(fluxes)[0, 0])
    assert not moved[pad].any()
    assert not moved[c == 0].any()
    assert moved[~pad].mean() > 0.5
    # the returned log-likelihood is that of the returned state
    ll = model.loglikelihood(img, l1, f1)
    np.testing.assert_allclose(N_(mh.last_loglik), N_(ll), rtol=2e-6, atol=1e-3)


def _se(a, b):
    return np.sqrt(np.var(a, ddof=1) / len(a) + np.var(b, ddof=1) / len(b))


def test_cssmc_statistical_vs_reference():
    from smcdet_amd.cssmc import CountStratifiedSMC
    path = os.path.join(GOLDEN, "stats_cssmc.json")
    with open(path) as f:
        ref = json.load(f)
    cfg = ref["config"]
    image = torch.tensor(ref["image"], dtype=torch.float32, device=DEV)
    H, smax = cfg["tile"], cfg["smax"]
    lz, post, iters = [], [], []
    for seed in range(24):
        torch.manual_seed(500 + seed)
        cs = CountStratifiedSMC(image, H, p_m71_prior(H, 0, smax), p_m71_model(H),
                                p_m71_mh(cfg["K"]), cfg["N"], cfg["rho"], cfg["method"],
                                M71["flux_detection_threshold"], 100, print_every=10 ** 9)
        cs.run()
        lz.append(N_(cs.log_normalizing_constant_per_count)[0, 0])
        post.append(N_(cs.count_posterior)[0, 0])
        iters.append(cs.iter)
        assert cs.counts.shape == (1, 1, cfg["N"])
        # every output catalog comes from the stratum of its count
        k = N_(cs.sample_index)[0, 0] // cfg["N"]
        np.testing.assert_array_equal(N_(cs.counts)[0, 0], k.astype(np.float32))
    lz, post = np.array(lz), np.array(post)
    rl = np.array([r["logZ"] for r in ref["runs"]])
    rp = np.array([r["count_posterior"] for r in ref["runs"]])
    np.testing.assert_allclose(lz[:, 0], cfg["loglik_empty"], rtol=1e-5)
    for s in range(1, smax + 1):
        d = lz[:, s].mean() - rl[:, s].mean()
        assert abs(d) <= 3 * _se(lz[:, s], rl[:, s]) + 1e-3, (s, lz[:, s].mean(), rl[:, s].mean())
        assert abs(d) <= 0.01 * abs(rl[:, s].mean()), (s, lz[:, s].mean(), rl[:, s].mean())
    se = np.sqrt(post.var(0, ddof=1) / len(post) + rp.var(0, ddof=1) / len(rp))
    assert np.all(np.abs(post.mean(0) - rp.mean(0)) <= 3 * se + 0.02), (post.mean(0), rp.mean(0))
