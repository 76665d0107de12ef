#!/usr/bin/env python
"""Golden-vector generator: runs the REFERENCE smcdet (imported from
/root/reference, CPU, float32 default dtype) and records inputs, every random
draw it makes, and its outputs as small .npz fixtures under tests/golden/.

Test infrastructure only.  It runs in the build container (where the
reference is mounted read-only); the GPU box only ever sees the .npz/.json
files it wrote.  Nothing here is imported by the product package.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py fixtures
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py stats   # slow

Recording: torch.rand and torch.distributions.Multinomial.sample are wrapped
so that every draw the reference makes (prior sampling, truncated-normal
proposals, accept uniforms, systematic-resampling offsets, component masks)
is captured in call order.  The reference's own RNG stream is unchanged.
"""
import json
import os
import sys
import time

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)

from smcdet.distributions import TruncatedDiagonalMVN, TruncatedPareto  # noqa: E402
from smcdet.images import ImageModel, M71ImageModel, generate_images  # noqa: E402
from smcdet.kernel import SingleComponentMALA, SingleComponentMH  # noqa: E402
from smcdet.prior import M71Prior, ParetoStarPrior  # noqa: E402
from smcdet.sampler import MHsampler, SMCsampler  # noqa: E402

# M71 parameters (notebooks/smc.ipynb cell 2; full precision per SURVEY §8a)
M71 = dict(
    flux_alpha=0.21411753249015655,
    flux_lower=0.06291294097900389,
    flux_upper=1804.6791992187502,
    flux_detection_threshold=0.25165176391601557,
    counts_rate=0.030264640226960182,
    background=104.1486587524414,
    adu_per_nmgy=241.02658081054688,
    psf_params=[1.107237458229065, 2.0800251960754395, 2.3254318237304688,
                5.240590572357178, 0.7346734404563904, 0.5114791393280029],
    psf_radius=8,
    noise_additive=1.0000007072408224e-10,
    noise_multiplicative=1.936462640762329,
)
# experiments/basic/generate_images.py:26-60
BASIC_PSF_STDEV = 0.93
BASIC_BACKGROUND = 200.0
_psf_max = 1 / (2 * np.pi * BASIC_PSF_STDEV ** 2)
BASIC_FLUX_SCALE = 5 * np.sqrt(BASIC_BACKGROUND) / _psf_max
BASIC_FLUX_ALPHA = (-np.log(1 - 0.99)) / (
    np.log(50 * np.sqrt(BASIC_BACKGROUND) / _psf_max) - np.log(BASIC_FLUX_SCALE))


class Recorder:
    """Wraps torch.rand / torch.rand_like / Multinomial.sample /
    Tensor.multinomial; records draws."""

    def __init__(self):
        self.draws = []  # list of (kind, np.ndarray)

    def __enter__(self):
        rec = self
        self._rand = torch.rand
        self._ms = torch.distributions.Multinomial.sample
        self._tm = torch.Tensor.multinomial
        self._rl = torch.rand_like

        def rand(*a, **k):
            out = rec._rand(*a, **k)
            rec.draws.append(("rand", out.detach().cpu().numpy().copy()))
            return out

        def ms(self_, sample_shape=torch.Size()):
            out = rec._ms(self_, sample_shape)
            rec.draws.append(("mask", out.detach().cpu().numpy().copy()))
            return out

        def tm(self_, *a, **k):
            out = rec._tm(self_, *a, **k)
            rec.draws.append(("multinomial", out.detach().cpu().numpy().copy()))
            return out

        def rl(*a, **k):
            out = rec._rl(*a, **k)
            rec.draws.append(("rand_like", out.detach().cpu().numpy().copy()))
            return out

        torch.rand = rand
        torch.rand_like = rl
        torch.distributions.Multinomial.sample = ms
        torch.Tensor.multinomial = tm
        return self

    def __exit__(self, *exc):
        torch.rand = self._rand
        torch.rand_like = self._rl
        torch.distributions.Multinomial.sample = self._ms
        torch.Tensor.multinomial = self._tm
        return False


def m71_model(H, psf_params=None):
    p = M71
    return M71ImageModel(
        image_height=H, image_width=H, background=p["background"],
        psf_radius=p["psf_radius"], adu_per_nmgy=p["adu_per_nmgy"],
        psf_params=torch.tensor(p["psf_params"] if psf_params is None else psf_params),
        noise_additive=p["noise_additive"],
        noise_multiplicative=p["noise_multiplicative"])


def m71_prior(H, smin, smax, pad=4, counts_rate=None, flux_lower=None):
    p = M71
    return M71Prior(
        min_objects=smin, max_objects=smax,
        counts_rate=p["counts_rate"] if counts_rate is None else counts_rate,
        image_height=H, image_width=H, flux_alpha=p["flux_alpha"],
        flux_lower=p["flux_lower"] if flux_lower is None else flux_lower,
        flux_upper=p["flux_upper"], pad=pad)


def basic_model(H):
    return ImageModel(image_height=H, image_width=H, psf_radius=8,
                      psf_stdev=BASIC_PSF_STDEV, background=BASIC_BACKGROUND)


def basic_prior(H, smin, smax, pad=2):
    return ParetoStarPrior(min_objects=smin, max_objects=smax, image_height=H,
                           image_width=H, flux_scale=BASIC_FLUX_SCALE * 0.9,
                           flux_alpha=BASIC_FLUX_ALPHA, pad=pad)


def m71_truth_image(H, seed, counts_rate=None, max_sources=None):
    """generate_images() with a Poisson-count M71 truth prior (as
    experiments/m71synthetic/generate_images.py:27-67)."""
    torch.manual_seed(seed)
    tp = m71_prior(H, 0, 100, pad=4, counts_rate=counts_rate,
                   flux_lower=M71["flux_detection_threshold"])
    while True:
        res = generate_images(tp, m71_model(H), M71["flux_detection_threshold"], 0, H, 1)
        if max_sources is None or int(res[0][0]) <= max_sources:
            return res


def basic_truth_image(H, seed):
    """experiments/basic/generate_images.py:26-94 (one image)."""
    torch.manual_seed(seed)
    tp = basic_prior(H, 0, 3)
    return generate_images(tp, basic_model(H), BASIC_FLUX_SCALE, 0, H, 1)


def sampler_for(image, tile_dim, prior, model, mh, N, method="systematic",
                max_iters=100):
    return SMCsampler(image=image, tile_dim=tile_dim, Prior=prior, ImageModel=model,
                      MutationKernel=mh, num_catalogs=N, ess_threshold_prop=0.5,
                      resample_method=method,
                      flux_detection_threshold=M71["flux_detection_threshold"],
                      max_smc_iters=max_iters, print_every=10 ** 9)


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def save(name, **arrs):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrs.items()})
    print("wrote", path, sum(np.asarray(v).nbytes for v in arrs.values()), "bytes raw")


# ----------------------------------------------------------------------------
def gen_psf():
    out = {}
    for H in (8, 16, 32):
        pts = [(H / 2 + 0.3, H / 2 + 0.7), (3.0, 5.0), (-3.2, 2.5), (H - 0.01, 0.01),
               (H + 3.9, -3.9), (0.5, 0.5), (-0.25, H - 0.75), (1.999, 2.001)]
        locs = torch.tensor(pts, dtype=torch.float32).reshape(1, 1, 2, 4, 2)
        m = m71_model(H)
        out[f"m71_H{H}_locs"] = np32(locs)
        out[f"m71_H{H}_psf"] = np32(m.psf(locs))
        if H == 16:
            b = basic_model(H)
            out[f"basic_H{H}_psf"] = np32(b.psf(locs))
    m = m71_model(8)
    out["m71_norm_const_f32"] = np.float32(m.psf_normalizing_constant.item())
    r = torch.linspace(0, 12, 97)
    out["m71_r"] = np32(r)
    out["m71_unnorm"] = np32(m._compute_unnormalized_psf(r))
    out["m71_norm"] = np32(m._compute_normalized_psf(r))
    out["basic_norm"] = np32(basic_model(8)._compute_normalized_psf(r))
    save("psf.npz", **out)


def gen_loglik():
    out = {}
    # M71 single tiles, prior catalogs around a synthetic truth image
    for H, S, N, seed in ((8, 10, 64, 1), (32, 10, 32, 2), (16, 3, 48, 3)):
        res = m71_truth_image(H, seed, counts_rate=M71["counts_rate"] if H == 8 else 0.003125)
        img = res[-1][0]
        torch.manual_seed(100 + seed)
        pr = m71_prior(H, S, S)
        counts, locs, fluxes = pr.sample(num_tiles_per_side=1, stratify_by_count=True,
                                         num_catalogs_per_count=N)
        # include a few states near a posterior mode: copy truth into particle 0
        tl, tf = res[1][0], res[2][0]
        k = min(S, tl.shape[0])
        locs[0, 0, 0, :k] = tl[:k]
        fluxes[0, 0, 0, :k] = tf[:k].clamp(min=pr.flux_lower)
        m = m71_model(H)
        tiled = img.unsqueeze(0).unsqueeze(0)
        key = f"m71_H{H}_S{S}"
        out[key + "_image"] = np32(img)
        out[key + "_locs"] = np32(locs)
        out[key + "_fluxes"] = np32(fluxes)
        out[key + "_counts"] = np32(counts)
        out[key + "_loglik"] = np32(m.loglikelihood(tiled, locs, fluxes))
        out[key + "_logprior"] = np32(pr.log_prob(counts, locs, fluxes))
        # float64 reference evaluation of the same states
        torch.set_default_dtype(torch.float64)
        try:
            m64 = m71_model(H)
            ll64 = m64.loglikelihood(tiled.double(), locs.double(), fluxes.double())
            out[key + "_loglik_f64"] = ll64.numpy()
        finally:
            torch.set_default_dtype(torch.float32)
    # multi-tile (2x2 tiles of 8x8 from a 16x16 image): checks unfold/tiling
    res = m71_truth_image(16, 7)
    img = res[-1][0]
    torch.manual_seed(107)
    pr = m71_prior(8, 4, 4)
    counts, locs, fluxes = pr.sample(num_tiles_per_side=2, stratify_by_count=True,
                                     num_catalogs_per_count=16)
    m = m71_model(8)
    tiled = img.unfold(0, 8, 8).unfold(1, 8, 8)
    out["m71_tiles_image"] = np32(img)
    out["m71_tiles_locs"] = np32(locs)
    out["m71_tiles_fluxes"] = np32(fluxes)
    out["m71_tiles_loglik"] = np32(m.loglikelihood(tiled, locs, fluxes))
    # Poisson (basic) model
    res = basic_truth_image(16, 11)
    img = res[-1][0]
    torch.manual_seed(111)
    pr = basic_prior(16, 3, 3)
    counts, locs, fluxes = pr.sample(num_tiles_per_side=1, stratify_by_count=True,
                                     num_catalogs_per_count=64)
    b = basic_model(16)
    tiled = img.unsqueeze(0).unsqueeze(0)
    out["basic_H16_S3_image"] = np32(img)
    out["basic_H16_S3_locs"] = np32(locs)
    out["basic_H16_S3_fluxes"] = np32(fluxes)
    out["basic_H16_S3_counts"] = np32(counts)
    out["basic_H16_S3_loglik"] = np32(b.loglikelihood(tiled, locs, fluxes))
    out["basic_H16_S3_logprior"] = np32(pr.log_prob(counts, locs, fluxes))
    # Poisson model with the rate > 5e4 (normal-approximation) branch exercised
    locs2 = locs.clone()
    fl2 = fluxes.clone()
    fl2[0, 0, :8, 0] = torch.linspace(2e5, 2e6, 8)
    locs2[0, 0, :8, 0] = torch.tensor([7.5, 8.5])
    img2 = img.clone()
    img2[7:10, 7:10] += 60000.0
    out["basic_bright_image"] = np32(img2)
    out["basic_bright_locs"] = np32(locs2)
    out["basic_bright_fluxes"] = np32(fl2)
    out["basic_bright_loglik"] = np32(b.loglikelihood(img2.unsqueeze(0).unsqueeze(0), locs2, fl2))
    save("loglik.npz", **out)


def gen_prior():
    out = {}
    torch.manual_seed(21)
    # counts varying 0..S to exercise the count mask (min < max)
    pr = m71_prior(8, 0, 12, counts_rate=0.01)
    with Recorder() as rec:
        counts, locs, fluxes = pr.sample(num_catalogs=40, num_tiles_per_side=2)
    out["m71_counts"] = np32(counts)
    out["m71_locs"] = np32(locs)
    out["m71_fluxes"] = np32(fluxes)
    out["m71_logprior"] = np32(pr.log_prob(counts, locs, fluxes))
    # stratified sampling draws (initialize() path, prior.py:47-64)
    torch.manual_seed(22)
    pr = m71_prior(8, 3, 5)
    with Recorder() as rec:
        counts, locs, fluxes = pr.sample(num_tiles_per_side=2, stratify_by_count=True,
                                         num_catalogs_per_count=8)
    assert [k for k, _ in rec.draws] == ["rand", "rand"]
    out["m71_strat_uloc"] = rec.draws[0][1]
    out["m71_strat_uflux"] = rec.draws[1][1]
    out["m71_strat_counts"] = np32(counts)
    out["m71_strat_locs"] = np32(locs)
    out["m71_strat_fluxes"] = np32(fluxes)
    out["m71_strat_logprior"] = np32(pr.log_prob(counts, locs, fluxes))
    torch.manual_seed(23)
    pr = basic_prior(16, 3, 3)
    with Recorder() as rec:
        counts, locs, fluxes = pr.sample(num_tiles_per_side=1, stratify_by_count=True,
                                         num_catalogs_per_count=32)
    out["basic_counts"] = np32(counts)
    out["basic_locs"] = np32(locs)
    out["basic_fluxes"] = np32(fluxes)
    out["basic_logprior"] = np32(pr.log_prob(counts, locs, fluxes))
    save("prior.npz", **out)


def gen_distributions():
    out = {}
    torch.manual_seed(31)
    # truncated normal: loc-like (sigma 0.1, box [-4, 36]) and flux-like
    mu_l = torch.cat([torch.rand(200, 2) * 40 - 4, torch.tensor([[-4.0, 36.0], [-3.95, 35.97]])])
    mu_f = torch.cat([torch.rand(100) * 3, torch.rand(100) * 1800,
                      torch.tensor([0.06291294097900389, 1804.6791992187502])])
    for name, mu, sig, lb, ub in (
            ("loc", mu_l, torch.tensor(0.1), -4 * torch.ones(2), torch.tensor([36.0, 36.0])),
            ("flux", mu_f, 2.5 * torch.ones(1), M71["flux_lower"] * torch.ones(1),
             M71["flux_upper"] * torch.ones(1))):
        d = TruncatedDiagonalMVN(mu, sig, lb, ub)
        with Recorder() as rec:
            x = d.sample()
        out[name + "_mu"] = np32(mu)
        out[name + "_u"] = rec.draws[0][1]
        out[name + "_x"] = np32(x)
        out[name + "_logprob_x"] = np32(d.log_prob(x))
        out[name + "_logZ"] = np32(d.log_prob_in_box)
    tp = TruncatedPareto(M71["flux_alpha"], M71["flux_lower"], M71["flux_upper"])
    with Recorder() as rec:
        f = tp.sample([500])
    out["tpareto_u"] = rec.draws[0][1]
    out["tpareto_x"] = np32(f)
    out["tpareto_logprob"] = np32(tp.log_prob(f))
    save("distributions.npz", **out)


def run_mh_recorded(image, tile_dim, prior, model, mh, N, tau, seed):
    """Runs SingleComponentMH.run once with recorded draws and proposals."""
    torch.manual_seed(seed)
    s = sampler_for(image, tile_dim, prior, model, mh, N)
    s.initialize()
    nt = s.num_tiles_per_side
    temperature = torch.full((nt, nt), float(tau))
    proposals = []
    orig = s.log_target

    def log_target(data, counts, locs, fluxes, temperature):
        v = orig(data, counts, locs, fluxes, temperature)
        proposals.append((np32(locs), np32(fluxes), np32(v)))
        return v

    locs0, fluxes0 = s.locs.clone(), s.fluxes.clone()
    with Recorder() as rec:
        locs1, fluxes1, acc = mh.run(s.tiled_image, s.counts, s.locs, s.fluxes,
                                     temperature, log_target)
    K = mh.num_iters
    kinds = [k for k, _ in rec.draws]
    assert kinds == ["mask", "rand", "rand", "rand"] * K, kinds[:8]
    masks = np.stack([rec.draws[4 * i][1] for i in range(K)])
    uloc = np.stack([rec.draws[4 * i + 1][1] for i in range(K)])
    uflux = np.stack([rec.draws[4 * i + 2][1] for i in range(K)])
    uacc = np.stack([rec.draws[4 * i + 3][1] for i in range(K)])
    comp = masks.argmax(-1).astype(np.int32)  # [K,nt,nt,N]
    j = comp[..., None]
    uloc_sel = np.take_along_axis(uloc, j[..., None].repeat(2, -1)[..., None, :].reshape(
        *j.shape[:-1], 1, 2), axis=-2)[..., 0, :]
    uflux_sel = np.take_along_axis(uflux, j, axis=-1)[..., 0]
    # log_target call order: iter0 numerator, iter0 denominator, then one numerator per iter
    prop_locs = np.stack([proposals[0][0]] + [proposals[i][0] for i in range(2, K + 1)])
    prop_fluxes = np.stack([proposals[0][1]] + [proposals[i][1] for i in range(2, K + 1)])
    prop_lt = np.stack([proposals[0][2]] + [proposals[i][2] for i in range(2, K + 1)])
    return dict(image=np32(s.image), counts=np32(s.counts), locs0=np32(locs0),
                fluxes0=np32(fluxes0), tau=np.float32(tau), comp=comp,
                uloc=uloc_sel.astype(np.float32), uflux=uflux_sel.astype(np.float32),
                uacc=uacc.astype(np.float32), locs1=np32(locs1), fluxes1=np32(fluxes1),
                acc=np32(acc), prop_locs=prop_locs, prop_fluxes=prop_fluxes,
                prop_logtarget=prop_lt, init_logtarget=proposals[1][2],
                locs_min=np32(mh.locs_min), locs_max=np32(mh.locs_max))


def gen_mh():
    # M71 8x8, S=4, N=32, K=20
    res = m71_truth_image(8, 41)
    mh = SingleComponentMH(20, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    d = run_mh_recorded(res[-1][0], 8, m71_prior(8, 4, 4), m71_model(8), mh, 32, 0.3, 141)
    save("mh_m71_8x8.npz", **d)
    # M71 32x32 (C2 geometry), S=10, N=8, K=10
    res = m71_truth_image(32, 42, counts_rate=0.003125, max_sources=10)
    mh = SingleComponentMH(10, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    d = run_mh_recorded(res[-1][0], 32, m71_prior(32, 10, 10), m71_model(32), mh, 8, 0.05, 142)
    save("mh_m71_32x32.npz", **d)
    # 2x2 tiles of 8x8 at tau=1 (multi-tile indexing)
    res = m71_truth_image(16, 43)
    mh = SingleComponentMH(10, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    d = run_mh_recorded(res[-1][0], 8, m71_prior(8, 3, 3), m71_model(8), mh, 8, 1.0, 143)
    save("mh_m71_tiles.npz", **d)
    # basic Poisson model (config 1 family) 16x16, S=3, N=32, K=20
    res = basic_truth_image(16, 44)
    pr = basic_prior(16, 3, 3)
    mh = SingleComponentMH(20, 0.1, 100, pr.flux_scale, 1e6)
    d = run_mh_recorded(res[-1][0], 16, pr, basic_model(16), mh, 32, 0.5, 144)
    save("mh_basic_16x16.npz", **d)


def run_mh_edge_recorded(image, tile_dim, prior, model, mh, N, tau, seed, plan, u_hit=0.9999999):
    """SingleComponentMH.run with sources placed just below the prior box's
    upper edge (H + pad - 0.01) and draws injected so that chosen proposals
    land exactly on it (distributions.py:44-48: p -> 1 - 1e-6, x rounds to
    ub): Uniform.log_prob(high) = -inf (prior.py:73), the proposal is
    rejected and the cached target becomes -inf * 0 = NaN (kernel.py:125), so
    the particle rejects the rest of the sweep.  plan = [(particle, source,
    coords, iteration)]: at `iteration` the particle's component is forced to
    `source` and its location uniforms for `coords` (0 = h, 1 = w) to u_hit.
    Records every draw actually used, every accept decision (prob <= alpha,
    kernel.py:116) and the proposals."""
    torch.manual_seed(seed)
    s = sampler_for(image, tile_dim, prior, model, mh, N)
    s.initialize()
    hi = prior.loc_prior.high
    for n, j, coords, _ in plan:
        for c in coords:
            s.locs[..., n, j, c] = float(hi[c]) - 0.01
    nt = s.num_tiles_per_side
    temperature = torch.full((nt, nt), float(tau))
    proposals, accepts = [], []
    orig = s.log_target

    def log_target(data, counts, locs, fluxes, temperature):
        v = orig(data, counts, locs, fluxes, temperature)
        proposals.append((np32(locs), np32(fluxes), np32(v)))
        return v

    state = {"k": -1, "prob": None}
    ms0, rand0 = torch.distributions.Multinomial.sample, torch.rand
    usample0, le0 = torch.distributions.Uniform.sample, torch.Tensor.__le__

    def ms(self_, sample_shape=torch.Size()):
        out = ms0(self_, sample_shape)
        state["k"] += 1
        state["nrand"] = 0
        S_ = out.shape[-1]
        for n, j, _, k in plan:
            if k == state["k"]:
                out[..., n, :] = 0
                out[..., n, j] = 1
            elif state["k"] < k and bool((out[..., n, j] == 1).all()):
                # keep the edge source where it was placed until its hit:
                # farther from the edge, whether a draw rounds onto it
                # depends on float32 rounding noise (a near-tie)
                out[..., n, j] = 0
                out[..., n, (j + 1) % S_] = 1
        return out

    def rand(*a, **kw):
        out = rand0(*a, **kw)
        if state["k"] >= 0:
            state["nrand"] += 1
            if state["nrand"] == 1:  # the location uniforms [nt,nt,N,S,2]
                for n, j, coords, k in plan:
                    if k == state["k"]:
                        for c in coords:
                            out[..., n, j, c] = u_hit
        return out

    def usample(self_, *a, **kw):
        out = usample0(self_, *a, **kw)
        state["prob"] = out
        return out

    def le(self_, other):
        out = le0(self_, other)
        if self_ is state["prob"]:
            accepts.append(out.numpy().copy())
        return out

    locs0, fluxes0 = s.locs.clone(), s.fluxes.clone()
    torch.distributions.Multinomial.sample = ms
    torch.rand = rand
    try:
        with Recorder() as rec:
            torch.distributions.Uniform.sample = usample
            torch.Tensor.__le__ = le
            try:
                locs1, fluxes1, acc = mh.run(s.tiled_image, s.counts, s.locs, s.fluxes,
                                             temperature, log_target)
            finally:
                torch.distributions.Uniform.sample = usample0
                torch.Tensor.__le__ = le0
    finally:
        torch.distributions.Multinomial.sample = ms0
        torch.rand = rand0
    K = mh.num_iters
    kinds = [k for k, _ in rec.draws]
    assert kinds == ["mask", "rand", "rand", "rand"] * K, kinds[:8]
    masks = np.stack([rec.draws[4 * i][1] for i in range(K)])
    uloc = np.stack([rec.draws[4 * i + 1][1] for i in range(K)])
    uflux = np.stack([rec.draws[4 * i + 2][1] for i in range(K)])
    uacc = np.stack([rec.draws[4 * i + 3][1] for i in range(K)])
    comp = masks.argmax(-1).astype(np.int32)
    j = comp[..., None]
    uloc_sel = np.take_along_axis(uloc, j[..., None].repeat(2, -1), axis=-2)[..., 0, :]
    uflux_sel = np.take_along_axis(uflux, j, axis=-1)[..., 0]
    prop_locs = np.stack([proposals[0][0]] + [proposals[i][0] for i in range(2, K + 1)])
    accept = np.stack(accepts)
    assert accept.shape == comp.shape, accept.shape
    # the injected proposals did land on the edge
    edge = np.zeros(comp.shape, bool)
    hi32 = np.float32(hi.numpy())
    for n, jj, coords, k in plan:
        pl = prop_locs[k, :, :, n, jj]
        edge[k, :, :, n] = np.any(pl[..., list(coords)] == hi32[list(coords)], -1)
    assert edge.sum() == len(plan), (edge.sum(), len(plan))
    return dict(image=np32(s.image), counts=np32(s.counts), locs0=np32(locs0),
                fluxes0=np32(fluxes0), tau=np.float32(tau), comp=comp,
                uloc=uloc_sel.astype(np.float32), uflux=uflux_sel.astype(np.float32),
                uacc=uacc.astype(np.float32), locs1=np32(locs1), fluxes1=np32(fluxes1),
                acc=np32(acc), accept=accept, edge_hit=edge, prop_locs=prop_locs,
                init_logtarget=proposals[1][2],
                locs_min=np32(mh.locs_min), locs_max=np32(mh.locs_max))


def gen_mh_edge():
    """Upper-edge proposals: M71 8x8 (S=4, N=32, K=30) and
    the C2 geometry 32x32 (S=10, N=16, K=24); h, w and both coordinates on the
    edge, hits early, mid-sweep and at the last iteration, and control
    particles without hits."""
    res = m71_truth_image(8, 45)
    plan = [(0, 0, (0,), 0), (1, 1, (0,), 3), (2, 2, (1,), 5), (3, 3, (1,), 11),
            (4, 0, (0, 1), 7), (5, 1, (0, 1), 29), (6, 2, (0,), 17), (7, 3, (1,), 22),
            (8, 0, (1,), 1), (9, 2, (0,), 28)]
    mh = SingleComponentMH(30, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    d = run_mh_edge_recorded(res[-1][0], 8, m71_prior(8, 4, 4), m71_model(8), mh, 32, 0.5,
                             145, plan)
    save("mh_m71_edge_8x8.npz", **d)
    res = m71_truth_image(32, 46, counts_rate=0.003125, max_sources=10)
    plan = [(0, 0, (0,), 0), (1, 4, (1,), 4), (2, 9, (0, 1), 9), (3, 5, (0,), 15),
            (4, 7, (1,), 23), (5, 2, (0,), 12)]
    # At 32x32 the reference's float32 log targets (1,024-pixel sums of terms
    # ~10) carry ~1e-2 nats of rounding, which decides near-tie MH decisions;
    # the kernels are exact to ~1e-6.  Take the first seed whose every decision
    # the float64 oracle reproduces with a margin >= 5e-3 nats.
    for seed in range(146, 200):
        mh = SingleComponentMH(24, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
        d = run_mh_edge_recorded(res[-1][0], 32, m71_prior(32, 10, 10), m71_model(32), mh, 16,
                                 0.2, seed, plan)
        if _decisions_pinned(d, "mh_m71_edge_32x32", 5e-3):
            break
    save("mh_m71_edge_32x32.npz", **d)


def _decisions_pinned(d, name, min_margin):
    """True if the float64 oracle (oracle/smc_oracle.py) reproduces every
    recorded decision of fixture d with |log U - log alpha| >= min_margin."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import smc_oracle as O
    from tests._params import mh_fixture_setup, tiles_of
    td, model, prior, mh = mh_fixture_setup(name)
    t = tiles_of(d["image"], td)
    tau = np.full(t.shape[:2], float(d["tau"]))
    _, _, _, loga, acc = O.mh_sweep(t, d["counts"], d["locs0"], d["fluxes0"], tau, prior, model,
                                    mh, d["comp"], d["uloc"], d["uflux"], d["uacc"], trace=True)
    with np.errstate(all="ignore"):
        m = np.abs(np.log(d["uacc"].astype(np.float64)) - np.minimum(loga, 0))
    m = np.where(np.isfinite(m), m, np.inf)
    ok = bool(np.array_equal(acc, d["accept"]) and m.min() >= min_margin)
    print(name, "min margin %.2e" % m.min(), "decisions equal", np.array_equal(acc, d["accept"]))
    return ok


def run_mala_recorded(image, tile_dim, prior, model, mala, N, tau, seed):
    """Runs SingleComponentMALA.run (smcdet/kernel.py:133-275) once with
    recorded draws, gradients (torch.autograd.grad outputs) and proposals."""
    torch.manual_seed(seed)
    s = sampler_for(image, tile_dim, prior, model, mala, N)
    s.initialize()
    nt = s.num_tiles_per_side
    temperature = torch.full((nt, nt), float(tau))
    targets = []
    orig = s.log_target

    def log_target(data, counts, locs, fluxes, temperature):
        v = orig(data, counts, locs, fluxes, temperature)
        targets.append((np32(locs), np32(fluxes), np32(v)))
        return v

    grads = []
    orig_grad = torch.autograd.grad

    def grad(*a, **k):
        out = orig_grad(*a, **k)
        grads.append((np32(out[0]), np32(out[1])))
        return out

    locs0, fluxes0 = s.locs.clone(), s.fluxes.clone()
    torch.autograd.grad = grad
    try:
        with Recorder() as rec:
            locs1, fluxes1, acc = mala.run(s.tiled_image, s.counts, s.locs.clone(),
                                           s.fluxes.clone(), temperature, log_target)
    finally:
        torch.autograd.grad = orig_grad
    K = mala.num_iters
    kinds = [k for k, _ in rec.draws]
    assert kinds == ["mask", "rand", "rand", "rand_like"] * K, kinds[:8]
    masks = np.stack([rec.draws[4 * i][1] for i in range(K)])
    uloc = np.stack([rec.draws[4 * i + 1][1] for i in range(K)])
    uflux = np.stack([rec.draws[4 * i + 2][1] for i in range(K)])
    uacc = np.stack([rec.draws[4 * i + 3][1] for i in range(K)])
    comp = masks.argmax(-1).astype(np.int32)  # [K,nt,nt,N]
    j = comp[..., None]
    def sel2(a, jj):
        return np.take_along_axis(a, jj[..., None].repeat(2, -1), axis=-2)[..., 0, :]

    def sel1(a, jj):
        return np.take_along_axis(a, jj, axis=-1)[..., 0]

    def triple(lc, fl, i):
        return np.concatenate([sel2(lc, j[i]), sel1(fl, j[i])[..., None]], -1)

    # two log_target / grad calls per iteration: current state, proposal
    g_cur = np.stack([triple(*grads[2 * i], i) for i in range(K)])
    g_prop = np.stack([triple(*grads[2 * i + 1], i) for i in range(K)])
    prop = np.stack([triple(targets[2 * i + 1][0], targets[2 * i + 1][1], i) for i in range(K)])
    lt_cur = np.stack([targets[2 * i][2] for i in range(K)])
    lt_prop = np.stack([targets[2 * i + 1][2] for i in range(K)])
    return dict(image=np32(s.image), counts=np32(s.counts), locs0=np32(locs0),
                fluxes0=np32(fluxes0), tau=np.float32(tau), comp=comp,
                uloc=sel2(uloc, j).astype(np.float32), uflux=sel1(uflux, j).astype(np.float32),
                uacc=uacc.astype(np.float32), locs1=np32(locs1), fluxes1=np32(fluxes1),
                acc=np32(acc), grad_cur=g_cur, grad_prop=g_prop, proposal=prop,
                logtarget_cur=lt_cur, logtarget_prop=lt_prop,
                locs_min=np32(mala.locs_min), locs_max=np32(mala.locs_max))


def gen_mala():
    # M71 8x8, S=4, N=32, K=20 (the MH fixture's geometry)
    res = m71_truth_image(8, 41)
    mala = SingleComponentMALA(20, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    d = run_mala_recorded(res[-1][0], 8, m71_prior(8, 4, 4), m71_model(8), mala, 32, 0.3, 151)
    save("mala_m71_8x8.npz", **d)
    # same image at tau = 1 (large gradients: proposal means leave the box)
    mala = SingleComponentMALA(20, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    d = run_mala_recorded(res[-1][0], 8, m71_prior(8, 4, 4), m71_model(8), mala, 32, 1.0, 152)
    save("mala_m71_8x8_tau1.npz", **d)
    # M71 32x32 (C2 geometry), S=10, N=8, K=10
    res = m71_truth_image(32, 42, counts_rate=0.003125, max_sources=10)
    mala = SingleComponentMALA(10, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    d = run_mala_recorded(res[-1][0], 32, m71_prior(32, 10, 10), m71_model(32), mala, 8, 0.05,
                          153)
    save("mala_m71_32x32.npz", **d)
    # 2x2 tiles of 8x8 (multi-tile indexing)
    res = m71_truth_image(16, 43)
    mala = SingleComponentMALA(10, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    d = run_mala_recorded(res[-1][0], 8, m71_prior(8, 3, 3), m71_model(8), mala, 8, 0.5, 154)
    save("mala_m71_tiles.npz", **d)
    # basic Poisson model 16x16, S=3, N=32, K=20
    res = basic_truth_image(16, 44)
    pr = basic_prior(16, 3, 3)
    mala = SingleComponentMALA(20, 0.1, 100, pr.flux_scale, 1e6)
    d = run_mala_recorded(res[-1][0], 16, pr, basic_model(16), mala, 32, 0.5, 155)
    save("mala_basic_16x16.npz", **d)


def run_mcmc_recorded(image, tile_dim, prior, model, total, burnin, keep, seed, edge_plan=None,
                      u_hit=0.9999999):
    """MHsampler (smcdet/sampler.py:301-493) with recorded draws: the initial
    prior draw, then per iteration the component mask, the location and flux
    uniforms of the truncated normals and the accept uniform.  edge_plan =
    [(tile_h, tile_w, source, coords, iteration)]: that source starts 0.01
    below the prior box's upper edge in `coords` and is kept still until
    `iteration`, where it is chosen and its location uniforms are u_hit, so
    the proposal lands exactly on the edge (log prior -inf: rejected, and the
    chain's cached target becomes NaN, sampler.py:522-526)."""
    import contextlib
    import io
    torch.manual_seed(seed)
    ms0, rand0 = torch.distributions.Multinomial.sample, torch.rand
    state = {"k": -1, "nrand": 0, "on": False}

    def ms(self_, sample_shape=torch.Size()):
        out = ms0(self_, sample_shape)
        if state["on"]:
            state["k"] += 1
            state["nrand"] = 0
            S_ = out.shape[-1]
            for th, tw, j, _, k in edge_plan or ():
                if state["k"] == k:
                    out[th, tw, 0, :] = 0
                    out[th, tw, 0, j] = 1
                elif state["k"] < k and bool(out[th, tw, 0, j] == 1):
                    out[th, tw, 0, j] = 0
                    out[th, tw, 0, (j + 1) % S_] = 1
        return out

    def rand(*a, **kw):
        out = rand0(*a, **kw)
        if state["on"]:
            state["nrand"] += 1
            if state["nrand"] == 1:  # the location uniforms [nt,nt,1,S,2]
                for th, tw, j, coords, k in edge_plan or ():
                    if state["k"] == k:
                        for c in coords:
                            out[th, tw, 0, j, c] = u_hit
        return out

    torch.distributions.Multinomial.sample = ms
    torch.rand = rand
    try:
        with Recorder() as rec:
            s = MHsampler(image=image, tile_dim=tile_dim, Prior=prior, ImageModel=model,
                          locs_stdev=0.1, fluxes_stdev=2.5,
                          flux_detection_threshold=M71["flux_detection_threshold"],
                          num_samples_total=total, num_samples_burnin=burnin,
                          keep_every_k=keep, print_every=10 ** 9)
            hi = prior.loc_prior.high
            for th, tw, j, coords, _ in edge_plan or ():
                for c in coords:
                    s.locs[th, tw, 0, j, c] = float(hi[c]) - 0.01
            init_locs, init_fluxes = np32(s.locs[..., 0, :, :]), np32(s.fluxes[..., 0, :])
            n_init = len(rec.draws)
            state["on"] = True
            with contextlib.redirect_stdout(io.StringIO()):
                s.run()
    finally:
        torch.distributions.Multinomial.sample = ms0
        torch.rand = rand0
    draws = rec.draws[n_init:]
    K = total - 1
    kinds = [k for k, _ in draws]
    assert kinds == ["mask", "rand", "rand", "rand"] * K, kinds[:8]
    masks = np.stack([draws[4 * i][1] for i in range(K)])[..., 0, :]     # [K,nt,nt,S]
    uloc = np.stack([draws[4 * i + 1][1] for i in range(K)])[..., 0, :, :]
    uflux = np.stack([draws[4 * i + 2][1] for i in range(K)])[..., 0, :]
    uacc = np.stack([draws[4 * i + 3][1] for i in range(K)])             # [K,nt,nt]
    comp = masks.argmax(-1).astype(np.int32)
    j = comp[..., None]
    uloc_sel = np.take_along_axis(uloc, j[..., None].repeat(2, -1), axis=-2)[..., 0, :]
    uflux_sel = np.take_along_axis(uflux, j, axis=-1)[..., 0]
    return dict(image=np32(s.image), init_locs=init_locs, init_fluxes=init_fluxes,
                comp=comp, uloc=uloc_sel.astype(np.float32),
                uflux=uflux_sel.astype(np.float32), uacc=uacc.astype(np.float32),
                total=np.int32(total), burnin=np.int32(burnin), keep=np.int32(keep),
                counts=np32(s.counts), locs=np32(s.locs), fluxes=np32(s.fluxes),
                accept=s.accept.numpy().astype(np.int32),
                pruned_counts=s.pruned_counts.numpy().astype(np.int64),
                pruned_locs=np32(s.pruned_locs), pruned_fluxes=np32(s.pruned_fluxes))


def gen_mcmc_edge():
    """MHsampler chains whose proposal lands on the prior box's upper edge
    (2x2 tiles of 8x8, S=3, 240 samples, burn-in 40, every 2nd kept): tile
    (0,0) at iteration 30 (h), tile (1,1) at iteration 120 (h and w); the other
    two tiles run on.  The reference keeps those chains frozen for the rest of
    the run (every later accept flag 0, every kept sample the same)."""
    res = m71_truth_image(16, 63)
    plan = [(0, 0, 1, (0,), 30), (1, 1, 2, (0, 1), 120)]
    d = run_mcmc_recorded(res[-1][0], 8, m71_prior(8, 3, 3), m71_model(8), 240, 40, 2, 163,
                          edge_plan=plan)
    acc = d["accept"]
    assert acc[0, 0, 30:].sum() == 0 and acc[1, 1, 120:].sum() == 0, "no freeze recorded"
    assert acc[0, 1, 30:].sum() > 0 and acc[1, 0, 120:].sum() > 0
    d["edge_plan"] = np.array([[th, tw, j, k] for th, tw, j, _, k in plan], np.int32)
    save("mcmc_m71_edge_tiles.npz", **d)


def gen_mcmc():
    # one 8x8 M71 tile, S=4: 300 samples, burn-in 100, every 2nd kept
    res = m71_truth_image(8, 61)
    d = run_mcmc_recorded(res[-1][0], 8, m71_prior(8, 4, 4), m71_model(8), 300, 100, 2, 161)
    save("mcmc_m71_8x8.npz", **d)
    # 16x16 image as 2x2 tiles of 8x8, S=3: 200 samples, burn-in 50, every 3rd
    res = m71_truth_image(16, 62)
    d = run_mcmc_recorded(res[-1][0], 8, m71_prior(8, 3, 3), m71_model(8), 200, 50, 3, 162)
    save("mcmc_m71_tiles.npz", **d)


def gen_smc_steps():
    out = {}
    # temper: loglik vectors from prior states of a 32x32 tile, several tau
    res = m71_truth_image(32, 51, counts_rate=0.003125, max_sources=10)
    img = res[-1][0]
    mh = SingleComponentMH(1, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    torch.manual_seed(151)
    s = sampler_for(img, 16, m71_prior(16, 5, 5), m71_model(16), mh, 512)
    s.initialize()
    lls = s.loglik.clone()  # [2,2,512]
    taus = torch.tensor([[0.0, 0.3], [0.999, 0.9999]])
    s.temperature = taus.clone()
    s.temper()
    out["temper_loglik"] = np32(lls)
    out["temper_tau_in"] = np32(taus)
    out["temper_tau_out"] = np32(s.temperature)
    out["temper_delta"] = (s.temperature.double() - taus.double()).numpy()
    out["temper_rho_N"] = np.float64(s.ess_threshold)
    # update_weights
    s.log_normalizing_constant = torch.tensor([[-3.0, 0.0], [10.0, -1000.0]])
    lz0 = s.log_normalizing_constant.clone()
    s.update_weights()
    out["weights_logZ_in"] = np32(lz0)
    out["weights_W"] = np32(s.weights)
    out["weights_ess"] = np32(s.ess)
    out["weights_logZ"] = np32(s.log_normalizing_constant)
    # systematic resampling with recorded offset
    torch.manual_seed(152)
    s.resample_method = "systematic"
    W = s.weights.clone()
    with Recorder() as rec:
        s_counts0 = s.counts.clone()
        s.resample()
    U = rec.draws[0][1]
    seq = torch.arange(512)
    u = (seq + torch.tensor(U).unsqueeze(-1)) / 512
    bins = W.cumsum(-1)
    idx = torch.stack([torch.stack([torch.bucketize(u[h, w], bins[h, w]) for w in range(2)])
                       for h in range(2)]).clamp(0, 511)
    out["resample_W"] = np32(W)
    out["resample_U"] = U
    out["resample_idx"] = idx.numpy().astype(np.int64)
    out["resample_counts_in"] = np32(s_counts0)
    # systematic on handcrafted weights (zeros, a single spike, ties)
    Wh = torch.zeros(3, 1, 64)
    Wh[0, 0, 5] = 1.0
    Wh[1, 0] = 1.0 / 64
    Wh[2, 0, ::8] = 0.125
    Uh = torch.tensor([[0.0], [0.5], [0.999999]])
    uh = (torch.arange(64) + Uh.unsqueeze(-1)) / 64
    bh = Wh.cumsum(-1)
    idxh = torch.stack([torch.bucketize(uh[i, 0], bh[i, 0]) for i in range(3)]).clamp(0, 63)
    out["resample_hand_W"] = np32(Wh)
    out["resample_hand_U"] = np32(Uh)
    out["resample_hand_idx"] = idxh.numpy().astype(np.int64)[:, None, :]
    # prune
    torch.manual_seed(153)
    locs = torch.rand(2, 2, 64, 6, 2) * 24 - 4
    locs[0, 0, 0, 0] = torch.tensor([0.0, 3.0])
    locs[0, 0, 0, 1] = torch.tensor([16.0, 3.0])
    fl = torch.rand(2, 2, 64, 6) * 0.6
    pc, pl, pf = s.prune(locs, fl)
    out["prune_locs"] = np32(locs)
    out["prune_fluxes"] = np32(fl)
    out["prune_counts"] = pc.numpy().astype(np.int64)
    out["prune_out_locs"] = np32(pl)
    out["prune_out_fluxes"] = np32(pf)
    out["prune_tile_dim"] = np.int64(16)
    out["prune_threshold"] = np.float64(M71["flux_detection_threshold"])
    save("smc_steps.npz", **out)


def _bucketize_systematic(W, U):
    """The reference's systematic indices (sampler.py:136-150) for one tile."""
    N = W.shape[-1]
    u = (torch.arange(N) + torch.as_tensor(U).reshape(())) / N
    return torch.bucketize(u, W.cumsum(-1)).clamp(0, N - 1)


def gen_smc_steps_4096(N=4096, K=3, n_steps=10, seed=171):
    """The tile pass at the headline particle count (VERDICT r2 next #1a):
    the reference's temper (brentq, sampler.py:99-125), update_weights
    (:181-196) and systematic resampling (:127-169) on the log-likelihood
    vectors of a real run -- one 32x32 M71 tile (c2_moderate image), S=10,
    N=4096, a short MH sweep (K=3) between steps -- recorded at every SMC
    iteration: temperature in/out, weights, ESS, log Z in/out, the offset U
    and the indices.  Step 1 starts at temperature 0 (an increment of ~1e-6,
    at brentq's xtol); extra cases re-temper the last step's log-likelihoods
    from temperatures 0.999 / 0.9999 / 0.99999 (increment 1 - tau)."""
    img = c2_moderate_truth_image()
    prior, model = m71_prior(32, 10, 10, counts_rate=0.003125), m71_model(32)
    mh = SingleComponentMH(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    torch.manual_seed(seed)
    s = sampler_for(img, 32, prior, model, mh, N)
    s.initialize()
    rows = []

    def tile_pass(resample):
        tau_in, lz_in = s.temperature.clone(), s.log_normalizing_constant.clone()
        s.temper()
        s.update_weights()
        row = dict(loglik=np32(s.loglik)[0, 0], tau_in=np32(tau_in)[0, 0],
                   tau_out=np32(s.temperature)[0, 0], logZ_in=np32(lz_in)[0, 0],
                   W=np32(s.weights)[0, 0], ess=np32(s.ess)[0, 0],
                   logZ=np32(s.log_normalizing_constant)[0, 0],
                   lw=np32(s.weights_log_unnorm)[0, 0])
        if resample:
            W = s.weights.clone()
            with Recorder() as rec:
                s.resample()
            U = rec.draws[0][1]
            row["U"] = U.reshape(()).astype(np.float32)
            row["idx"] = _bucketize_systematic(W[0, 0], U).numpy().astype(np.int64)
        rows.append(row)

    tile_pass(True)
    for _ in range(n_steps - 1):
        s.mutate()
        tile_pass(True)
        if bool((s.temperature >= 1).all()):
            break
    # temperatures close to 1: increment 1 - tau (the f(1 - tau) >= 0 branch)
    # or a tiny brentq root; same log-likelihoods as the last step
    for tau in (0.999, 0.9999, 0.99999):
        s.temperature = torch.full((1, 1), tau)
        s.log_normalizing_constant = torch.full((1, 1), -4400.0)
        tile_pass(False)
    # ... and brentq roots close to 1 - tau: the same log-likelihoods spread
    # 200x / 5000x wider (an ESS below rho N already at increment 1 - tau)
    ll0 = s.loglik.clone()
    orig_ll = s.ImageModel.loglikelihood
    for tau, scale in ((0.999, 200.0), (0.99, 5000.0)):
        s.ImageModel.loglikelihood = lambda *a, scale=scale: ll0 * scale
        s.temperature = torch.full((1, 1), tau)
        s.log_normalizing_constant = torch.full((1, 1), -4400.0)
        tile_pass(True)
    s.ImageModel.loglikelihood = orig_ll
    out = {}
    for i, r in enumerate(rows):
        for k, v in r.items():
            out[f"c{i:02d}_{k}"] = v
    out["n_cases"] = np.int64(len(rows))
    out["rho_N"] = np.float64(s.ess_threshold)
    save("smc_steps_4096.npz", **out)
    print("cases", len(rows), "taus", [float(r["tau_out"]) for r in rows])


def gen_mh_teacher(N=1024, K=100, steps=(4, 5, 6), seed=181, min_margin=1e-4):
    """Teacher-forced MH replay at the headline geometry (VERDICT r2 next
    #1b): one 32x32 M71 tile (c2_moderate image), S=10, N=1024, K=100, the
    reference's own SMC run.  For each SMC iteration in `steps` (consecutive)
    it records the state the reference mutates (after its resampling), the
    temperature, every draw of SingleComponentMH.run (component, the chosen
    source's location / flux uniforms, the accept uniform), every accept
    decision (prob <= alpha, kernel.py:115-116) and the returned state; from
    the second recorded step on also the resampling indices that link it to
    the previous step's returned state (sampler.py:127-169).  pin[n] = the
    first iteration whose decision the float64 oracle makes with a margin
    |log U - min(log alpha, 0)| < min_margin along the reference's
    trajectory (K when none): decisions before it are pinned exactly."""
    import contextlib
    import io
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import smc_oracle as O
    from tests._params import o_m71_model, o_m71_prior
    img = c2_moderate_truth_image()
    prior, model = m71_prior(32, 10, 10, counts_rate=0.003125), m71_model(32)
    mh = SingleComponentMH(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    torch.manual_seed(seed)
    s = sampler_for(img, 32, prior, model, mh, N, max_iters=10 ** 6)
    with contextlib.redirect_stdout(io.StringIO()):
        s.initialize()
        s.temper()
        s.update_weights()
    out = dict(image=np32(s.image), K=np.int64(K), N=np.int64(N), steps=np.array(steps),
               locs_min=np32(mh.locs_min), locs_max=np32(mh.locs_max),
               min_margin=np.float64(min_margin))
    o_prior, o_model = o_m71_prior(32, 10, 10, counts_rate=0.003125), o_m71_model(32)
    o_mh = O.MHParams(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    for it in range(1, steps[-1] + 1):
        W = s.weights.clone()
        locs_prev, fluxes_prev = s.locs.clone(), s.fluxes.clone()
        with Recorder() as rec:
            s.resample()
        idx = _bucketize_systematic(W[0, 0], rec.draws[0][1]).numpy().astype(np.int64)
        if it not in steps:
            s.mutate()
            s.temper()
            s.update_weights()
            print("iteration", it, "tau", float(s.temperature), flush=True)
            continue
        key = f"s{steps.index(it)}_"
        # the recorded resampling reproduces the reference's gather exactly
        assert torch.equal(s.locs[0, 0], locs_prev[0, 0][torch.as_tensor(idx)])
        tau = float(s.temperature)
        locs0, fluxes0, counts = s.locs.clone(), s.fluxes.clone(), s.counts.clone()
        accepts = []
        usample0, le0 = torch.distributions.Uniform.sample, torch.Tensor.__le__
        state = {"prob": None}

        def usample(self_, *a, **kw):
            o = usample0(self_, *a, **kw)
            state["prob"] = o
            return o

        def le(self_, other):
            o = le0(self_, other)
            if self_ is state["prob"]:
                accepts.append(o.numpy().copy())
            return o

        with Recorder() as rec:
            torch.distributions.Uniform.sample = usample
            torch.Tensor.__le__ = le
            try:
                s.mutate()
            finally:
                torch.distributions.Uniform.sample = usample0
                torch.Tensor.__le__ = le0
        kinds = [k for k, _ in rec.draws]
        assert kinds == ["mask", "rand", "rand", "rand"] * K, kinds[:8]
        masks = np.stack([rec.draws[4 * i][1] for i in range(K)])
        uloc = np.stack([rec.draws[4 * i + 1][1] for i in range(K)])
        uflux = np.stack([rec.draws[4 * i + 2][1] for i in range(K)])
        uacc = np.stack([rec.draws[4 * i + 3][1] for i in range(K)]).astype(np.float32)
        comp = masks.argmax(-1).astype(np.int32)                      # [K,1,1,N]
        j = comp[..., None]
        uloc_sel = np.take_along_axis(uloc, j[..., None].repeat(2, -1), axis=-2)[..., 0, :]
        uflux_sel = np.take_along_axis(uflux, j, axis=-1)[..., 0]
        accept = np.stack(accepts)
        assert accept.shape == comp.shape
        # float64 oracle along the reference's draws: decision margins
        _, _, _, loga, oacc = O.mh_sweep(np32(s.tiled_image), np32(counts), np32(locs0),
                                         np32(fluxes0), np.full((1, 1), tau), o_prior, o_model,
                                         o_mh, comp, uloc_sel, uflux_sel, uacc, trace=True)
        with np.errstate(all="ignore"):
            marg = np.abs(np.log(uacc.astype(np.float64)) - np.minimum(loga, 0))
        marg = np.where(np.isnan(marg), np.inf, marg)[:, 0, 0]          # [K,N]
        low = marg < min_margin
        pin = np.where(low.any(0), low.argmax(0), K).astype(np.int16)
        # where pinned, the oracle decides exactly as the reference did
        pinned = np.arange(K)[:, None] < pin[None, :]
        assert np.array_equal(oacc[:, 0, 0][pinned], accept[:, 0, 0][pinned]), \
            "oracle and reference disagree on a pinned decision"
        print(f"step {it}: tau {tau:.6f}, pinned decisions {int(pinned.sum())} of {K * N}, "
              f"particles fully pinned {int((pin == K).sum())}, accept rate "
              f"{accept.mean():.3f}", flush=True)
        out.update({key + "tau": np.float32(tau), key + "idx": idx,
                    key + "counts": np32(counts), key + "locs0": np32(locs0),
                    key + "fluxes0": np32(fluxes0), key + "comp": comp.astype(np.int8),
                    key + "uloc": uloc_sel.astype(np.float32),
                    key + "uflux": uflux_sel.astype(np.float32), key + "uacc": uacc,
                    key + "accept": accept, key + "locs1": np32(s.locs),
                    key + "fluxes1": np32(s.fluxes), key + "acc": np32(s.mutation_acc_rates),
                    key + "pin": pin})
        s.temper()
        s.update_weights()
    save("mh_teacher_c2.npz", **out)


def run_smc_recorded(image, tile_dim, prior, model, mh, N, method, seed, max_iters):
    torch.manual_seed(seed)
    s = sampler_for(image, tile_dim, prior, model, mh, N, method=method, max_iters=max_iters)
    trace = {"tau": [], "logZ": [], "ess": [], "acc": []}
    orig_uw = s.update_weights

    def uw():
        orig_uw()
        trace["tau"].append(np32(s.temperature))
        trace["logZ"].append(np32(s.log_normalizing_constant))
        trace["ess"].append(np32(s.ess))
        trace["acc"].append(np32(getattr(s, "mutation_acc_rates", torch.zeros_like(s.temperature))))

    s.update_weights = uw
    import contextlib
    import io
    with Recorder() as rec, contextlib.redirect_stdout(io.StringIO()):
        s.run()
    draws = {f"draw_{i:04d}_{k}": v for i, (k, v) in enumerate(rec.draws)}
    return s, trace, draws


def _replay_margin(image, draws, S, K, N):
    """Smallest MH decision margin of an oracle replay of recorded draws."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import smc_oracle as O
    from tests._params import o_m71_mh, o_m71_model, o_m71_prior
    d = {k: v for k, v in draws.items()}
    r = O.smc_run_replay(image, 8, o_m71_prior(8, S, S), o_m71_model(8), o_m71_mh(K), N,
                         O.DrawStream(d), flux_detection_threshold=M71["flux_detection_threshold"])
    return r["min_margin"]


def gen_smc_replay():
    # end-to-end replay: M71 8x8 tile, S=4, N=64, K=5, systematic
    res = m71_truth_image(8, 61)
    mh = SingleComponentMH(5, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    s, trace, draws = run_smc_recorded(res[-1][0], 8, m71_prior(8, 4, 4), m71_model(8), mh,
                                       64, "systematic", 161, 100)
    out = dict(image=np32(s.image), tile_dim=np.int64(8), N=np.int64(64), K=np.int64(5),
               S=np.int64(4), iters=np.int64(s.iter), counts=np32(s.counts), locs=np32(s.locs),
               fluxes=np32(s.fluxes), weights=np32(s.weights), ess=np32(s.ess),
               logZ=np32(s.log_normalizing_constant), temperature=np32(s.temperature),
               acc=np32(s.mutation_acc_rates), pruned_counts=s.pruned_counts.numpy(),
               pruned_locs=np32(s.pruned_locs), pruned_fluxes=np32(s.pruned_fluxes),
               trace_tau=np.stack(trace["tau"]), trace_logZ=np.stack(trace["logZ"]),
               trace_ess=np.stack(trace["ess"]), **draws)
    save("smc_replay_m71_8x8.npz", **out)
    # 2x2 tiles of 8x8 (lockstep stop across tiles), S=3, N=32, K=4.  The
    # first seed from 162 whose every MH decision the float64 oracle makes
    # with |log U - log alpha| >= 1e-4 nats (the reference's float32
    # proposals and sums differ from exact arithmetic by ~1e-5 here), so the
    # whole run is pinned exactly
    res = m71_truth_image(16, 62)
    for seed in range(162, 262):
        mh = SingleComponentMH(4, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
        s, trace, draws = run_smc_recorded(res[-1][0], 8, m71_prior(8, 3, 3), m71_model(8), mh,
                                           32, "systematic", seed, 100)
        margin = _replay_margin(np32(s.image), draws, 3, 4, 32)
        print("smc_replay_m71_tiles seed", seed, "min margin %.2e" % margin, flush=True)
        if margin >= 1e-4:
            break
    out = dict(image=np32(s.image), tile_dim=np.int64(8), N=np.int64(32), K=np.int64(4),
               S=np.int64(3), iters=np.int64(s.iter), counts=np32(s.counts), locs=np32(s.locs),
               fluxes=np32(s.fluxes), weights=np32(s.weights), ess=np32(s.ess),
               logZ=np32(s.log_normalizing_constant), temperature=np32(s.temperature),
               acc=np32(s.mutation_acc_rates), pruned_counts=s.pruned_counts.numpy(),
               pruned_locs=np32(s.pruned_locs), pruned_fluxes=np32(s.pruned_fluxes),
               trace_tau=np.stack(trace["tau"]), trace_logZ=np.stack(trace["logZ"]),
               trace_ess=np.stack(trace["ess"]), **draws)
    save("smc_replay_m71_tiles.npz", **out)


# ----------------------------------------------------------------------------
def gen_stats(which, seeds, part=None):
    """Statistical targets: reference SMCsampler.run() over many seeds."""
    import contextlib
    import io
    torch.set_num_threads(int(os.environ.get("GOLDEN_THREADS", "8")))
    max_iters = 100
    if which == "basic":
        res = basic_truth_image(16, 1)
        img = res[-1][0]
        pr = basic_prior(16, 3, 3)
        mk = lambda: SingleComponentMH(100, 0.1, 100, pr.flux_scale, 1e6)  # noqa: E731
        model, tile, N, method = basic_model(16), 16, 256, "systematic"
    elif which in ("m71", "m71_multinomial"):
        res = m71_truth_image(8, 0)
        img = res[-1][0]
        pr = m71_prior(8, 10, 10)
        mk = lambda: SingleComponentMH(100, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])  # noqa
        model, tile, N = m71_model(8), 8, 1000
        # notebooks/smc.ipynb cell 7 resamples multinomially
        method = "systematic" if which == "m71" else "multinomial"
    elif which == "m71_mala":
        # SingleComponentMALA (smcdet/kernel.py:133-275): 8x8, S=4, N=500, K=50
        res = m71_truth_image(8, 0)
        img = res[-1][0]
        pr = m71_prior(8, 4, 4)
        mk = lambda: SingleComponentMALA(50, 0.1, 2.5, M71["flux_lower"],  # noqa: E731
                                         M71["flux_upper"])
        model, tile, N, method = m71_model(8), 8, 500, "systematic"
    elif which == "c2_moderate":
        # the headline geometry on a 32x32 tile of moderately bright stars
        # (c2_moderate_truth_image): the reduced sampler (N=512, K=20) mixes on
        # it, so log Z across seeds is tight enough to test at the 1% level
        img = c2_moderate_truth_image()
        pr = m71_prior(32, 10, 10, counts_rate=0.003125)
        mk = lambda: SingleComponentMH(20, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])  # noqa
        model, tile, N, method = m71_model(32), 32, 512, "systematic"
        max_iters = 1000
    elif which in ("c2_moderate_4096", "c2_moderate_4096_k100"):
        # the same image at the headline particle count N=4096 (BASELINE
        # configs[1]); K=20 for >= 20 seeds, K=100 (the headline K) for a few
        img = c2_moderate_truth_image()
        pr = m71_prior(32, 10, 10, counts_rate=0.003125)
        K = 100 if which.endswith("k100") else 20
        mk = lambda: SingleComponentMH(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])  # noqa
        model, tile, N, method = m71_model(32), 32, 4096, "systematic"
        max_iters = 1000
    elif which == "c4":
        # BASELINE configs[3]: an 8x8 M71 cutout at the real
        # source density (the "m71" image: generate_images with M71Prior(0, 100),
        # experiments/m71synthetic/generate_images.py:27-67), S=10, N=4096, K=100
        res = m71_truth_image(8, 0)
        img = res[-1][0]
        pr = m71_prior(8, 10, 10)
        mk = lambda: SingleComponentMH(100, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])  # noqa
        model, tile, N, method = m71_model(8), 8, 4096, "systematic"
    elif which == "c2_reduced":
        # the headline geometry (one 32x32 M71 tile, S=10,
        # counts_rate 5/40^2 truth with <= 10 sources) at reduced N and K
        res = m71_truth_image(32, 0, counts_rate=0.003125, max_sources=10)
        img = res[-1][0]
        pr = m71_prior(32, 10, 10, counts_rate=0.003125)
        mk = lambda: SingleComponentMH(20, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])  # noqa
        model, tile, N, method = m71_model(32), 32, 512, "systematic"
        max_iters = 1000  # runs to temperature 1 take ~150-250 iterations here
    else:
        raise ValueError(which)
    rows = []
    for seed in seeds:
        torch.manual_seed(seed)
        s = sampler_for(img, tile, pr, model, mk(), N, method=method, max_iters=max_iters)
        esses, taus = [], []
        orig_uw = s.update_weights

        def uw(s=s, esses=esses, taus=taus, orig_uw=orig_uw):
            orig_uw()
            esses.append(float(s.ess.flatten()[0]))
            taus.append(float(s.temperature.flatten()[0]))

        s.update_weights = uw
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            s.run()
        dt = time.perf_counter() - t0
        pc = s.pruned_counts.flatten()
        hist = np.bincount(pc.numpy().astype(np.int64), minlength=pr.max_objects + 1)
        rows.append(dict(seed=seed, logZ=float(s.log_normalizing_constant.flatten()[0]),
                         iters=int(s.iter), ess_trace=esses, tau_trace=taus,
                         final_ess=float(s.ess.flatten()[0]),
                         pruned_hist=(hist / hist.sum()).tolist(),
                         mean_total_flux=float(s.posterior_mean_total_flux(s.fluxes).flatten()[0]),
                         mean_total_flux_pruned=float(
                             s.posterior_mean_total_flux(s.pruned_fluxes).flatten()[0]),
                         runtime_s=dt))
        print(which, seed, rows[-1]["logZ"], rows[-1]["iters"], f"{dt:.1f}s", flush=True)
        # written after every seed: long background runs keep what they finished
        cfg = dict(which=which, tile=tile, N=N, S=pr.max_objects, K=mk().num_iters,
                   method=method,
                   counts_rate=float(pr.counts_rate) if hasattr(pr, "counts_rate") else None,
                   rho=0.5, torch_threads=torch.get_num_threads(), max_smc_iters=max_iters,
                   kernel="mala" if which.endswith("mala") else "mh")
        path = os.path.join(HERE, f"stats_{which}.json" if part is None
                            else f"stats_{which}.part{part}.json")
        with open(path, "w") as f:
            json.dump(dict(config=cfg, image=img.numpy().tolist(), runs=rows), f)
    print("wrote", path)


def c2_moderate_truth_image():
    """32x32 M71 image of four stars of 2-12 nmgy (peaks ~60-350 ADU over
    the 104 ADU background) and one faint one, drawn with the reference's
    M71ImageModel.sample."""
    torch.manual_seed(72)
    l = torch.tensor([[[[[7.3, 9.6], [21.8, 6.2], [15.1, 24.7], [26.4, 27.9], [4.2, 22.5]]]]])
    f = torch.tensor([[[[12.0, 6.0, 4.0, 2.0, 0.8]]]])
    return m71_model(32).sample(l, f)[0, 0, :, :, 0]


def cssmc_truth_image():
    """8x8 M71 image of two moderate stars (flux 6 and 3 nmgy) for the
    count-stratified targets."""
    torch.manual_seed(71)
    l = torch.tensor([[[[[2.5, 3.2], [5.7, 5.1]]]]])
    f = torch.tensor([[[[6.0, 3.0]]]])
    return m71_model(8).sample(l, f)[0, 0, :, :, 0]


def gen_cssmc(seeds, smax=4, N=512, K=50, which="cssmc", part=None):
    """CS-SMC targets (manuscript.tex:314-356): for each count s, the
    reference's fixed-count SMCsampler (M71Prior with min = max = s) over many
    seeds -> log Z_s; log Z_0 = the reference's log-likelihood of the empty
    catalog (one source of flux 0); log p(s) from the reference prior's own
    Poisson count prior; p(s|x) from each seed's log Z vector."""
    import contextlib
    import io
    torch.set_num_threads(int(os.environ.get("GOLDEN_THREADS", "8")))
    # "c5": BASELINE configs[4]: the C4 cutout (the "m71"
    # image) with count strata 0..6 at N=8192 per count, K=100
    # (manuscript.tex:566,648)
    img = cssmc_truth_image() if which == "cssmc" else m71_truth_image(8, 0)[-1][0]
    model = m71_model(8)
    ll0 = float(model.loglikelihood(img.reshape(1, 1, 8, 8), torch.full((1, 1, 1, 1, 2), 4.0),
                                    torch.zeros(1, 1, 1, 1)).flatten()[0])
    counts = torch.arange(0, smax + 1, dtype=torch.float32)
    log_ps = m71_prior(8, 0, smax).count_prior.log_prob(counts).numpy().astype(np.float64)
    rows = []
    for seed in seeds:
        lz = [ll0]
        iters = [1]
        for s in range(1, smax + 1):
            torch.manual_seed(1000 * seed + s)
            mh = SingleComponentMH(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
            smp = sampler_for(img, 8, m71_prior(8, s, s), model, mh, N)
            with contextlib.redirect_stdout(io.StringIO()):
                smp.run()
            lz.append(float(smp.log_normalizing_constant.flatten()[0]))
            iters.append(int(smp.iter))
        v = np.array(lz) + log_ps
        p = np.exp(v - v.max())
        rows.append(dict(seed=seed, logZ=lz, iters=iters, count_posterior=(p / p.sum()).tolist()))
        print(which, seed, np.round(lz, 2).tolist(), iters, flush=True)
        cfg = dict(tile=8, N=N, K=K, smin=0, smax=smax, method="systematic", rho=0.5, pad=4,
                   log_count_prior=log_ps.tolist(), loglik_empty=ll0)
        path = os.path.join(HERE, f"stats_{which}.json" if part is None
                            else f"stats_{which}.part{part}.json")
        with open(path, "w") as f:
            json.dump(dict(config=cfg, image=img.numpy().tolist(), runs=rows), f)
    print("wrote", path)


class JoinableM71ImageModel(M71ImageModel):
    """The reference M71ImageModel plus the update_psf_grid hook that
    Aggregate.join calls (aggregate.py:241) and no reference image model
    defines.  ImageModel.psf reads image_height / image_width on every call
    (images.py:28-76), so the hook has nothing to update."""

    def update_psf_grid(self):
        pass


def agg_truth_image():
    """16x16 M71 image of five stars, two near the tile boundaries at 8."""
    torch.manual_seed(73)
    l = torch.tensor([[[[[3.2, 4.1], [7.6, 11.3], [12.4, 7.9], [10.8, 13.6], [5.5, 8.4]]]]])
    f = torch.tensor([[[[6.0, 4.0, 3.0, 1.5, 2.5]]]])
    m = JoinableM71ImageModel(image_height=16, image_width=16, background=M71["background"],
                              psf_radius=M71["psf_radius"], adu_per_nmgy=M71["adu_per_nmgy"],
                              psf_params=torch.tensor(M71["psf_params"]),
                              noise_additive=M71["noise_additive"],
                              noise_multiplicative=M71["noise_multiplicative"])
    return m.sample(l, f)[0, 0, :, :, 0]


def agg_inputs(seed, N=48, S=4, H=8, pad=4):
    """Synthetic 2x2-tile particle populations: counts 0..S, compacted
    catalogs uniform in the padded tile, fluxes 0.5-20 nmgy."""
    rng = np.random.default_rng(seed)
    counts = rng.integers(0, S + 1, (2, 2, N)).astype(np.float32)
    mask = np.arange(S) < counts[..., None]
    locs = rng.uniform(-pad, H + pad, (2, 2, N, S, 2)).astype(np.float32) * mask[..., None]
    fluxes = rng.uniform(0.5, 20.0, (2, 2, N, S)).astype(np.float32) * mask
    w = rng.random((2, 2, N)).astype(np.float32)
    w /= w.sum(-1, keepdims=True)
    lnc = rng.normal(-400.0, 5.0, (2, 2)).astype(np.float32)
    return counts, locs, fluxes, w, lnc


def gen_agg():
    """The parts of Aggregate (smcdet/aggregate.py) that run at HEAD, on
    synthetic populations over a 2x2 grid of 8x8 tiles: drop_sources_from_overlap
    (:189-215), join (:217-263, with JoinableM71ImageModel), unjoin
    (:265-324), log_target (:105-130), sort_by_count (:424-437), temper
    (:140-174) and update_weights (:439-483) over two tempering steps."""
    from smcdet.aggregate import Aggregate
    torch.manual_seed(0)
    img = agg_truth_image()
    data = img.unfold(0, 8, 8).unfold(1, 8, 8).contiguous()
    counts, locs, fluxes, w, lnc = agg_inputs(5)
    out = dict(image=np32(img), data=np32(data), counts=counts, locs=locs, fluxes=fluxes,
               weights=w, lnc=lnc)

    def fresh():
        model = JoinableM71ImageModel(image_height=8, image_width=8, background=M71["background"],
                                      psf_radius=M71["psf_radius"],
                                      adu_per_nmgy=M71["adu_per_nmgy"],
                                      psf_params=torch.tensor(M71["psf_params"]),
                                      noise_additive=M71["noise_additive"],
                                      noise_multiplicative=M71["noise_multiplicative"])
        mh = SingleComponentMH(10, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
        return Aggregate(m71_prior(8, 0, 4), model, mh, data.clone(), torch.tensor(counts),
                         torch.tensor(locs), torch.tensor(fluxes), torch.tensor(w),
                         torch.tensor(lnc), M71["flux_detection_threshold"], "multinomial", 0.5)

    for axis in (0, 1):
        agg = fresh()
        c, l, f = agg.drop_sources_from_overlap(axis, torch.tensor(counts), torch.tensor(locs),
                                                torch.tensor(fluxes))
        out[f"drop{axis}_counts"], out[f"drop{axis}_locs"], out[f"drop{axis}_fluxes"] = \
            np32(c), np32(l), np32(f)
        child_model = __import__("copy").deepcopy(agg.ImageModel)
        dat, cs, ls, fs = agg.join(axis, agg.data, c, l, f)
        out[f"join{axis}_data"], out[f"join{axis}_counts"] = np32(dat), np32(cs)
        out[f"join{axis}_locs"], out[f"join{axis}_fluxes"] = np32(ls), np32(fs)
        ud, uc, ul, uf = agg.unjoin(axis, dat, ls, fs)
        out[f"unjoin{axis}_data"], out[f"unjoin{axis}_counts"] = np32(ud), np32(uc)
        out[f"unjoin{axis}_locs"], out[f"unjoin{axis}_fluxes"] = np32(ul), np32(uf)
        tau = torch.full((agg.numH, agg.numW), 0.3)
        lt = agg.log_target(axis, child_model, ud, ul, uf, dat, cs, ls, fs, tau)
        out[f"logtarget{axis}"] = np32(lt)
        out[f"logtarget{axis}_tau"] = np32(tau)
        # two tempering steps over the count groups of the joint population
        agg.data, agg.counts, agg.locs, agg.fluxes = dat, cs, ls, fs
        agg.sort_by_count()
        out[f"sorted{axis}_counts"] = np32(agg.counts)
        out[f"sorted{axis}_locs"] = np32(agg.locs)
        out[f"sorted{axis}_fluxes"] = np32(agg.fluxes)
        groups = agg.num_catalogs_per_count
        out[f"groups{axis}"] = np.array([[np.array(groups[h][x] + [0] * (8 - len(groups[h][x])))
                                          for x in range(agg.numW)] for h in range(agg.numH)])
        ud, uc, ul, uf = agg.unjoin(axis, agg.data, agg.locs, agg.fluxes)
        lc = child_model.loglikelihood(ud, ul, uf)
        agg.loglik_diff = agg.ImageModel.loglikelihood(agg.data, agg.locs, agg.fluxes) - \
            lc.unfold(axis, 2, 2).sum(-1)
        out[f"loglik_diff{axis}"] = np32(agg.loglik_diff)
        rng = np.random.default_rng(11 + axis)
        agg.log_normalizing_constant = [[rng.normal(-300, 3, len(groups[h][x])).tolist()
                                         for x in range(agg.numW)] for h in range(agg.numH)]
        out[f"lnc_in{axis}"] = np.array([[np.array(agg.log_normalizing_constant[h][x]
                                                   + [0.0] * (8 - len(groups[h][x])))
                                          for x in range(agg.numW)] for h in range(agg.numH)])
        agg.temperature_prev = torch.zeros(agg.numH, agg.numW)
        agg.temperature = torch.zeros(agg.numH, agg.numW)
        for step in (1, 2):
            if step == 2:  # a second step from tau > 0 with a perturbed increment
                agg.loglik_diff = agg.loglik_diff * 0.5 + torch.tensor(
                    rng.normal(0, 2, tuple(agg.loglik_diff.shape)).astype(np.float32))
                out[f"loglik_diff{axis}_2"] = np32(agg.loglik_diff)
            agg.temper()
            agg.update_weights()
            out[f"tau{axis}_{step}"] = np32(agg.temperature)
            out[f"w_intra{axis}_{step}"] = np32(agg.weights_intracount)
            out[f"weights{axis}_{step}"] = np32(agg.weights)
            out[f"lnc{axis}_{step}"] = np.array([[np.array(
                [float(v) for v in agg.log_normalizing_constant[h][x]]
                + [0.0] * (8 - len(groups[h][x]))) for x in range(agg.numW)]
                for h in range(agg.numH)])
    save("agg_m71_pieces.npz", **out)


if __name__ == "__main__":
    torch.set_default_dtype(torch.float32)
    what = sys.argv[1] if len(sys.argv) > 1 else "fixtures"
    if what == "fixtures":
        gen_psf()
        gen_loglik()
        gen_prior()
        gen_distributions()
        gen_mh()
        gen_mh_edge()
        gen_smc_steps()
        gen_smc_replay()
        gen_mala()
        gen_mcmc()
        gen_mcmc_edge()
        gen_agg()
    elif what == "steps4096":
        gen_smc_steps_4096()
    elif what == "mh-teacher":
        gen_mh_teacher()
    elif what == "mala":
        gen_mala()
    elif what == "mh-edge":
        gen_mh_edge()
    elif what == "smc-replay":
        gen_smc_replay()
    elif what == "mcmc":
        gen_mcmc()
    elif what == "mcmc-edge":
        gen_mcmc_edge()
    elif what == "agg":
        gen_agg()
    elif what == "cssmc":
        n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
        gen_cssmc(list(range(n)))
    elif what == "c5":
        # c5 [n] [first]: count-stratified reference runs on the C4 cutout
        n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
        first = int(sys.argv[3]) if len(sys.argv) > 3 else None
        gen_cssmc(list(range(first or 0, (first or 0) + n)), smax=6, N=8192, K=100, which="c5",
                  part=first)
    elif what == "stats":
        # stats <which> [n] [first]: seeds first..first+n-1; with `first` the
        # rows go to stats_<which>.part<first>.json (parallel partial runs),
        # merged by `stats-merge <which>`
        which = sys.argv[2]
        n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
        first = int(sys.argv[4]) if len(sys.argv) > 4 else None
        gen_stats(which, list(range(first or 0, (first or 0) + n)), part=first)
    elif what == "stats-merge":
        import glob
        which = sys.argv[2]
        parts = sorted(glob.glob(os.path.join(HERE, f"stats_{which}.part*.json")))
        main = os.path.join(HERE, f"stats_{which}.json")
        docs = ([json.load(open(main))] if os.path.exists(main) else []) + \
            [json.load(open(p)) for p in parts]
        runs = {r["seed"]: r for d in docs for r in d["runs"]}  # later parts win
        runs = [runs[k] for k in sorted(runs)]
        assert all(d["image"] == docs[0]["image"] for d in docs)
        with open(os.path.join(HERE, f"stats_{which}.json"), "w") as f:
            json.dump(dict(config=docs[0]["config"], image=docs[0]["image"], runs=runs), f)
        for p in parts:
            os.remove(p)
        print("merged", len(runs), "runs from", len(parts), "parts")
    else:
        raise SystemExit(f"unknown target {what}")
