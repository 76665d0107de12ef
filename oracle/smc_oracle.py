"""CPU ORACLE for the smcdet hot path — TEST INFRASTRUCTURE ONLY.

A numpy restatement of the reference algorithm (timwhite0/smcdet @ 2026-03-13,
`smcdet/images.py`, `smcdet/prior.py`, `smcdet/distributions.py`,
`smcdet/kernel.py`, `smcdet/sampler.py`).  Every function cites the reference
file:line it restates.  It is the CHECKER for the HIP path: only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may import it.  The
product package (`smcdet_amd`) never imports, links or executes anything here.

Parity pinning: this restatement is checked against golden vectors recorded
from the reference itself (tests/golden/make_golden.py imports /root/reference
in the build container and records inputs, every random draw and outputs);
see tests/test_oracle_golden.py.

Randomness is always explicit: every function that the reference drives with
torch.rand / Multinomial takes the uniforms (or component indices) as arrays,
so a recorded reference run can be replayed bit-for-bit in its decisions.

dtype: arithmetic runs in `dtype` (float64 by default).  Model parameters are
rounded to float32 first wherever the reference stores them as float32
tensors, so the float64 oracle differs from the float32 reference only by
arithmetic rounding.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
from scipy.optimize import brentq
from scipy.special import erf, erfinv, gammaln

F32 = np.float32
FLT_MAX = float(np.finfo(np.float32).max)


def _f32(x):
    return float(np.float32(x))


# ---------------------------------------------------------------------------
# model / prior / kernel parameter containers (float32-rounded like the ref)
# ---------------------------------------------------------------------------
@dataclass
class M71Model:
    """smcdet/images.py:105-135 (M71ImageModel)."""
    H: int
    W: int
    background: float
    psf_radius: int
    adu_per_nmgy: float
    psf_params: tuple
    noise_additive: float = 0.0
    noise_multiplicative: float = 1.0

    def __post_init__(self):
        self.background = _f32(self.background)
        self.adu_per_nmgy = _f32(self.adu_per_nmgy)
        self.psf_params = tuple(_f32(p) for p in self.psf_params)
        self.noise_additive = _f32(self.noise_additive)
        self.noise_multiplicative = _f32(self.noise_multiplicative)
        self.norm_const = m71_psf_normalizer(self.psf_params, self.psf_radius)

    def psf_value(self, r2, dtype=np.float64):
        return m71_psf_unnormalized(r2, self.psf_params, dtype) / dtype(self.norm_const)


@dataclass
class BasicModel:
    """smcdet/images.py:6-26 (ImageModel with Normal-pdf PSF, Poisson noise)."""
    H: int
    W: int
    background: float
    psf_radius: int
    psf_stdev: float

    def __post_init__(self):
        self.background = _f32(self.background)
        self.psf_stdev = _f32(self.psf_stdev)

    def psf_value(self, r2, dtype=np.float64):
        s = dtype(self.psf_stdev)
        # Normal(0, s).log_prob(r).exp()  (images.py:17,25-26)
        return np.exp(-r2 / (2 * s * s) - np.log(s) - dtype(0.5 * math.log(2 * math.pi)))


@dataclass
class M71PriorP:
    """smcdet/prior.py:192-226 (M71Prior) over PoissonProcessPrior :78-101.
    box = (lo_h, lo_w, hi_h, hi_w) replaces [-pad, H+pad) x [-pad, W+pad)
    (a tile's own box when the tiles partition the padded image; the Poisson
    mean is counts_rate times the box area, as for the padded tile)."""
    min_objects: int
    max_objects: int
    counts_rate: float
    H: int
    W: int
    pad: float
    flux_alpha: float
    flux_lower: float
    flux_upper: float
    box: tuple = None

    @property
    def loc_low(self):
        if self.box is not None:
            return np.array([_f32(self.box[0]), _f32(self.box[1])])
        return _f32(-self.pad)

    @property
    def loc_high(self):
        if self.box is not None:
            return (_f32(self.box[2]), _f32(self.box[3]))
        return (_f32(self.H + self.pad), _f32(self.W + self.pad))

    def poisson_mean(self):
        if self.box is not None:
            b = self.box
            return _f32(self.counts_rate * (b[2] - b[0]) * (b[3] - b[1]))
        return _f32(self.counts_rate * (self.H + 2 * self.pad) * (self.W + 2 * self.pad))


@dataclass
class ParetoPriorP:
    """smcdet/prior.py:157-189 (ParetoStarPrior) over PointProcessPrior :8-75."""
    min_objects: int
    max_objects: int
    H: int
    W: int
    pad: float
    flux_scale: float
    flux_alpha: float

    @property
    def loc_low(self):
        return _f32(-self.pad)

    @property
    def loc_high(self):
        return (_f32(self.H + self.pad), _f32(self.W + self.pad))


@dataclass
class MHParams:
    """smcdet/kernel.py:7-24 (SingleComponentMH.__init__); bounds are float32."""
    num_iters: int
    locs_stdev: float
    fluxes_stdev: float
    fluxes_min: float
    fluxes_max: float

    def __post_init__(self):
        self.locs_stdev = _f32(self.locs_stdev)
        self.fluxes_stdev = _f32(self.fluxes_stdev)
        self.fluxes_min = _f32(self.fluxes_min)
        self.fluxes_max = _f32(self.fluxes_max)


# ---------------------------------------------------------------------------
# PSF
# ---------------------------------------------------------------------------
def m71_psf_unnormalized(r2, psf_params, dtype=np.float64):
    """images.py:137-141, written in r^2 (= ||pixel+0.5-loc||^2)."""
    s1, s2, sp, beta, b, p0 = (dtype(p) for p in psf_params)
    r2 = np.asarray(r2, dtype=dtype)
    t1 = np.exp(-r2 / (2 * s1))
    t2 = b * np.exp(-r2 / (2 * s2))
    t3 = p0 * (1 + r2 / (beta * sp)) ** (-beta / 2)
    return (t1 + t2 + t3) / (1 + b + p0)


def m71_psf_normalizer(psf_params, psf_radius):
    """images.py:122-135: sum of the unnormalised PSF over a (32R)^2 grid whose
    centre sits at (16R, 16R) with the +0.5 pixel-centre offset.  Evaluated in
    float64 and rounded to float32 (the reference accumulates in float32:
    12.7525005 vs 12.752501 here, 1 ulp)."""
    n = 32 * psf_radius
    g = np.arange(n, dtype=np.float64) - n / 2.0 + 0.5
    r2 = g[:, None] ** 2 + g[None, :] ** 2
    return _f32(m71_psf_unnormalized(r2, psf_params, np.float64).sum())


def psf_dense(locs, model, dtype=np.float64):
    """images.py:28-76.  locs [nH,nW,N,S,2] -> psf [nH,nW,H,W,N,S]: source j
    contributes phi(||p+0.5-loc_j||) at every pixel p of the (2R+1)^2 window
    anchored at floor(loc_j) that lies inside the tile; zero elsewhere."""
    locs = np.asarray(locs, dtype=dtype)
    H, W, R = model.H, model.W, model.psf_radius
    hh = np.arange(H, dtype=dtype)[:, None, None, None]
    ww = np.arange(W, dtype=dtype)[None, :, None, None]
    lh = locs[..., 0][:, :, None, None]  # [nH,nW,1,1,N,S]
    lw = locs[..., 1][:, :, None, None]
    fh, fw = np.floor(lh), np.floor(lw)
    inwin = (np.abs(hh - fh) <= R) & (np.abs(ww - fw) <= R)
    r2 = (hh + 0.5 - lh) ** 2 + (ww + 0.5 - lw) ** 2
    val = model.psf_value(r2, dtype)
    return np.where(inwin, val, dtype(0))


def render_rate(locs, fluxes, model, dtype=np.float64):
    """images.py:160-167 (M71) / :86-89 (basic): lambda = B + sum_j g*f_j*psf_j,
    g = adu_per_nmgy for M71, 1 for the basic model.  -> [nH,nW,H,W,N]."""
    locs = np.asarray(locs, dtype=dtype)
    fluxes = np.asarray(fluxes, dtype=dtype)
    H, W, R = model.H, model.W, model.psf_radius
    g = dtype(getattr(model, "adu_per_nmgy", 1.0))
    hh = np.arange(H, dtype=dtype)[:, None, None]
    ww = np.arange(W, dtype=dtype)[None, :, None]
    nH, nW, N, S, _ = locs.shape
    rate = np.zeros((nH, nW, H, W, N), dtype=dtype)
    for j in range(S):
        lh = locs[:, :, None, None, :, j, 0]
        lw = locs[:, :, None, None, :, j, 1]
        inwin = (np.abs(hh - np.floor(lh)) <= R) & (np.abs(ww - np.floor(lw)) <= R)
        r2 = (hh + 0.5 - lh) ** 2 + (ww + 0.5 - lw) ** 2
        psf = np.where(inwin, model.psf_value(r2, dtype), dtype(0))
        rate += psf * (g * fluxes[:, :, None, None, :, j])
    return rate + dtype(model.background)


# ---------------------------------------------------------------------------
# log-likelihoods
# ---------------------------------------------------------------------------
def m71_pixel_loglik(x, rate, model, dtype=np.float64):
    """images.py:169-175 per pixel: Normal(rate, sqrt(s0^2 + eta*rate)).log_prob(x)."""
    v = dtype(model.noise_additive) + dtype(model.noise_multiplicative) * rate
    return -((x - rate) ** 2) / (2 * v) - 0.5 * np.log(v) - dtype(0.5 * math.log(2 * math.pi))


def poisson_pixel_loglik(x, rate, dtype=np.float64):
    """images.py:91-102 per pixel: Poisson(rate).log_prob(x), or
    Normal(rate, sqrt(rate)).log_prob(x) where rate > 50000."""
    with np.errstate(divide="ignore", invalid="ignore"):
        xlogy = np.where(x == 0, dtype(0), x * np.log(rate))
    lp = xlogy - rate - gammaln(x + 1)
    ln = -((x - rate) ** 2) / (2 * rate) - 0.5 * np.log(rate) - dtype(0.5 * math.log(2 * math.pi))
    return np.where(rate > 50000, ln, lp)


def loglikelihood(tiled_image, locs, fluxes, model, dtype=np.float64):
    """M71ImageModel.loglikelihood (images.py:159-175) or ImageModel.loglikelihood
    (images.py:85-102).  tiled_image [nH,nW,H,W] -> [nH,nW,N]."""
    rate = render_rate(locs, fluxes, model, dtype)
    x = np.asarray(tiled_image, dtype=dtype)[..., None]
    if isinstance(model, M71Model):
        ll = m71_pixel_loglik(x, rate, model, dtype)
    else:
        ll = poisson_pixel_loglik(x, rate, dtype)
    return ll.sum(axis=(2, 3))


# ---------------------------------------------------------------------------
# priors
# ---------------------------------------------------------------------------
def trunc_pareto_log_prob(f, alpha, lower, upper, dtype=np.float64):
    """distributions.py:64-74, 87-89."""
    a, L, U = dtype(_f32(alpha)), dtype(_f32(lower)), dtype(_f32(upper))
    c = np.log(a) + a * np.log(L) + a * np.log(U) - np.log(U ** a - L ** a)
    return c - (a + 1) * np.log(f)


def trunc_pareto_sample(u, alpha, lower, upper, dtype=np.float64):
    """distributions.py:76-85 (inverse CDF of the bounded Pareto)."""
    a, L, U = dtype(_f32(alpha)), dtype(_f32(lower)), dtype(_f32(upper))
    u = np.asarray(u, dtype=dtype)
    num = U ** a - u * U ** a + u * L ** a
    return (num / (L ** a * U ** a)) ** (-1 / a)


def log_prior(counts, locs, fluxes, prior, dtype=np.float64):
    """M71Prior.log_prob (prior.py:220-226 -> :67-75) or ParetoStarPrior.log_prob
    (prior.py:183-189).  Count prior + uniform locations + flux prior, the last
    two summed over the first `count` sources only."""
    counts = np.asarray(counts, dtype=dtype)
    locs = np.asarray(locs, dtype=dtype)
    fluxes = np.asarray(fluxes, dtype=dtype)
    S = locs.shape[-2]
    mask = np.arange(S)[None] < counts[..., None]
    if isinstance(prior, M71PriorP):
        mu = dtype(prior.poisson_mean())
        lp = counts * np.log(mu) - mu - gammaln(counts + 1)  # Poisson.log_prob
    else:
        k = prior.max_objects - prior.min_objects + 1
        insup = (counts >= prior.min_objects) & (counts <= prior.max_objects)
        lp = np.where(insup, dtype(np.log(np.float32(1.0 / k))), -np.inf)
    lo = np.asarray(prior.loc_low, dtype=dtype)
    hi = np.array(prior.loc_high, dtype=dtype)
    inside = (locs >= lo) & (locs < hi)
    lu = np.where(inside, -np.log(hi - lo), -np.inf)  # Uniform.log_prob
    lp = lp + (lu.sum(-1) * mask).sum(-1)
    if isinstance(prior, M71PriorP):
        L = dtype(_f32(prior.flux_lower))
        ff = fluxes + L * (fluxes == 0)
        lf = trunc_pareto_log_prob(ff, prior.flux_alpha, prior.flux_lower, prior.flux_upper, dtype)
    else:
        sc = dtype(_f32(prior.flux_scale))
        a = dtype(_f32(prior.flux_alpha))
        ff = fluxes + sc * (fluxes == 0)
        lf = np.log(a) + a * np.log(sc) - (a + 1) * np.log(ff)  # Pareto.log_prob
    return lp + (lf * mask).sum(-1)


def prior_sample_stratified(prior, num_tiles_per_side, n_per_count, uloc, uflux,
                            dtype=np.float64):
    """PointProcessPrior.sample with stratify_by_count=True (prior.py:47-64) and
    the flux draw of M71Prior.sample / ParetoStarPrior.sample (prior.py:212-217,
    :175-180), with the uniforms given explicitly:
    uloc [T,T,n,S,2], uflux [T,T,n,S] (n = num_counts * n_per_count)."""
    T = num_tiles_per_side
    strata = np.repeat(np.arange(prior.min_objects, prior.max_objects + 1), n_per_count)
    counts = (strata * np.ones((T, T, strata.size))).astype(dtype)
    S = prior.max_objects
    mask = np.arange(S)[None] < counts[..., None]
    lo = np.asarray(prior.loc_low, dtype=dtype)
    hi = np.array(prior.loc_high, dtype=dtype)
    locs = lo + np.asarray(uloc, dtype=dtype) * (hi - lo)
    locs = locs * mask[..., None]
    if isinstance(prior, M71PriorP):
        fl = trunc_pareto_sample(uflux, prior.flux_alpha, prior.flux_lower, prior.flux_upper, dtype)
    else:
        # torch Pareto.rsample: scale * exp(Exponential(alpha)) via icdf of a uniform
        raise NotImplementedError("ParetoStarPrior.sample draws through torch.distributions.Pareto")
    return counts, locs, fl * mask


# ---------------------------------------------------------------------------
# truncated diagonal normal (distributions.py:22-58)
# ---------------------------------------------------------------------------
def _phi(z):
    return 0.5 * (1 + erf(z / math.sqrt(2)))


def tn_log_Z(mu, sigma, lb, ub):
    """distributions.py:33-35: log(Phi(ub) - Phi(lb)), nan_to_num'd."""
    with np.errstate(divide="ignore", invalid="ignore"):
        lz = np.log(_phi((ub - mu) / sigma) - _phi((lb - mu) / sigma))
    return np.nan_to_num(lz, nan=0.0, posinf=FLT_MAX, neginf=-FLT_MAX)


def tn_sample(mu, sigma, lb, ub, u):
    """distributions.py:40-48 with the uniform u given."""
    p = np.clip(u, 1e-6, 1.0 - 1e-6)
    ptil = _phi((lb - mu) / sigma) + p * np.exp(tn_log_Z(mu, sigma, lb, ub))
    ptil = np.clip(ptil, 1e-6, 1.0 - 1e-6)
    x = mu + sigma * math.sqrt(2) * erfinv(2 * ptil - 1)
    return np.clip(x, lb, ub)


def tn_log_prob(v, mu, sigma, lb, ub):
    """distributions.py:50-52: Normal(mu, sigma).log_prob(v) - log Z."""
    ln = -((v - mu) ** 2) / (2 * sigma * sigma) - np.log(sigma) - 0.5 * math.log(2 * math.pi)
    return ln - tn_log_Z(mu, sigma, lb, ub)


# ---------------------------------------------------------------------------
# single-component MH sweep (kernel.py:26-130), replayed draws
# ---------------------------------------------------------------------------
def log_target(tiled_image, counts, locs, fluxes, tau, prior, model, dtype=np.float64):
    """sampler.py:87-91: Prior.log_prob + tau * ImageModel.loglikelihood."""
    lp = log_prior(counts, locs, fluxes, prior, dtype)
    ll = loglikelihood(tiled_image, locs, fluxes, model, dtype)
    return lp + np.asarray(tau, dtype=dtype)[..., None] * ll


def mh_sweep(tiled_image, counts, locs, fluxes, tau, prior, model, mh,
             comp, uloc, uflux, uacc, dtype=np.float64, trace=False, edge_freeze=True):
    """SingleComponentMH.run (kernel.py:26-130) with its draws given explicitly:
    comp [K,nH,nW,N] (the one-hot component of Multinomial.sample, :44),
    uloc [K,nH,nW,N,2] / uflux [K,nH,nW,N] (torch.rand of the truncated-normal
    proposals for the chosen component, :47-61), uacc [K,nH,nW,N] (:115).
    Returns (locs, fluxes, acc_rate_of_last_iteration [nH,nW]) and, with
    trace=True, per-iteration log-alpha and accept flags.  edge_freeze=False
    caches the target with np.where instead of the reference's arithmetic
    (no NaN after a rejected upper-edge proposal: what the reference would do
    with torch.where as its MALA kernel caches, kernel.py:273)."""
    locs = np.array(locs, dtype=dtype)
    fluxes = np.array(fluxes, dtype=dtype)
    K = comp.shape[0]
    lb_l = np.asarray(prior.loc_low, dtype=dtype)
    ub_l = np.array(prior.loc_high, dtype=dtype)
    sl, sf = dtype(mh.locs_stdev), dtype(mh.fluxes_stdev)
    lb_f, ub_f = dtype(mh.fluxes_min), dtype(mh.fluxes_max)
    cur_lt = log_target(tiled_image, counts, locs, fluxes, tau, prior, model, dtype)  # :89-96
    loga_tr, acc_tr = [], []
    accept = None
    for k in range(K):
        j = comp[k][..., None]  # [nH,nW,N,1]
        lj = np.take_along_axis(locs, j[..., None].repeat(2, -1), axis=-2)[..., 0, :]
        fj = np.take_along_axis(fluxes, j, axis=-1)[..., 0]
        # proposals are stored as the reference's float32 state holds them: a
        # draw within half an ulp of the box's upper edge lands exactly on it
        lnew = tn_sample(lj, sl, lb_l, ub_l, uloc[k].astype(dtype))  # :47-52
        fnew = tn_sample(fj, sf, lb_f, ub_f, uflux[k].astype(dtype))  # :53-61
        lnew = lnew.astype(np.float32).astype(dtype)
        fnew = fnew.astype(np.float32).astype(dtype)
        pl = locs.copy()
        pf = fluxes.copy()
        np.put_along_axis(pl, j[..., None].repeat(2, -1), lnew[..., None, :], axis=-2)
        np.put_along_axis(pf, j, fnew[..., None], axis=-1)
        new_lt = log_target(tiled_image, counts, pl, pf, tau, prior, model, dtype)  # :64-70
        q_num = (tn_log_prob(lj, lnew, sl, lb_l, ub_l).sum(-1)  # :71-85
                 + tn_log_prob(fj, fnew, sf, lb_f, ub_f))
        q_den = (tn_log_prob(lnew, lj, sl, lb_l, ub_l).sum(-1)  # :97-111
                 + tn_log_prob(fnew, fj, sf, lb_f, ub_f))
        loga = (new_lt + q_num) - (cur_lt + q_den)
        with np.errstate(over="ignore", invalid="ignore"):
            alpha = np.minimum(np.exp(loga), 1.0)  # :114
        accept = uacc[k].astype(dtype) <= alpha  # :115-116
        locs = np.where(accept[..., None, None], pl, locs)  # :118-122
        fluxes = np.where(accept[..., None], pf, fluxes)
        # :125 caches log_num_target * accept + log_denom_target * ~accept: a
        # rejected -inf target (a location on the box's upper edge, log prior
        # -inf) becomes NaN, and every later proposal of the particle is rejected
        if edge_freeze:
            with np.errstate(invalid="ignore"):
                cur_lt = new_lt * accept + cur_lt * (~accept)
        else:
            cur_lt = np.where(accept, new_lt, cur_lt)
        if trace:
            loga_tr.append(loga)
            acc_tr.append(accept)
    acc_rate = accept.astype(dtype).mean(-1)  # :130
    if trace:
        return locs, fluxes, acc_rate, np.stack(loga_tr), np.stack(acc_tr)
    return locs, fluxes, acc_rate


# ---------------------------------------------------------------------------
# SMC steps (sampler.py)
# ---------------------------------------------------------------------------
def _lse(x):
    m = np.max(x)
    if not np.isfinite(m):
        return m
    return m + np.log(np.sum(np.exp(x - m)))


def tempering_objective(loglik, delta, ess_threshold, dtype=np.float64):
    """sampler.py:93-97: exp(2 LSE(delta*l) - LSE(2 delta*l)) - rho*N.  The
    reference multiplies a float32 tensor by the python float delta, i.e. at
    float32(delta); that rounding is reproduced in float32 mode."""
    d = dtype(delta)
    ll = np.asarray(loglik, dtype=dtype)
    return float(np.exp(2 * _lse(d * ll) - _lse(2 * d * ll)) - ess_threshold)


def temper(loglik, temperature, ess_threshold, dtype=np.float64):
    """sampler.py:99-125 per tile: if f(1-tau) < 0, delta = brentq(f, 0, 1-tau,
    xtol=rtol=1e-6), else delta = 1-tau.  delta is stored float32 and the new
    temperature is the float32 sum tau + delta.  Returns (tau_new, delta)."""
    temperature = np.asarray(temperature, dtype=np.float32)
    nH, nW = temperature.shape
    delta = np.zeros((nH, nW), dtype=np.float32)
    for h in range(nH):
        for w in range(nW):
            top = 1 - float(temperature[h, w])

            def f(d, h=h, w=w):
                return tempering_objective(loglik[h, w], d, ess_threshold, dtype)

            if f(top) < 0:
                delta[h, w] = brentq(f, 0.0, top, xtol=1e-6, rtol=1e-6)
            else:
                delta[h, w] = top
    return (temperature + delta).astype(np.float32), delta


def update_weights(loglik, temperature, temperature_prev, log_norm_const, N,
                   dtype=np.float64):
    """sampler.py:181-196: log w = nan_to_num((tau - tau_prev) * l, nan=-inf);
    W = softmax; ESS = 1/sum W^2; logZ += m + log(sum exp(w - m) / N)."""
    d = (np.asarray(temperature, np.float32) - np.asarray(temperature_prev, np.float32))
    lw = d.astype(dtype)[..., None] * np.asarray(loglik, dtype=dtype)
    lw = np.nan_to_num(lw, nan=-np.inf, posinf=FLT_MAX, neginf=-FLT_MAX)
    m = lw.max(-1)
    e = np.exp(lw - m[..., None])
    s = e.sum(-1)
    W = e / s[..., None]
    ess = 1.0 / (W ** 2).sum(-1)
    logZ = np.asarray(log_norm_const, dtype=dtype) + m + np.log(s / N)
    return W, ess, logZ


def systematic_resample_index(W, U):
    """sampler.py:135-150: u_n = (n + U)/N (float32), bins = cumsum(W) (CPU
    torch accumulates float32 cumsum in double and rounds each output),
    idx = bucketize(u, bins, right=False) = first i with bins[i] >= u_n,
    clamped to [0, N-1]."""
    W = np.asarray(W, dtype=np.float32)
    nH, nW, N = W.shape
    bins = np.cumsum(W.astype(np.float64), axis=-1).astype(np.float32)
    n = np.arange(N, dtype=np.float32)
    u = ((n[None, None] + np.asarray(U, np.float32)[..., None]).astype(np.float32)
         / np.float32(N)).astype(np.float32)
    idx = np.empty((nH, nW, N), dtype=np.int64)
    for h in range(nH):
        for w in range(nW):
            idx[h, w] = np.searchsorted(bins[h, w], u[h, w], side="left")
    return np.clip(idx, 0, N - 1)


def gather_particles(idx, counts, locs, fluxes):
    """sampler.py:150-169."""
    c = np.take_along_axis(counts, idx, axis=-1)
    f = np.take_along_axis(fluxes, idx[..., None], axis=2)
    l = np.take_along_axis(locs, idx[..., None, None], axis=2)
    return c, l, f


def prune(locs, fluxes, tile_dim, flux_detection_threshold):
    """sampler.py:198-219: keep sources with 0 < loc < tile_dim (both coords)
    and flux > threshold; count them; compact kept sources to the front in
    their original order (zeros behind)."""
    locs = np.asarray(locs)
    fluxes = np.asarray(fluxes)
    mask = np.all((locs > 0) & (locs < tile_dim), axis=-1)
    mask &= fluxes > np.float32(flux_detection_threshold)
    counts = mask.sum(-1)
    order = np.argsort(~mask, axis=-1, kind="stable")
    pl = np.take_along_axis(locs * mask[..., None], order[..., None], axis=-2)
    pf = np.take_along_axis(fluxes * mask, order, axis=-1)
    return counts, pl, pf


class DrawStream:
    """Replays a recorded reference draw sequence (tests/golden/*replay*.npz)."""

    def __init__(self, npz):
        names = npz.files if hasattr(npz, "files") else list(npz)
        keys = sorted(k for k in names if k.startswith("draw_"))
        self.items = [(k.split("_", 2)[2], npz[k]) for k in keys]
        self.pos = 0

    def next(self, kind):
        k, v = self.items[self.pos]
        assert k == kind, (self.pos, k, kind)
        self.pos += 1
        return v


def smc_run_replay(image, tile_dim, prior, model, mh, num_catalogs, draws,
                   ess_threshold_prop=0.5, max_smc_iters=100,
                   flux_detection_threshold=0.0, dtype=np.float64):
    """SMCsampler.run (sampler.py:221-256) with systematic resampling, replaying
    the recorded reference draws.  Returns a dict of the sampler's attributes
    (plus min_margin: the smallest |log U - min(log alpha, 0)| of any MH
    decision of the run, i.e. how close the run came to a near-tie)."""
    image = np.asarray(image, dtype=np.float32)
    nt = image.shape[0] // tile_dim
    tiled = image[: nt * tile_dim, : nt * tile_dim].reshape(nt, tile_dim, nt, tile_dim)
    tiled = tiled.transpose(0, 2, 1, 3)
    N = num_catalogs
    rhoN = ess_threshold_prop * num_catalogs
    # initialize (sampler.py:57-85)
    n_per = N
    uloc = draws.next("rand")
    uflux = draws.next("rand")
    counts, locs, fluxes = prior_sample_stratified(prior, nt, n_per, uloc, uflux, dtype)
    N = counts.shape[-1]
    tau = np.zeros((nt, nt), np.float32)
    logZ = np.zeros((nt, nt), dtype)
    # temper + update_weights
    ll = loglikelihood(tiled, locs, fluxes, model, dtype)
    tau_prev = tau
    tau, _ = temper(ll, tau, rhoN, np.float32 if dtype == np.float32 else dtype)
    W, ess, logZ = update_weights(ll, tau, tau_prev, logZ, N, dtype)
    it = 0
    acc = None
    min_margin = np.inf
    trace = {"tau": [tau.copy()], "logZ": [logZ.copy()], "ess": [ess.copy()]}
    K = mh.num_iters
    while np.any(tau < 1) and it <= max_smc_iters:
        it += 1
        U = draws.next("rand")
        idx = systematic_resample_index(W, U)
        counts, locs, fluxes = gather_particles(idx, counts, locs, fluxes)
        comp, ul, uf, ua = [], [], [], []
        for _ in range(K):
            mask = draws.next("mask")
            rl = draws.next("rand")
            rf = draws.next("rand")
            ra = draws.next("rand")
            j = mask.argmax(-1)
            comp.append(j)
            ul.append(np.take_along_axis(rl, j[..., None, None].repeat(2, -1), axis=-2)[..., 0, :])
            uf.append(np.take_along_axis(rf, j[..., None], axis=-1)[..., 0])
            ua.append(ra)
        locs, fluxes, acc, loga, _ = mh_sweep(tiled, counts, locs, fluxes, tau, prior, model,
                                              mh, np.stack(comp), np.stack(ul), np.stack(uf),
                                              np.stack(ua), dtype, trace=True)
        with np.errstate(all="ignore"):
            mg = np.abs(np.log(np.stack(ua).astype(np.float64)) - np.minimum(loga, 0))
        mg = mg[np.isfinite(mg)]
        if mg.size:
            min_margin = min(min_margin, float(mg.min()))
        ll = loglikelihood(tiled, locs, fluxes, model, dtype)
        tau_prev = tau
        tau, _ = temper(ll, tau, rhoN, np.float32 if dtype == np.float32 else dtype)
        W, ess, logZ = update_weights(ll, tau, tau_prev, logZ, N, dtype)
        trace["tau"].append(tau.copy())
        trace["logZ"].append(logZ.copy())
        trace["ess"].append(ess.copy())
    U = draws.next("rand")
    idx = systematic_resample_index(W, U)
    counts, locs, fluxes = gather_particles(idx, counts, locs, fluxes)
    W = np.full_like(W, 1.0 / N)
    pc, pl, pf = prune(locs, fluxes, tile_dim, flux_detection_threshold)
    return dict(counts=counts, locs=locs, fluxes=fluxes, weights=W, ess=ess,
                logZ=logZ, temperature=tau, iters=it, acc=acc, pruned_counts=pc,
                pruned_locs=pl, pruned_fluxes=pf, min_margin=min_margin,
                trace={k: np.stack(v) for k, v in trace.items()})


# ---------------------------------------------------------------------------
# count-stratified SMC combination (manuscript/manuscript.tex:344-354)
# ---------------------------------------------------------------------------
def log_count_prior(prior, dtype=np.float64):
    """log p(s), s = min..max: Poisson(mu).log_prob (prior.py:91-97) for the
    M71 prior, DiscreteUniform(min, max).log_prob (distributions.py:14-19)
    otherwise."""
    s = np.arange(prior.min_objects, prior.max_objects + 1, dtype=dtype)
    if isinstance(prior, M71PriorP):
        mu = dtype(prior.poisson_mean())
        return s * np.log(mu) - mu - gammaln(s + 1)
    return np.full(s.shape, -np.log(s.size), dtype=dtype)


def count_posterior(log_Z, log_prior_s):
    """p(s|x) = p(s) Z_s / sum_s' p(s') Z_s' (manuscript.tex:344) over the last
    axis of log_Z [..., NS]; float64."""
    v = np.asarray(log_Z, np.float64) + np.asarray(log_prior_s, np.float64)
    m = v.max(-1, keepdims=True)
    e = np.exp(v - m)
    return e / e.sum(-1, keepdims=True)


def count_posterior_draw(probs, u_strata, u_pick, N, method="systematic"):
    """s^n ~ p(s|x) and a uniform particle of that stratum (manuscript.tex:349).
    probs [T, NS] (float64), u_strata [T] (systematic) or [T, n_out]
    (multinomial), u_pick [T, n_out] float32.  Stratum of draw n = first k with
    cumsum(probs)[k] >= u_n (u_n = (n + U)/n_out for systematic), particle
    m_n = min(floor(v_n * N), N - 1) in float32.  Returns flat indices
    k_n * N + m_n [T, n_out]."""
    probs = np.asarray(probs, np.float64)
    T, NS = probs.shape
    u_pick = np.asarray(u_pick, np.float32)
    n_out = u_pick.shape[-1]
    cdf = np.cumsum(probs, -1)
    if method == "systematic":
        u = (np.arange(n_out)[None] + np.asarray(u_strata, np.float64)[:, None]) / n_out
    else:
        u = np.asarray(u_strata, np.float32).astype(np.float64)
    k = np.empty((T, n_out), np.int64)
    for t in range(T):
        k[t] = np.minimum(np.searchsorted(cdf[t], u[t], side="left"), NS - 1)
    m = np.minimum((u_pick * np.float32(N)).astype(np.int64), N - 1)
    return k * N + m
