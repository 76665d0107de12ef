"""ctypes wrapper of oracle/mh_oracle.c (CPU ORACLE / CPU BASELINE — test
infrastructure only; never imported by the product package)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from . import smc_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libmh_oracle.so")
LIB_F32 = os.path.join(HERE, "libmh_oracle_f32.so")


class _Model(ctypes.Structure):
    _fields_ = [("model", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
                ("R", ctypes.c_int)] + [(k, ctypes.c_double) for k in (
                    "bg", "g", "s1", "s2", "sp", "beta", "b", "p0", "norm", "psf_stdev",
                    "s0sq", "eta")]


class _Prior(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int)] + [(k, ctypes.c_double) for k in (
        "alpha", "lower", "loc_low", "loc_high_h", "loc_high_w")]


class _MH(ctypes.Structure):
    _fields_ = [("K", ctypes.c_int)] + [(k, ctypes.c_double) for k in (
        "sl", "sf", "lb_h", "lb_w", "ub_h", "ub_w", "lb_f", "ub_f")]


_lib = None
_lib_f32 = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        _lib.mh_oracle_sweep.restype = ctypes.c_int
        _lib.mala_oracle_sweep.restype = ctypes.c_int
        _lib.mh_oracle_loglik.restype = ctypes.c_int
        _lib.mh_oracle_sweep_cached.restype = ctypes.c_int
        _lib.mh_oracle_loglik_cached.restype = ctypes.c_int
    return _lib


def lib_f32():
    """The float32 arithmetic-class build (mh_oracle.c -DOM_F32): only the
    cached sweep and the log-likelihood."""
    global _lib_f32
    if _lib_f32 is None:
        if not os.path.exists(LIB_F32):
            build()
        _lib_f32 = ctypes.CDLL(LIB_F32)
        _lib_f32.mh_oracle_sweep_cached.restype = ctypes.c_int
        _lib_f32.mh_oracle_loglik_cached.restype = ctypes.c_int
    return _lib_f32


def _arith_lib(arith):
    if arith not in ("f64", "f32"):
        raise ValueError(f"arith must be 'f64' or 'f32', not {arith!r}")
    return lib_f32() if arith == "f32" else lib()


def _pack(model, prior, mh):
    m = _Model()
    m.H, m.W, m.R = model.H, model.W, model.psf_radius
    m.bg = model.background
    if isinstance(model, O.M71Model):
        m.model = 1
        m.g = model.adu_per_nmgy
        m.s1, m.s2, m.sp, m.beta, m.b, m.p0 = model.psf_params
        m.norm = model.norm_const
        m.s0sq, m.eta = model.noise_additive, model.noise_multiplicative
    else:
        m.model = 2
        m.g = 1.0
        m.psf_stdev = model.psf_stdev
    p = _Prior()
    p.kind = 1 if isinstance(prior, O.M71PriorP) else 2
    p.alpha = float(np.float32(prior.flux_alpha))
    p.lower = float(np.float32(prior.flux_lower if isinstance(prior, O.M71PriorP)
                               else prior.flux_scale))
    p.loc_low = float(np.float32(prior.loc_low))
    p.loc_high_h, p.loc_high_w = (float(np.float32(v)) for v in prior.loc_high)
    h = _MH()
    h.K = mh.num_iters
    h.sl, h.sf = mh.locs_stdev, mh.fluxes_stdev
    h.lb_h = h.lb_w = prior.loc_low
    h.ub_h, h.ub_w = prior.loc_high
    h.lb_f, h.ub_f = mh.fluxes_min, mh.fluxes_max
    return m, p, h


def mh_sweep(tiled_image, counts, locs, fluxes, tau, prior, model, mh, replay=None, seed=0,
             threads=0, frozen_out=False, cached=False, arith="f64"):
    """Runs the C sweep; returns (locs, fluxes, acc_rate[nH,nW]) (+ the
    [nH,nW,N] mask of particles frozen by an upper-edge proposal).
    cached=True: the cached re-render (mh_oracle_sweep_cached; bit-identical
    in float64); arith="f32": its float32 arithmetic-class build."""
    if arith != "f64" and not cached:
        raise ValueError("the float32 build has the cached sweep only")
    img = np.ascontiguousarray(tiled_image, dtype=np.float32)
    nH, nW, N, S, _ = np.shape(locs)
    T = nH * nW
    c = np.ascontiguousarray(counts, dtype=np.float32)
    l = np.array(locs, dtype=np.float32, order="C")
    f = np.array(fluxes, dtype=np.float32, order="C")
    t = np.ascontiguousarray(np.broadcast_to(np.asarray(tau, np.float32), (nH, nW)))
    acc = np.zeros((T, N), np.uint8)
    m, p, h = _pack(model, prior, mh)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p) if a is not None else None  # noqa: E731
    rc_ = ru = rf = ra = None
    if replay is not None:
        rc_ = np.ascontiguousarray(replay["comp"], dtype=np.int32)
        ru = np.ascontiguousarray(replay["uloc"], dtype=np.float32)
        rf = np.ascontiguousarray(replay["uflux"], dtype=np.float32)
        ra = np.ascontiguousarray(replay["uacc"], dtype=np.float32)
    if cached:
        upper = float(getattr(prior, "flux_upper", 0.0))
        _arith_lib(arith).mh_oracle_sweep_cached(
            ctypes.byref(m), ctypes.byref(p), ctypes.byref(h), P(img), P(c), P(l), P(f), P(t), T,
            N, S, P(rc_), P(ru), P(rf), P(ra), ctypes.c_uint64(seed), threads, P(acc),
            ctypes.c_double(upper))
    else:
        lib().mh_oracle_sweep(ctypes.byref(m), ctypes.byref(p), ctypes.byref(h), P(img), P(c),
                              P(l), P(f), P(t), T, N, S, P(rc_), P(ru), P(rf), P(ra),
                              ctypes.c_uint64(seed), threads, P(acc))
    acc = acc.reshape(nH, nW, N)
    rate = (acc == 1).mean(-1)
    return (l, f, rate, acc == 2) if frozen_out else (l, f, rate)


def sweep_draws(seed, T, N, K, S):
    """The draws mh_oracle_sweep makes from its own stream when no replay
    arrays are given (oracle/mh_oracle.c: splitmix64 per particle, state
    seed ^ 0xA5A5A5A5 (pid + 1); per iteration the component, then the h, w,
    flux and accept uniforms, 24-bit, exact in float32), as replay arrays
    comp [K,T,N] int32, uloc [K,T,N,2], uflux / uacc [K,T,N] float32: a
    sweep replaying them makes the same decisions as the seeded sweep (the
    paired replays of tests/test_gpu_paired.py)."""
    u64 = np.uint64
    pid = np.arange(T * N, dtype=np.uint64)
    st = u64(seed) ^ (u64(0xA5A5A5A5) * (pid + u64(1)))
    out = np.empty((K, 5, T * N), np.float64)
    with np.errstate(over="ignore"):
        for k in range(K):
            for d in range(5):
                st = st + u64(0x9E3779B97F4A7C15)
                z = (st ^ (st >> u64(30))) * u64(0xBF58476D1CE4E5B9)
                z = (z ^ (z >> u64(27))) * u64(0x94D049BB133111EB)
                z = z ^ (z >> u64(31))
                out[k, d] = (z >> u64(40)).astype(np.float64) * (1.0 / 16777216.0)
    comp = np.minimum((out[:, 0] * S).astype(np.int32), S - 1)
    return {"comp": comp.reshape(K, T, N),
            "uloc": np.stack([out[:, 1], out[:, 2]], -1).astype(np.float32).reshape(K, T, N, 2),
            "uflux": out[:, 3].astype(np.float32).reshape(K, T, N),
            "uacc": out[:, 4].astype(np.float32).reshape(K, T, N)}


def loglik(tiled_image, locs, fluxes, model, threads=0, arith="f64"):
    """Image log-likelihoods [nH,nW,N] (float64 array) of the catalogs, by the
    C restatement (images.py:159-175 / :85-102); arith="f32": computed in the
    float32 build (values are float32 numbers)."""
    img = np.ascontiguousarray(tiled_image, dtype=np.float32)
    nH, nW, N, S, _ = np.shape(locs)
    l = np.ascontiguousarray(locs, dtype=np.float32)
    f = np.ascontiguousarray(fluxes, dtype=np.float32)
    out = np.empty(nH * nW * N, np.float64)
    prior = O.M71PriorP(S, S, 0.0, model.H, model.W, 0, 1.0, 1.0, 2.0) \
        if isinstance(model, O.M71Model) else O.ParetoPriorP(S, S, model.H, model.W, 0, 1.0, 1.0)
    m, _, _ = _pack(model, prior, O.MHParams(0, 1.0, 1.0, 0.1, 1.0))
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    fn = lib().mh_oracle_loglik if arith == "f64" else _arith_lib(arith).mh_oracle_loglik_cached
    fn(ctypes.byref(m), P(img), P(l), P(f), nH * nW, N, S, threads, P(out))
    return out.reshape(nH, nW, N)


def mala_sweep(tiled_image, counts, locs, fluxes, tau, prior, model, mala, replay=None, seed=0,
               threads=0, record=False):
    """SingleComponentMALA.run (smcdet/kernel.py:133-275) in C.  `mala` has
    the MHParams fields with locs_stdev / fluxes_stdev = the step sizes.
    Returns (locs, fluxes, acc_rate[nH,nW]) and, with record=True, also the
    per-iteration gradients and proposals [K,nH,nW,N,3]."""
    img = np.ascontiguousarray(tiled_image, dtype=np.float32)
    nH, nW, N, S, _ = np.shape(locs)
    T = nH * nW
    K = mala.num_iters
    c = np.ascontiguousarray(counts, dtype=np.float32)
    l = np.array(locs, dtype=np.float32, order="C")
    f = np.array(fluxes, dtype=np.float32, order="C")
    t = np.ascontiguousarray(np.broadcast_to(np.asarray(tau, np.float32), (nH, nW)))
    acc = np.zeros((T, N), np.uint8)
    grads = np.zeros((K, nH, nW, N, 3), np.float32) if record else None
    props = np.zeros((K, nH, nW, N, 3), np.float32) if record else None
    m, p, h = _pack(model, prior, mala)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p) if a is not None else None  # noqa: E731
    rc_ = ru = rf = ra = None
    if replay is not None:
        rc_ = np.ascontiguousarray(replay["comp"], dtype=np.int32)
        ru = np.ascontiguousarray(replay["uloc"], dtype=np.float32)
        rf = np.ascontiguousarray(replay["uflux"], dtype=np.float32)
        ra = np.ascontiguousarray(replay["uacc"], dtype=np.float32)
    lib().mala_oracle_sweep(ctypes.byref(m), ctypes.byref(p), ctypes.byref(h), P(img), P(c),
                            P(l), P(f), P(t), T, N, S, P(rc_), P(ru), P(rf), P(ra),
                            ctypes.c_uint64(seed), threads, P(acc), P(grads), P(props))
    out = (l, f, acc.reshape(nH, nW, N).mean(-1))
    return out + (grads, props) if record else out


def mh_chain(tiled_image, counts, init_locs, init_fluxes, prior, model, mh, total, burnin, keep,
             replay):
    """MHsampler.run (smcdet/sampler.py:420-486): one MH chain per tile at
    temperature 1, as total-1 single-iteration sweeps of the C restatement
    under the recorded draws (replay [K, nH, nW] / [K, nH, nW, 2]).  Returns
    the kept samples (sample m = state after iteration m-1, m >= burnin,
    every keep-th) [nH,nW,M,S,2] / [nH,nW,M,S] and the accept flags [nH,nW,K]."""
    import copy
    nH, nW = np.shape(init_locs)[:2]
    m1 = copy.copy(mh)
    m1.num_iters = 1
    l = np.asarray(init_locs, np.float32)[:, :, None].copy()
    f = np.asarray(init_fluxes, np.float32)[:, :, None].copy()
    c = np.asarray(counts, np.float32).reshape(nH, nW, 1)
    kept_l, kept_f, acc = [], [], []
    if burnin == 0:
        kept_l.append(l[:, :, 0].copy())
        kept_f.append(f[:, :, 0].copy())
    # an upper-edge proposal freezes the chain for the rest of the run
    # (sampler.py:522-526 caches NaN as the current log target)
    frozen = np.zeros((nH, nW), bool)
    for k in range(total - 1):
        rp = {"comp": replay["comp"][k][None, ..., None],
              "uloc": replay["uloc"][k][None, :, :, None],
              "uflux": replay["uflux"][k][None, ..., None],
              "uacc": replay["uacc"][k][None, ..., None]}
        l2, f2, a, fz = mh_sweep(tiled_image, c, l, f, 1.0, prior, model, m1, replay=rp,
                                 threads=1, frozen_out=True)
        keep_old = frozen[..., None, None, None]
        l = np.where(keep_old, l, l2)
        f = np.where(frozen[..., None, None], f, f2)
        a = np.where(frozen, 0.0, a)
        frozen |= fz[..., 0]
        acc.append(a)
        m = k + 1
        if m >= burnin and (m - burnin) % keep == 0:
            kept_l.append(l[:, :, 0].copy())
            kept_f.append(f[:, :, 0].copy())
    return (np.stack(kept_l, 2), np.stack(kept_f, 2),
            np.stack(acc, -1).astype(np.int32))
