"""CPU ORACLE for tile aggregation (smcdet/aggregate.py) — TEST INFRASTRUCTURE ONLY.

A numpy restatement of the reference's Aggregate (divide-and-conquer SMC over
neighbouring tiles), used as the checker of smcdet_amd/aggregate.py and the
smcdet_aggregate_* kernels.  Only tests/ may import it.

The reference cannot run at HEAD (Aggregate.join calls
ImageModel.update_psf_grid, which no image model defines, and Aggregate.mutate
passes nine arguments to a six-argument SingleComponentMH.run), so this is the
repaired design of DESIGN.md §9, and each function names what it keeps and
what it repairs.  The pieces that do run in the reference (drop, join with the
missing update_psf_grid supplied, unjoin, log_target, temper, update_weights,
sort_by_count) are pinned by tests/golden/agg_m71_pieces.npz
(make_golden.py gen_agg); the rest is parity unpinned.

Catalog convention: counts [..,N], locs [..,N,S,2], fluxes [..,N,S]; the
sources of a particle are slots 0..count-1 (compacted to the front) and the
slots past the count hold zeros.  The reference tests presence as `loc != 0`
(aggregate.py:192-211, :246-253, :320-321); on compacted catalogs the two agree
except for a source exactly on a coordinate 0, which has probability zero.
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import brentq

from oracle.smc_oracle import (M71Model, BasicModel, log_prior, loglikelihood, tempering_objective,
                               tn_log_prob, tn_sample)


def present(counts, S):
    return np.arange(S) < np.asarray(counts)[..., None]


def compact(keep, locs, fluxes):
    """Stable compaction of the kept slots to the front (zeros behind): the
    reference's sort-by-nonzero + gather (aggregate.py:252-261, :280-317)."""
    order = np.argsort(~keep, axis=-1, kind="stable")
    l = np.take_along_axis(locs * keep[..., None], order[..., None], axis=-2)
    f = np.take_along_axis(fluxes * keep, order, axis=-1)
    return keep.sum(-1), l, f


def drop_sources_from_overlap(axis, counts, locs, fluxes, dim):
    """aggregate.py:189-215: tiles at even positions along `axis` drop their
    sources at coordinate >= dim (the padding shared with the next tile) or
    == 0; odd tiles drop those at coordinate <= 0.  Returns compacted catalogs
    (the reference zeroes in place and compacts in join)."""
    counts = np.asarray(counts)
    locs = np.asarray(locs)
    fluxes = np.asarray(fluxes)
    S = locs.shape[-2]
    c = locs[..., axis]
    keep = present(counts, S)
    n_ax = locs.shape[axis]
    even = (np.arange(n_ax) % 2 == 0).reshape([n_ax if i == axis else 1 for i in range(c.ndim)])
    keep = keep & np.where(even, (c < dim) & (c != 0), c > 0)
    cnt, l, f = compact(keep, locs, fluxes)
    return cnt.astype(counts.dtype), l, f


def join(axis, data, counts, locs, fluxes, dim):
    """aggregate.py:217-263: tiles 2i and 2i+1 along `axis` become one tile of
    twice the size (data stacked along the axis), the second tile's sources
    shifted by `dim` (the child tile side) along the axis, the two catalogs
    concatenated and compacted to max(1, max count) slots.  Returns
    (data, counts, locs, fluxes)."""
    data = np.asarray(data)
    a0 = np.take(data, np.arange(0, data.shape[axis], 2), axis=axis)
    a1 = np.take(data, np.arange(1, data.shape[axis], 2), axis=axis)
    dat = np.concatenate([a0, a1], axis=2 + axis)
    c0 = np.take(counts, np.arange(0, counts.shape[axis], 2), axis=axis)
    c1 = np.take(counts, np.arange(1, counts.shape[axis], 2), axis=axis)
    l0 = np.take(locs, np.arange(0, locs.shape[axis], 2), axis=axis)
    l1 = np.take(locs, np.arange(1, locs.shape[axis], 2), axis=axis).copy()
    f0 = np.take(fluxes, np.arange(0, fluxes.shape[axis], 2), axis=axis)
    f1 = np.take(fluxes, np.arange(1, fluxes.shape[axis], 2), axis=axis)
    S = locs.shape[-2]
    p1 = present(c1, S)
    l1[..., axis] = np.where(p1, l1[..., axis] + dim, 0)
    keep = np.concatenate([present(c0, S), p1], axis=-1)
    ls = np.concatenate([l0, l1], axis=-2)
    fs = np.concatenate([f0, f1], axis=-1)
    cnt, ls, fs = compact(keep, ls, fs)
    smax = max(1, int(cnt.max()))
    return dat, cnt.astype(np.asarray(counts).dtype), ls[..., :smax, :], fs[..., :smax]


def unjoin(axis, data, counts, locs, fluxes, dim):
    """aggregate.py:265-324: a joint tile of side `dim` along `axis` back into
    its two halves; sources with coordinate <= dim/2 go to the first half,
    the others (shifted by -dim/2) to the second; each half compacted.  The
    child tiles are returned interleaved (2i, 2i+1) along the axis -- the
    reference concatenates them half-major (torch.cat(..., dim=axis)) and then
    pairs consecutive tiles (child_loglik.unfold(axis, 2, 2), :536-541), which
    pairs the wrong children whenever more than one joint tile lies along the
    axis (repaired here)."""
    data = np.asarray(data)
    half = dim // 2
    d0 = np.take(data, np.arange(0, half), axis=2 + axis)
    d1 = np.take(data, np.arange(half, dim), axis=2 + axis)
    S = locs.shape[-2]
    p = present(counts, S)
    c = locs[..., axis]
    m = c <= dim / 2
    k0, l0, f0 = compact(p & m, locs, fluxes)
    k1, l1, f1 = compact(p & ~m, locs, fluxes)
    l1 = l1.copy()
    l1[..., axis] = np.where(present(k1, S), l1[..., axis] - dim / 2, 0)

    def inter(x, y):
        st = np.stack([x, y], axis=axis + 1)
        sh = list(x.shape)
        sh[axis] *= 2
        return st.reshape(sh)
    return (inter(d0, d1), inter(k0, k1).astype(np.asarray(counts).dtype), inter(l0, l1),
            inter(f0, f1))


def child_model(model, axis):
    kw = dict(model.__dict__)
    kw.pop("norm_const", None)
    if axis == 0:
        kw["H"] = model.H // 2
    else:
        kw["W"] = model.W // 2
    return type(model)(**kw)


def parent_child_loglik(data, counts, locs, fluxes, model, axis, dtype=np.float64):
    """(l_p, l_c1 + l_c2) of joint tiles [nH,nW,H,W] (aggregate.py:536-541 with
    the children of each joint tile paired correctly)."""
    lp = loglikelihood(data, locs, fluxes, model, dtype)
    cd, cc, cl, cf = unjoin(axis, data, counts, locs, fluxes, model.H if axis == 0 else model.W)
    lc = loglikelihood(cd, cl, cf, child_model(model, axis), dtype)
    n = lc.shape[axis] // 2
    lc = np.take(lc, np.arange(0, 2 * n, 2), axis=axis) + np.take(lc, np.arange(1, 2 * n, 2),
                                                                  axis=axis)
    return lp, lc


def agg_log_target(data, counts, locs, fluxes, tau, prior, model, axis, dtype=np.float64):
    """aggregate.py:105-130: log p(z) + (1-tau) * sum_children l_c + tau * l_p."""
    lp, lc = parent_child_loglik(data, counts, locs, fluxes, model, axis, dtype)
    t = np.asarray(tau, dtype=dtype)[..., None]
    return log_prior(counts, locs, fluxes, prior, dtype) + (1 - t) * lc + t * lp


def agg_mh_sweep(data, counts, locs, fluxes, tau, prior, model, axis, mh, comp, uloc, uflux,
                 uacc, dtype=np.float64, trace=False):
    """Aggregate.mutate (aggregate.py:176-187) as SingleComponentMH.run
    (kernel.py:26-130) under agg_log_target, draws given explicitly (layout
    of smc_oracle.mh_sweep).  Repaired: the moved component is a present
    source (comp < count); the reference draws it from all max_objects slots
    (kernel.py:35-37), which turns an empty slot into an uncounted source.
    The upper-edge NaN freeze (kernel.py:125) is kept."""
    locs = np.array(locs, dtype=dtype)
    fluxes = np.array(fluxes, dtype=dtype)
    K = comp.shape[0]
    lb_l = np.asarray(prior.loc_low, dtype=dtype)
    ub_l = np.array(prior.loc_high, dtype=dtype)
    sl, sf = dtype(mh.locs_stdev), dtype(mh.fluxes_stdev)
    lb_f, ub_f = dtype(mh.fluxes_min), dtype(mh.fluxes_max)
    cur = agg_log_target(data, counts, locs, fluxes, tau, prior, model, axis, dtype)
    moving = np.asarray(counts) > 0
    acc_tr, loga_tr, accept = [], [], np.zeros(np.shape(counts), bool)
    for k in range(K):
        j = comp[k][..., None]
        lj = np.take_along_axis(locs, j[..., None].repeat(2, -1), axis=-2)[..., 0, :]
        fj = np.take_along_axis(fluxes, j, axis=-1)[..., 0]
        lnew = tn_sample(lj, sl, lb_l, ub_l, uloc[k].astype(dtype)).astype(np.float32).astype(dtype)
        fnew = tn_sample(fj, sf, lb_f, ub_f, uflux[k].astype(dtype)).astype(np.float32).astype(dtype)
        pl, pf = locs.copy(), fluxes.copy()
        np.put_along_axis(pl, j[..., None].repeat(2, -1), lnew[..., None, :], axis=-2)
        np.put_along_axis(pf, j, fnew[..., None], axis=-1)
        new = agg_log_target(data, counts, pl, pf, tau, prior, model, axis, dtype)
        q_num = tn_log_prob(lj, lnew, sl, lb_l, ub_l).sum(-1) + tn_log_prob(fj, fnew, sf, lb_f, ub_f)
        q_den = tn_log_prob(lnew, lj, sl, lb_l, ub_l).sum(-1) + tn_log_prob(fnew, fj, sf, lb_f, ub_f)
        loga = (new + q_num) - (cur + q_den)
        with np.errstate(over="ignore", invalid="ignore"):
            alpha = np.minimum(np.exp(loga), 1.0)
        accept = (uacc[k].astype(dtype) <= alpha) & moving
        locs = np.where(accept[..., None, None], pl, locs)
        fluxes = np.where(accept[..., None], pf, fluxes)
        with np.errstate(invalid="ignore"):
            cur = np.where(moving, new * accept + cur * (~accept), cur)
        acc_tr.append(accept)
        with np.errstate(invalid="ignore"):
            loga_tr.append(np.where(moving, loga - np.log(uacc[k].astype(dtype)), np.inf))
    if trace:
        # per iteration: accept flags and the decision margin log alpha - log U
        # (nan after an edge freeze; +inf for particles that never move)
        return (locs, fluxes, np.stack(acc_tr) if K else np.zeros((0,) + np.shape(counts), bool),
                np.stack(loga_tr) if K else np.zeros((0,) + np.shape(counts)))
    return locs, fluxes


def sort_by_count(counts, locs, fluxes):
    """aggregate.py:424-437: particles of each tile ordered by count (stable
    here), and the group sizes per tile."""
    order = np.argsort(counts, axis=-1, kind="stable")
    c = np.take_along_axis(counts, order, -1)
    l = np.take_along_axis(locs, order[..., None, None], 2)
    f = np.take_along_axis(fluxes, order[..., None], 2)
    groups = [[np.unique(c[h, w], return_counts=True)[1].tolist() for w in range(c.shape[1])]
              for h in range(c.shape[0])]
    return c, l, f, groups


def temper_groups(loglik_diff, groups, temperature, ess_prop, dtype=np.float64):
    """aggregate.py:140-174: per count group, delta solves ESS = ess_prop *
    group size (brentq xtol = rtol = 1e-6) or is 1 - tau; the tile's increment
    is the minimum over its groups.  Returns (tau_new, per-group deltas)."""
    temperature = np.asarray(temperature, np.float32)
    nH, nW = temperature.shape
    sol = np.zeros((nH, nW), np.float32)
    deltas = []
    for h in range(nH):
        for w in range(nW):
            top = 1 - float(temperature[h, w])
            splits = np.split(np.asarray(loglik_diff[h, w]), np.cumsum(groups[h][w])[:-1])
            ds = []
            for part in splits:
                thr = ess_prop * part.shape[0]

                def f(d, part=part, thr=thr):
                    return tempering_objective(part, d, thr, dtype)
                ds.append(np.float32(brentq(f, 0.0, top, xtol=1e-6, rtol=1e-6) if f(top) < 0
                                     else top))
            deltas.append(ds)
            sol[h, w] = min(ds)
    return (temperature + sol).astype(np.float32), deltas


def update_weights_groups(loglik_diff, groups, temperature, temperature_prev, lnc,
                          dtype=np.float64):
    """aggregate.py:439-483: softmax of (tau - tau_prev) * l within each count
    group; the group's log evidence += log mean exp; overall weights = within-
    group weights * softmax over the groups' log evidences.  lnc: per tile a
    list of group log evidences.  Returns (w_intra, weights, lnc_new)."""
    d = (np.asarray(temperature, np.float32) - np.asarray(temperature_prev, np.float32))
    lw = d.astype(dtype)[..., None] * np.asarray(loglik_diff, dtype)
    wi = np.zeros_like(lw)
    W = np.zeros_like(lw)
    out = []
    for h in range(lw.shape[0]):
        row = []
        for w in range(lw.shape[1]):
            cuts = np.cumsum(groups[h][w])[:-1]
            parts = np.split(lw[h, w], cuts)
            new = []
            wis = []
            for prev, p in zip(lnc[h][w], parts):
                m = p.max()
                e = np.exp(p - m)
                wis.append(e / e.sum())
                new.append(prev + np.log(e.mean()) + m)
            wi[h, w] = np.concatenate(wis)
            sm = np.exp(np.asarray(new) - np.max(new))
            sm = sm / sm.sum()
            W[h, w] = np.concatenate([x * s for x, s in zip(wis, sm)])
            row.append(new)
        out.append(row)
    return wi, W, out


def merge_log_evidence(lnc_children, joint_counts, axis):
    """Repaired aggregate.py:362-422.  After the children's particles are
    resampled by their weights and joined, the population is (approximately)
    distributed as the product of the children's posteriors, whose evidence
    is Z_c1 * Z_c2; joint count group j holds the fraction n_j / N of it.  So
    log Z_j = log Z_c1 + log Z_c2 + log(n_j / N), with log Z_c the log-sum-exp
    of a child's group evidences.  (The reference builds its per-group pmf
    from child counts that drop_sources_from_overlap has already overwritten
    in place, which gives log 0 -> nan_to_num -> -3.4e38 evidences.)
    lnc_children[h][w]: list of group log evidences of child tile (h, w);
    joint_counts [nH',nW',N] sorted by count.  Returns lnc[h'][w'] lists."""
    def lse(v):
        v = np.asarray(v, np.float64)
        m = v.max()
        return float(m + np.log(np.exp(v - m).sum()))
    nH, nW, N = joint_counts.shape
    out = []
    for h in range(nH):
        row = []
        for w in range(nW):
            if axis == 0:
                a, b = lnc_children[2 * h][w], lnc_children[2 * h + 1][w]
            else:
                a, b = lnc_children[h][2 * w], lnc_children[h][2 * w + 1]
            base = lse(a) + lse(b)
            _, n = np.unique(joint_counts[h, w], return_counts=True)
            row.append([base + float(np.log(k / N)) for k in n])
        out.append(row)
    return out


__all__ = ["M71Model", "BasicModel", "present", "compact", "drop_sources_from_overlap", "join",
           "unjoin", "child_model", "parent_child_loglik", "agg_log_target", "agg_mh_sweep",
           "sort_by_count", "temper_groups", "update_weights_groups", "merge_log_evidence"]
