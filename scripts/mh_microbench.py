#!/usr/bin/env python
"""Interleaved A/B timing of MH-sweep variants at the C2 geometry (one
process, rounds interleaved; reports median and min ms per launch).

Variants: incremental (default), the diagnostic ablations
(SMCDET_MH_ABLATE_LIKELIHOOD / _PROPOSAL: timing only), full recompute, and
the per-tile temper+reweight+resample launch."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from smcdet_amd import _hip  # noqa: E402
from tests._params import p_m71_mh, p_m71_model, p_m71_prior  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--particles", type=int, default=4096)
    ap.add_argument("--tiles", type=int, default=1)
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--sources", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--full", action="store_true", help="include the full-recompute variant")
    ap.add_argument("--only", default=None, help="run just this variant (for rocprofv3 --pmc)")
    ap.add_argument("--variants", default=None,
                    help="comma-separated subset of the variants, interleaved (A/B)")
    ap.add_argument("--no-extra", action="store_true", help="skip the tile/loglik kernel timings")
    ap.add_argument("--block-slots", default=None,
                    help="comma-separated SMCDET_MH_BLOCK_SLOTS values, one variant each")
    ap.add_argument("--tau", type=float, default=0.3)
    # library-independent inputs (torch CPU generator + the c2_moderate fixture
    # image), so that libraries whose prior/noise kernels draw different
    # streams still time the MH sweep on identical states (scripts/ab_kernel.sh)
    ap.add_argument("--state", choices=["torch", "device"], default="torch")
    ap.add_argument("--warm", type=int, default=3, help="MH sweeps before timing (torch state)")
    # start every sweep from persisted rate images (as SMCsampler does) instead
    # of an initial render of all sources
    ap.add_argument("--persist", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    H, S, Np = a.tile, a.sources, a.particles
    nt = int(round(a.tiles ** 0.5))
    model, prior = p_m71_model(H), p_m71_prior(H, S, S, counts_rate=0.003125)
    if a.state == "torch":
        from tests._params import GOLDEN, M71
        ref = json.load(open(os.path.join(GOLDEN, "stats_c2_moderate.json")))
        assert H == 32, "--state torch uses the 32x32 fixture image"
        img = torch.tensor(ref["image"], dtype=torch.float32).reshape(1, 1, H, H)
        img = img.expand(nt, nt, H, H).contiguous().to(dev)
        g = torch.Generator().manual_seed(1)
        counts = torch.full((nt, nt, Np), float(S), device=dev)
        locs = (torch.rand(nt, nt, Np, S, 2, generator=g) * (H + 8) - 4).to(dev)
        al, lo, hi = M71["flux_alpha"], M71["flux_lower"], M71["flux_upper"]
        u = torch.rand(nt, nt, Np, S, generator=g, dtype=torch.float64)
        fl = ((hi ** al - u * hi ** al + u * lo ** al) / (lo ** al * hi ** al)) ** (-1 / al)
        fluxes = fl.float().clamp(lo, hi).to(dev)
    else:
        truth = p_m71_prior(H, 0, 100, counts_rate=0.003125)
        img = torch.empty(nt, nt, H, H, device=dev)
        for i in range(nt):
            for j in range(nt):
                while True:
                    c, l, f = truth.sample(num_catalogs=1, device=dev)
                    if int(c.max()) <= S:
                        break
                img[i, j] = model.sample(l, f)[0, 0, :, :, 0]
        counts, locs, fluxes = prior.sample(num_tiles_per_side=nt, stratify_by_count=True,
                                            num_catalogs_per_count=Np, device=dev)
    tau = torch.full((nt, nt), a.tau, device=dev)
    if a.state == "torch" and a.warm:
        from smcdet_amd._rng import PhiloxStream
        mw = p_m71_mh(a.K)
        mw.rng = PhiloxStream(123)
        for _ in range(a.warm):
            locs, fluxes, _ = mw.run(img, counts, locs, fluxes, tau, prior=prior, image_model=model)
    variants = {"incremental": (False, 0),
                "no_likelihood": (False, _hip.SMCDET_MH_ABLATE_LIKELIHOOD if hasattr(
                    _hip, "SMCDET_MH_ABLATE_LIKELIHOOD") else 256),
                "no_proposal": (False, 512),
                "no_both": (False, 768),
                "scalar_slots": (False, 1024),
                "no_block": (False, 16384)}
    if a.full:
        variants["full_recompute"] = (True, 0)
    for kk in (0, 1, 25, 200):
        variants[f"K={kk}"] = (False, 0, kk)
    if a.only:
        variants = {a.only: variants[a.only]}
    # block-form thresholds (SMCDET_MH_BLOCK_SLOTS, read at every launch):
    # variant "blk<n>" = the default form with that threshold (0 = off)
    envs = {}
    for n in (a.block_slots.split(",") if a.block_slots else []):
        variants[f"blk{n}"] = (False, 0)
        envs[f"blk{n}"] = n
    if a.variants:
        variants = {k: variants[k] for k in a.variants.split(",")}
    times = {k: [] for k in variants}
    mhs = {}
    for k, v in variants.items():
        full, fl = v[0], v[1]
        mh = p_m71_mh(v[2] if len(v) > 2 else a.K, full_recompute=full)
        mh.debug_flags = fl
        mhs[k] = mh
    ll = model.loglikelihood(img, locs, fluxes)
    REP = 5  # back-to-back launches per timing: host launch overhead overlaps GPU work

    def timeit(fn):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(REP):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / REP

    T = nt * nt
    t_ = torch.zeros(T, device=dev)
    tp, lw, W = torch.empty(T, device=dev), torch.empty_like(ll), torch.empty_like(ll)
    ess, lz = torch.empty(T, device=dev), torch.zeros(T, device=dev)
    idx = torch.empty(ll.shape, device=dev, dtype=torch.int64)
    mh0 = p_m71_mh(0)
    ll64 = ll[..., :64].contiguous()
    extra = {
        "loglik_kernel": lambda: model.loglikelihood(img, locs, fluxes),
        "K=0,no_loglik_out": lambda: mh0.run(img, counts, locs, fluxes, tau, prior=prior,
                                             image_model=model, want_loglik=False),
        "tile_kernel": lambda: _hip.check(_hip.lib().smcdet_temper_reweight(
            _hip.ptr(ll), _hip.ptr(torch.zeros(T, device=dev)), _hip.ptr(tp), _hip.ptr(lw),
            _hip.ptr(W), _hip.ptr(ess), _hip.ptr(lz), T, Np, 0.5 * Np, 1, 1, 0, _hip.ptr(idx),
            0, None, 0, None, None, None, _hip.stream_of(ll)), "tr"),
        "temper_only": lambda: _hip.check(_hip.lib().smcdet_temper(
            _hip.ptr(ll), _hip.ptr(torch.zeros(T, device=dev)), _hip.ptr(tp), T, Np, 0.5 * Np,
            _hip.stream_of(ll)), "t"),
        "temper_only_N64": lambda: _hip.check(_hip.lib().smcdet_temper(
            _hip.ptr(ll64), _hip.ptr(torch.zeros(T, device=dev)), _hip.ptr(tp), T, 64, 32.0,
            _hip.stream_of(ll)), "t64"),
        "weights_only": lambda: _hip.check(_hip.lib().smcdet_update_weights(
            _hip.ptr(ll), _hip.ptr(t_), _hip.ptr(tp), _hip.ptr(lw), _hip.ptr(W), _hip.ptr(ess),
            _hip.ptr(lz), T, Np, _hip.stream_of(ll)), "w"),
        "resample_only": lambda: _hip.check(_hip.lib().smcdet_resample_index(
            _hip.ptr(W), T, Np, 1, 1, 0, None, _hip.ptr(idx), _hip.stream_of(ll)), "r"),
    }
    if a.no_extra:
        extra = {}
    rates = {}
    if a.persist:
        # rate images of (locs, fluxes); every timed sweep reads them (and
        # writes a second buffer) without moving the state it started from
        r_in = torch.empty(nt, nt, Np, H * H, device=dev)
        r_out = torch.empty_like(r_in)
        p_m71_mh(0).run(img, counts, locs, fluxes, tau, prior=prior, image_model=model,
                        rate_out=r_in)
        rates = {"rate_in": r_in, "rate_out": r_out}
    for r in range(a.rounds + 1):
        for k, mh in mhs.items():
            if k in envs:
                os.environ["SMCDET_MH_BLOCK_SLOTS"] = envs[k]
            else:
                os.environ.pop("SMCDET_MH_BLOCK_SLOTS", None)
            v = timeit(lambda: mh.run(img, counts, locs, fluxes, tau, prior=prior,
                                      image_model=model, **rates))
            if r:
                times[k].append(v)
        for k, fn in extra.items():
            v = timeit(fn)
            if r:
                times.setdefault(k, []).append(v)
    out = {k: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v))}
           for k, v in times.items()}
    steps = nt * nt * Np * a.K
    for k, v in out.items():
        if k in variants and not k.startswith("K="):
            v["particle_steps_per_s"] = steps / (v["median_ms"] * 1e-3)
    print(json.dumps({"config": vars(a), "variants": out}, indent=1))


if __name__ == "__main__":
    main()
