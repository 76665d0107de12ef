#!/usr/bin/env python
"""The C2 lower log Z mode by arithmetic class (VERDICT r4 "next" #2).

At the headline configuration (one 32x32 M71 tile, S=10, N=4096, K=100,
rho=0.5, systematic) a share of runs ends in a lower log Z mode ~65-80 nats
below the main one.  Sources compared (cut: log Z < -4310, as
scripts/logz_modes.py):
  * GPU: scripts/logz_modes.py runs (profiles/r04/logz_modes_2048*.jsonl:
    2048 independent runs per variant; float32 arithmetic);
  * oracle f64: tests/golden/stats_c2_moderate_4096_k100_oracle.json (the
    float64 restatement, make_oracle_stats.py);
  * oracle f32: ..._oracle_f32.json (the same seeds and streams in the
    reference's float32 arithmetic class);
  * reference: tests/golden/stats_c2_moderate_4096_k100.json (the reference's
    own float32 torch runs).
Two-proportion z tests of the GPU share against each CPU target, the paired
f32-vs-f64 comparison on common seeds (McNemar), and the means.

    python scripts/mode_share.py [--json profiles/r05/mode_share.json]
"""
import argparse
import json
import math
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")
CUT = -4310.0


def _runs(name):
    p = os.path.join(G, name)
    if not os.path.exists(p):
        return {}
    return {r["seed"]: r["logZ"] for r in json.load(open(p))["runs"]}


def two_prop(k1, n1, k2, n2):
    """Two-sided z test of equal proportions (pooled); exact-ish for the
    sizes here.  Returns (z, p)."""
    p = (k1 + k2) / (n1 + n2)
    se = math.sqrt(p * (1 - p) * (1 / n1 + 1 / n2)) if 0 < p < 1 else float("inf")
    z = (k1 / n1 - k2 / n2) / se if se > 0 else 0.0
    return z, math.erfc(abs(z) / math.sqrt(2))


def mcnemar(b, c):
    n, k = b + c, min(b, c)
    if n == 0:
        return 1.0
    return min(1.0, 2.0 * sum(math.comb(n, i) for i in range(k + 1)) / 2.0 ** n)


def summary(lz):
    a = np.asarray(list(lz), np.float64)
    return {"n": int(a.size), "lower": int((a < CUT).sum()), "share": float((a < CUT).mean()),
            "share_se": float(np.sqrt((a < CUT).mean() * (1 - (a < CUT).mean()) / a.size)),
            "mean": float(a.mean()), "se": float(a.std(ddof=1) / np.sqrt(a.size)),
            "median": float(np.median(a))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    gpu = {}
    for f, key in (("logz_modes_2048.jsonl", "default"),):
        for line in open(os.path.join(ROOT, "profiles", "r04", f)):
            d = json.loads(line)
            gpu[d["variant"] if key == "default" else key] = d
    f64, f32, ref = (_runs("stats_c2_moderate_4096_k100_oracle.json"),
                     _runs("stats_c2_moderate_4096_k100_oracle_f32.json"),
                     _runs("stats_c2_moderate_4096_k100.json"))
    out = {"cut": CUT, "targets": {"oracle_f64": summary(f64.values()),
                                   "oracle_f32": summary(f32.values()) if f32 else None,
                                   "reference": summary(ref.values())},
           "gpu": {v: {"n": d["n"], "lower": round(d["share_below_cut"] * d["n"]),
                       "share": d["share_below_cut"], "mean": d["logZ_mean"]}
                   for v, d in gpu.items() if d.get("cut") == CUT}}
    tests = {}
    for v, g in out["gpu"].items():
        for t, s in out["targets"].items():
            if s is None:
                continue
            z, p = two_prop(g["lower"], g["n"], s["lower"], s["n"])
            tests[f"gpu_{v}_vs_{t}"] = {"z": z, "p": p}
    if f32:
        common = sorted(set(f32) & set(f64))
        lo64 = np.array([f64[s] < CUT for s in common])
        lo32 = np.array([f32[s] < CUT for s in common])
        b, c = int((lo32 & ~lo64).sum()), int((~lo32 & lo64).sum())
        d = np.array([f32[s] - f64[s] for s in common])
        tests["paired_f32_vs_f64"] = {
            "n": len(common), "same_mode": int((lo32 == lo64).sum()), "lower_f32_only": b,
            "lower_f64_only": c, "mcnemar_p": mcnemar(b, c),
            "mean_dlogz": float(d.mean()), "se_dlogz": float(d.std(ddof=1) / np.sqrt(d.size))
            if d.size > 1 else None}
        z, p = two_prop(int(lo32.sum()), len(common), int(lo64.sum()), len(common))
        tests["f32_vs_f64_unpaired"] = {"z": z, "p": p}
    out["tests"] = tests
    print(json.dumps(out, indent=1))
    if a.json:
        os.makedirs(os.path.dirname(os.path.abspath(a.json)), exist_ok=True)
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
