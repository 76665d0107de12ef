#!/usr/bin/env python
"""C5 count-stratified evidence: GPU vs the oracle target vs the reference.

Per count s the log Z_s of independent runs (tests/golden/stats_c5_oracle.json,
stats_c5.json, and the GPU runs test_c5_statistical_vs_oracle writes with
SMCDET_C5_STATS_OUT): mean, SD, quantiles; and p(s|x) two ways -- the mean of
the per-run posteriors (what the tests compare), and the probability that
count s wins (argmax of log p(s) + log Z_s) when each stratum's log Z is an
independent draw from its own runs (the strata of a CS-SMC run are
independent samplers, manuscript.tex:322-356), by Monte Carlo over the
pooled per-count samples.  The second form uses every run of every count, so
it resolves the posterior far better than the per-run mean of a few runs.

    python scripts/c5_analysis.py [gpu_c5_stats.json] [--json out.json]
"""
import argparse
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")


def per_count(lz):
    lz = np.asarray(lz, np.float64)
    return [{"mean": float(c.mean()), "sd": float(c.std(ddof=1)) if c.size > 1 else None,
             "se": float(c.std(ddof=1) / np.sqrt(c.size)) if c.size > 1 else None,
             "q": np.percentile(c, [0, 10, 50, 90, 100]).round(2).tolist()} for c in lz.T]


def win_probs(lz, log_ps, draws=200000, seed=0):
    lz = np.asarray(lz, np.float64)
    rng = np.random.default_rng(seed)
    n, k = lz.shape
    pick = rng.integers(0, n, size=(draws, k))
    v = lz[pick, np.arange(k)] + np.asarray(log_ps)
    w = np.bincount(v.argmax(1), minlength=k) / draws
    return w.round(4).tolist()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("gpu", nargs="?", default=None)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    ref = json.load(open(os.path.join(G, "stats_c5.json")))
    orc = json.load(open(os.path.join(G, "stats_c5_oracle.json")))
    log_ps = ref["config"]["log_count_prior"]
    srcs = {"reference": ([r["logZ"] for r in ref["runs"]],
                          [r["count_posterior"] for r in ref["runs"]]),
            "oracle": ([r["logZ"] for r in orc["runs"]],
                       [r["count_posterior"] for r in orc["runs"]])}
    if a.gpu:
        g = json.load(open(a.gpu))
        srcs["gpu"] = (g["logZ"], g["count_posterior"])
    out = {}
    for k, (lz, post) in srcs.items():
        out[k] = {"runs": len(lz), "per_count": per_count(lz),
                  "posterior_mean": np.mean(post, 0).round(4).tolist(),
                  "win_prob_independent_strata": win_probs(lz, log_ps)}
    for k, v in out.items():
        print(k, v["runs"], "runs")
        for s, c in enumerate(v["per_count"]):
            print(f"  count {s}: mean {c['mean']:.2f} sd {c['sd'] or 0:.2f} q {c['q']}")
        print("  p(s|x) mean of runs   ", v["posterior_mean"])
        print("  p(s|x) strata-resampled", v["win_prob_independent_strata"])
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
