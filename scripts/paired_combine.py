#!/usr/bin/env python
"""Pools the per-run results of the paired C2 replays run in parts
(tests/test_gpu_paired.py with SMCDET_PAIRED_ALL=1 SMCDET_PAIRED_PART=k/P,
one SMCDET_PAIRED_OUT JSON per part) into one summary over every oracle run
of the target, with the test's own statistics and gates: the pairing (ladders
equal for two iterations), the number of pairs in different log Z modes
against the frozen oracle-only rate DISCORDANCE (one-sided binomial), the
McNemar test of GPU-lower-only vs oracle-lower-only, and |delta log Z| over the
runs in the same mode.

    python scripts/paired_combine.py gpurun_out/r06_p*/paired_all.json > profiles/r06/paired_c2_all.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
from scipy.stats import binomtest  # noqa: E402

from tests.test_gpu_paired import DISCORDANCE, _compare  # noqa: E402


def main():
    runs = {}
    for path in sys.argv[1:]:
        for r in json.load(open(path))["runs"]:
            runs[r["seed"]] = r
    res = [runs[k] for k in sorted(runs)]
    lz = np.array([r["logZ"] for r in res])
    lz_o = np.array([r["oracle_logZ"] for r in res])
    cut = float(np.median(lz_o) - 40.0)
    gpu = _compare(lz, lz_o, cut)
    first = np.array([r["first_tau_divergence"] for r in res])
    disc = len(res) - gpu["same_mode"]
    out = {"n": len(res), "parts": len(sys.argv) - 1, "cut": cut, "gpu_vs_oracle": gpu,
           "discordant": disc, "discordance_rate": disc / len(res),
           "frozen_null_rate": DISCORDANCE,
           "binomial_p_greater": binomtest(disc, len(res), DISCORDANCE,
                                           alternative="greater").pvalue,
           "ladder_first_divergence": {"min": int(first.min()),
                                       "median": float(np.median(first)),
                                       "share_ge_2": float((first >= 2).mean())},
           "mean_dlogz_se": float((lz - lz_o).std(ddof=1) / np.sqrt(len(res)))}
    out["gates"] = {
        "pairing (share_ge_2 >= 0.9)": bool(out["ladder_first_divergence"]["share_ge_2"] >= 0.9),
        "discordance vs frozen null (binomial p > 0.001)": bool(out["binomial_p_greater"] > 0.001),
        "median |dlogZ| same mode <= 5": bool(gpu["abs_dlogz_median_same_mode"] <= 5.0),
        "McNemar p > 0.01": bool(gpu["mcnemar_p"] > 0.01)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
