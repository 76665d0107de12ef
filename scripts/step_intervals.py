#!/usr/bin/env python
"""Per-kernel mean duration and the mean start-to-start interval of the MH
sweep launches (= the GPU's time per SMC step) over the last N sweep launches
of a rocprofv3 --kernel-trace CSV:
    python scripts/step_intervals.py <run_kernel_trace.csv> [N]"""
import csv
import sys
from collections import defaultdict


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    mh = [r for r in rows if "mh_sweep_kernel" in r["Kernel_Name"]][-(n + 1):]
    t0, t1 = int(mh[0]["Start_Timestamp"]), int(mh[-1]["Start_Timestamp"])
    window = [r for r in rows if t0 <= int(r["Start_Timestamp"]) < t1]
    dur = defaultdict(list)
    for r in window:
        dur[r["Kernel_Name"].split("(")[0][-40:]].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"step (sweep start to start) {(t1 - t0) / 1e3 / (len(mh) - 1):.2f} us over {len(mh) - 1}")
    for k, v in dur.items():
        print(f"  {k:40s} n={len(v):3d} mean {sum(v) / len(v):8.2f} us")


if __name__ == "__main__":
    main()
