#!/usr/bin/env python
"""Averages rocprofv3 PMC counters per dispatch of one kernel (last
`--skip` warm-up dispatches excluded) from gpurun_out/prof/*/run_counter_collection.csv."""
import argparse
import csv
import glob
import json
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("--root", default="gpurun_out/prof")
ap.add_argument("--kernel", default="mh_sweep_kernel")
ap.add_argument("--skip", type=int, default=2)
ap.add_argument("--json", default=None)
a = ap.parse_args()
vals = defaultdict(list)
grid = None
for f in sorted(glob.glob(f"{a.root}/*/run_counter_collection.csv")):
    per = defaultdict(list)
    for r in csv.DictReader(open(f)):
        if a.kernel not in r["Kernel_Name"]:
            continue
        per[(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
        grid = int(r["Grid_Size"])
    byname = defaultdict(list)
    for (name, did), v in sorted(per.items(), key=lambda kv: int(kv[0][1])):
        byname[name].append(sum(v))
    for name, v in byname.items():
        vals[name] = v[a.skip:] if len(v) > a.skip else v
out = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
for k, v in out.items():
    print(f"{k:36s} {v:16.1f}")
if a.json:
    json.dump({"kernel": a.kernel, "grid": grid, "per_dispatch": out}, open(a.json, "w"), indent=1)
