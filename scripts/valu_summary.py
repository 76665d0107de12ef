#!/usr/bin/env python
"""Per-launch VALU counts of the MH sweep from a rocprofv3 PMC pass
(scripts/profile.sh SQ=...), normalised per particle-step, for bench.py's
`compute.executed` block (profiles/pmc_valu_mh_<round>.json).

    python scripts/valu_summary.py --root gpurun_out/prof --steps 409600 \
        --json profiles/pmc_valu_mh_r02.json
"""
import argparse
import csv
import glob
import json
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("--root", default="gpurun_out/prof")
ap.add_argument("--kernel", default="mh_sweep_kernel")
ap.add_argument("--skip", type=int, default=2, help="warm-up dispatches excluded")
ap.add_argument("--steps", type=float, required=True, help="particle-steps per launch (N*K*T)")
ap.add_argument("--json", default=None)
a = ap.parse_args()
vals = defaultdict(list)
for f in sorted(glob.glob(f"{a.root}/*/run_counter_collection.csv")):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if a.kernel not in r["Kernel_Name"]:
            continue
        per[(r["Counter_Name"], int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
    byname = defaultdict(list)
    for (name, did), v in sorted(per.items(), key=lambda kv: kv[0][1]):
        byname[name].append(v)
    for name, v in byname.items():
        vals[name] = v[a.skip:] if len(v) > a.skip else v
disp = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
ps = {k: v / a.steps for k, v in disp.items()}
flop = ps.get("SQ_INSTS_VALU_FLOPS_FP32", 0.0) + ps.get("SQ_INSTS_VALU_FLOPS_FP32_TRANS", 0.0)
ps["fp32_flop"] = flop
for k, v in disp.items():
    print(f"{k:36s} per launch {v:16.1f}  per particle-step {ps[k]:12.3f}")
print(f"{'fp32_flop (FLOPS_FP32 + _TRANS)':36s} per particle-step {flop:12.3f}")
if a.json:
    json.dump({"kernel": a.kernel, "particle_steps_per_launch": a.steps,
               "per_dispatch": disp, "per_particle_step": ps,
               "note": "rocprofv3 --pmc pass over bench.py (C2); SQ counters summed over "
                       "XCC/SE instances per dispatch; warm-up dispatches excluded"},
              open(a.json, "w"), indent=1)
