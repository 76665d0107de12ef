#!/usr/bin/env python
"""Summarises the rocprofv3 passes of scripts/profile.sh for one kernel into
the JSON bench.py reads (profiles/pmc_mh_r03.json):

* per-dispatch averages of every PMC counter (instances summed per dispatch;
  the first `--skip` dispatches are warm-up and excluded);
* per particle-step figures (`--steps-per-launch`);
* HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (KB units;
  FETCH_SIZE x 2 is the gfx950 correction of MI355X_MICROARCH.md's HBM
  section);
* the effective clock of the profiled launches: GRBM_GUI_ACTIVE (summed over
  the 8 XCDs) / 8 / the dispatch's duration from the same pass's kernel trace
  (MI355X_MICROARCH.md, "DVFS give-back");
* the kernel's average duration in the trace pass;
* source_hash: the sha1 of the library sources (smcdet_amd._hip.source_hash)
  the counters were measured on -- bench.py ignores a summary whose hash is
  not the loaded library's.
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--root", default="gpurun_out/prof")
ap.add_argument("--kernel", default="mh_sweep_kernel")
ap.add_argument("--skip", type=int, default=2)
ap.add_argument("--steps-per-launch", type=float, default=4096 * 100)
ap.add_argument("--json", default=None)
ap.add_argument("--note", default="")
a = ap.parse_args()


def kernel_durations(d):
    """{dispatch id: duration ns} of the kernel in <d>/run_kernel_trace.csv."""
    out = {}
    for f in glob.glob(f"{d}/**/run_kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if a.kernel in r["Kernel_Name"]:
                out[int(r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return out


vals = defaultdict(list)
clock = []
trace_ms = None
for d in sorted(glob.glob(f"{a.root}/*")):
    if not os.path.isdir(d):
        continue
    per = defaultdict(float)
    for f in glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if a.kernel not in r["Kernel_Name"]:
                continue
            per[(r["Counter_Name"], int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
    byname = defaultdict(list)
    for (name, did), v in sorted(per.items(), key=lambda kv: kv[0][1]):
        byname[name].append((did, v))
    dur = kernel_durations(d)
    for name, v in byname.items():
        v = v[a.skip:] if len(v) > a.skip else v
        vals[name] += [x for _, x in v]
        if name == "GRBM_GUI_ACTIVE" and dur:
            for did, cyc in v:
                if did in dur:
                    clock.append((cyc / 8.0, dur[did]))
    if not byname and dur:  # the kernel-trace pass
        ds = sorted(dur.items())[a.skip:]
        trace_ms = sum(x for _, x in ds) / max(len(ds), 1) / 1e6

per_dispatch = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
per_step = {k: v / a.steps_per_launch for k, v in per_dispatch.items()}
if "SQ_INSTS_VALU_FLOPS_FP32" in per_step:
    per_step["fp32_flop"] = per_step["SQ_INSTS_VALU_FLOPS_FP32"] + \
        per_step.get("SQ_INSTS_VALU_FLOPS_FP32_TRANS", 0.0)
out = {"kernel": a.kernel, "particle_steps_per_launch": a.steps_per_launch,
       "per_dispatch": per_dispatch, "per_particle_step": per_step,
       "kernel_ms_trace_pass": trace_ms}
if "FETCH_SIZE" in per_dispatch and "WRITE_SIZE" in per_dispatch:
    out["hbm_bytes_per_launch"] = (2 * per_dispatch["FETCH_SIZE"] + per_dispatch["WRITE_SIZE"]) * 1024
if clock:
    cyc = sum(c for c, _ in clock) / len(clock)
    ns = sum(t for _, t in clock) / len(clock)
    out["effective_clock"] = {
        "ghz": cyc / ns, "cycles_per_xcd": cyc, "launch_ms": ns / 1e6, "dispatches": len(clock),
        "note": "GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration, same rocprofv3 pass "
                "(--pmc GRBM_GUI_ACTIVE --kernel-trace); profiled passes run a few % below "
                "the un-profiled clock (MI355X_MICROARCH.md DVFS give-back (2))"}
try:
    from smcdet_amd import _hip
    out["source_hash"] = _hip.source_hash()
except Exception as e:  # noqa: BLE001
    out["source_hash"] = None
    out["source_hash_error"] = repr(e)
out["note"] = a.note or ("rocprofv3 passes of scripts/profile.sh over bench.py C2 --no-c3; "
                         "counters summed over XCC/SE instances per dispatch; warm-up "
                         "dispatches excluded")
for k, v in per_dispatch.items():
    print(f"{k:36s} {v:18.1f} {per_step[k]:12.4f}/step")
if clock:
    print("effective clock %.3f GHz over %d dispatches" % (out["effective_clock"]["ghz"], len(clock)))
if a.json:
    json.dump(out, open(a.json, "w"), indent=1)
    print("wrote", a.json)
