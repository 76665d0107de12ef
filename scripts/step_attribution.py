#!/usr/bin/env python
"""Attributes the C2 SMC step from a rocprofv3 --kernel-trace CSV of bench.py
(VERDICT r2 next #5): per step (MH sweep launch -> tile kernel launch -> the
next sweep) the sweep's duration, the idle gap before the tile kernel, the
tile kernel's duration and the idle gap before the next sweep; the launch
ordinal range selects the timed region (after `--skip` warm-up steps).

    python scripts/step_attribution.py <run_kernel_trace.csv> [--skip 3] [--steps 20]
"""
import argparse
import csv
import json

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--skip", type=int, default=3)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--sweep", default="mh_sweep_kernel")
ap.add_argument("--tile", default="tile_kernel")
ap.add_argument("--json", default=None)
# the last N clean steps instead of --skip/--steps (a trace whose timed
# region is its end, e.g. bench.py with the prewarm and no untimed tail)
ap.add_argument("--tail", type=int, default=0)
a = ap.parse_args()

rows = [r for r in csv.DictReader(open(a.trace))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ev = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
sweeps = [i for i, e in enumerate(ev) if a.sweep in e[0]]
steps = []
for n, i in enumerate(sweeps[:-1]):
    j = sweeps[n + 1]
    tiles = [k for k in range(i + 1, j) if a.tile in ev[k][0]]
    if len(tiles) != 1 or j != tiles[0] + 1:
        continue  # not a clean sweep -> tile -> sweep step
    t = tiles[0]
    s0, e0 = ev[i][1], ev[i][2]
    s1, e1 = ev[t][1], ev[t][2]
    steps.append(dict(sweep_us=(e0 - s0) / 1e3, gap_sweep_tile_us=(s1 - e0) / 1e3,
                      tile_us=(e1 - s1) / 1e3, gap_tile_sweep_us=(ev[j][1] - e1) / 1e3,
                      step_us=(ev[j][1] - s0) / 1e3))
sel = steps[-a.tail:] if a.tail > 0 else steps[a.skip:a.skip + a.steps]
out = {"steps": len(sel), "source": a.trace}
for k in sel[0]:
    v = np.array([s[k] for s in sel])
    out[k] = {"mean": float(v.mean()), "median": float(np.median(v)), "min": float(v.min()),
              "max": float(v.max())}
for k, v in out.items():
    print(k, v)
if a.json:
    json.dump(out, open(a.json, "w"), indent=1)
