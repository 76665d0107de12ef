#!/usr/bin/env python
"""Static register / scratch / occupancy figures of every MH sweep
instantiation (hipcc -Rpass-analysis=kernel-resource-usage on
smcdet_amd/csrc/mh_kernel.hip): VGPRs, spilled VGPRs / SGPRs, scratch bytes
per lane, occupancy.  Template order: <MODEL, REPLAY, FULL, PPL, PAIRED,
TAIL, GL, PC, RV, TB>.
    python scripts/kernel_resources.py > profiles/r05/kernel_resources.txt
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(ROOT, "smcdet_amd", "csrc", sys.argv[1] if len(sys.argv) > 1 else "mh_kernel.hip")
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                    "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/dev/null"],
                   capture_output=True, text=True)
rows, cur = [], None
for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = subprocess.run(["c++filt"], input=m.group(1), capture_output=True,
                              text=True).stdout.strip()
        cur = {"name": name}
        rows.append(cur)
        continue
    m = re.search(r"(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs Spill|"
                  r"VGPRs Spill): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1)] = int(m.group(2))
print(f"{'kernel':<90} VGPR  spillV spillS scratchB/lane waves/SIMD")
for c in rows:
    n = c["name"].replace("void smcdet::", "").replace("(smcdet::MhArgs)", "")
    print(f"{n:<90} {c.get('VGPRs', 0):4d} {c.get('VGPRs Spill', 0):6d} {c.get('SGPRs Spill', 0):6d} "
          f"{c.get('ScratchSize [bytes/lane]', 0):13d} {c.get('Occupancy [waves/SIMD]', 0):10d}")
