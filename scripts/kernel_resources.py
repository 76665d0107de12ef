#!/usr/bin/env python
"""Static register / scratch / occupancy figures of every kernel the library
compiles (hipcc -Rpass-analysis=kernel-resource-usage on each source of the
Makefile's SRCS): VGPRs, spilled VGPRs / SGPRs, scratch bytes per lane,
occupancy.  MH sweep template order: <MODEL, REPLAY, FULL, PPL, PAIRED,
TAIL, GL, PC, RV, TB>.  --diag: the diagnostic build (-DSMCDET_DIAG).
    python scripts/kernel_resources.py > profiles/r06/kernel_resources.txt
    python scripts/kernel_resources.py --diag > profiles/r06/kernel_resources_diag.txt
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = ["common.hip", "model_kernels.hip", "mh_kernel.hip", "mala_kernel.hip",
        "chain_kernel.hip", "smc_kernels.hip", "agg_kernel.hip"]
args = [a for a in sys.argv[1:] if not a.startswith("--")]
diag = "--diag" in sys.argv
rows = []
for f in (args or SRCS):
    src = os.path.join(ROOT, "smcdet_amd", "csrc", f)
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
           "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/dev/null"]
    if diag:
        cmd.insert(1, "-DSMCDET_DIAG")
    r = subprocess.run(cmd, capture_output=True, text=True)
    cur = None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = subprocess.run(["c++filt"], input=m.group(1), capture_output=True,
                                  text=True).stdout.strip()
            cur = {"name": name, "file": f}
            rows.append(cur)
            continue
        m = re.search(r"(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"SGPRs Spill|VGPRs Spill): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
print(f"# {'diagnostic' if diag else 'product'} build: {len(rows)} kernels, "
      f"{sum(1 for c in rows if c.get('VGPRs Spill', 0))} with VGPR spills")
print(f"{'kernel':<96} VGPR  spillV spillS scratchB/lane waves/SIMD")
for c in rows:
    n = re.sub(r"\(.*\)$", "", c["name"].replace("void smcdet::", "").replace("smcdet::", ""))
    print(f"{n[:96]:<96} {c.get('VGPRs', 0):4d} {c.get('VGPRs Spill', 0):6d} "
          f"{c.get('SGPRs Spill', 0):6d} {c.get('ScratchSize [bytes/lane]', 0):13d} "
          f"{c.get('Occupancy [waves/SIMD]', 0):10d}")
