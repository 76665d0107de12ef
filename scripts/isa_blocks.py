#!/usr/bin/env python
"""Per-basic-block instruction statistics of one MH-sweep instantiation
(VALU, transcendental, packed, SALU, readlane, LDS, scratch counts and the
branches out of each block), from the gfx950 assembly of
smcdet_amd/csrc/mh_kernel.hip -- how DESIGN.md §4.1 attributes the VALU
instructions per iteration.

    python scripts/isa_blocks.py [source.hip] [instantiation substring]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "smcdet_amd/csrc/mh_kernel.hip")
kern = sys.argv[2] if len(sys.argv) > 2 else "Li1ELb0ELb0ELi16ELb1"  # M71, Philox, incremental, 32x32
out = "/tmp/smcdet_isa_blocks.s"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                "--cuda-device-only", "-S", src, "-o", out], check=True,
               stderr=subprocess.DEVNULL)
s = open(out).read()
name = [m for m in re.findall(r"^(_ZN6smcdet15mh_sweep_kernel\w+):", s, re.M) if kern in m][0]
i = s.index(name + ":")
j = s.index(".Lfunc_end", i)
blocks, cur = [], None
for ln in s[i:j].split("\n"):
    m = re.match(r"^(\.LBB\w+):", ln)
    if m:
        cur = {"name": m.group(1), "ins": []}
        blocks.append(cur)
        continue
    if ln.startswith("\t") and not ln.startswith("\t.") and not ln.startswith("\t;") and cur:
        cur["ins"].append(ln.strip())
for b in blocks:
    ins = b["ins"]
    cnt = lambda f: sum(1 for t in ins if f(t))  # noqa: E731
    print(f"{b['name']:14s} n={len(ins):4d} valu={cnt(lambda t: t.startswith('v_')):4d} "
          f"trans={cnt(lambda t: re.match(r'v_(exp|log|rcp|sqrt|rsq)_f32', t)):3d} "
          f"pk={cnt(lambda t: t.startswith('v_pk_')):3d} "
          f"salu={cnt(lambda t: t.startswith('s_') and 'branch' not in t and 'waitcnt' not in t and 'nop' not in t):3d} "
          f"rl={cnt(lambda t: t.startswith('v_readlane') or t.startswith('v_readfirstlane')):2d} "
          f"ds={cnt(lambda t: t.startswith('ds_')):2d} scr={cnt(lambda t: t.startswith('scratch_'))} | "
          + " ; ".join(t for t in ins if "branch" in t))
