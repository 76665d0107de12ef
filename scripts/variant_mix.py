#!/usr/bin/env python
"""Which union-window path the C2 MH steps take: the bench's
C2 sampler is stepped, and at a few SMC iterations every (particle, source)
pair's window box (clipped to the tile) and its chance of a moved anchor
(proposal sd 0.1 px: P(floor h or floor w changes)) give the expected share of
same-anchor steps by union-window slot count, and of moved-anchor steps."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
from scipy.stats import norm  # noqa: E402

import bench  # noqa: E402

sys.argv = [sys.argv[0]]
a = bench.parse()
dev = torch.device("cuda", 0)
s, mh, _, _, _ = bench.build_sampler(a, dev, 0)
s.initialize()
s._temper_reweight(with_resample=True)
H = W = a.tile
R, sd = 8, 0.1
out = {}
for it in range(1, 31):
    idx, s._pending_idx = s._pending_idx, None
    s._step(idx)
    if it in (1, 5, 10, 15, 20, 25, 30):
        torch.cuda.synchronize()
        L = s.locs.reshape(-1, a.sources, 2).cpu().numpy().astype(np.float64)
        fh, fw = np.floor(L[..., 0]), np.floor(L[..., 1])
        ru = np.minimum(fh + R, H - 1) - np.maximum(fh - R, 0) + 1
        cu = np.minimum(fw + R, W - 1) - np.maximum(fw - R, 0) + 1
        npos = np.clip(ru, 0, None) * np.clip(cu, 0, None)
        slots = np.ceil(npos / 64).astype(int)
        fr_h, fr_w = L[..., 0] - fh, L[..., 1] - fw
        stay = ((norm.cdf((1 - fr_h) / sd) - norm.cdf(-fr_h / sd))
                * (norm.cdf((1 - fr_w) / sd) - norm.cdf(-fr_w / sd)))
        block = (slots >= 5) & (ru >= 16) & (cu >= 16)
        row = {"temperature": float(s.temperature.min()),
               "moved_anchor": float(1 - stay.mean()),
               "same_block": float((stay * block).mean())}
        for k in range(0, 7):
            row[f"same_{k}slot"] = float((stay * (slots == k) * ~block).mean())
        out[it] = row
        print(it, json.dumps({k: round(v, 3) for k, v in row.items()}), flush=True)
json.dump(out, open(os.environ.get("VARIANT_MIX_OUT", "/tmp/variant_mix.json"), "w"), indent=1)
