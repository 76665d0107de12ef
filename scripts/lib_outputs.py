#!/usr/bin/env python
"""Outputs of fixed-seed MH sweeps (a C2-geometry 32x32 tile and a 2x2 grid of
8x8 M71 tiles, Philox draws) from the loaded library (SMCDET_HIP_LIB), saved
to an .npz -- for checking that two builds are bit-identical:

    python scripts/lib_outputs.py out_a.npz ; SMCDET_HIP_LIB=... python scripts/lib_outputs.py out_b.npz
    python scripts/lib_outputs.py --compare out_a.npz out_b.npz
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
    for k in a.files:
        print(k, "identical" if k not in bad else "DIFFERS", a[k].shape)
    sys.exit(1 if bad else 0)

import torch  # noqa: E402

from smcdet_amd._rng import PhiloxStream  # noqa: E402
from tests._params import p_m71_mh, p_m71_model, p_m71_prior  # noqa: E402

dev = torch.device("cuda", 0)
out = {}
for H, nt, N, tau in ((32, 1, 2048, 0.05), (8, 2, 2048, 0.3)):
    torch.manual_seed(5)
    truth = p_m71_prior(H * nt, 0, 40, counts_rate=0.004)
    _, l, f = truth.sample(num_catalogs=1, device=dev)
    img = p_m71_model(H * nt).sample(l, f)[0, 0, :, :, 0]
    img = img.reshape(nt, H, nt, H).permute(0, 2, 1, 3).contiguous()
    prior, model = p_m71_prior(H, 10, 10, counts_rate=0.003125), p_m71_model(H)
    torch.manual_seed(8)
    counts, locs, fluxes = prior.sample(num_tiles_per_side=nt, stratify_by_count=True,
                                        num_catalogs_per_count=N, device=dev)
    mh = p_m71_mh(100)
    mh.rng = PhiloxStream(17)
    lo, fo, acc = mh.run(img, counts, locs, fluxes, torch.full((nt, nt), tau, device=dev),
                         prior=prior, image_model=model)
    out[f"locs_{H}"] = lo.cpu().numpy()
    out[f"fluxes_{H}"] = fo.cpu().numpy()
    out[f"loglik_{H}"] = mh.last_loglik.cpu().numpy()
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1])
