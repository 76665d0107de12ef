#!/usr/bin/env python
"""Launch-gap probe (run under `rocprofv3 --kernel-trace`): back-to-back MH
sweeps at the C2 geometry with and without persisted rate images
(rate_out: 16.8 MB of dirty lines per launch), and a small torch kernel
sequence as the baseline gap.  scripts/gap_summary.py reads the trace."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from tests._params import p_m71_mh, p_m71_model, p_m71_prior  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    H, S, N = 32, 10, 4096
    model, prior = p_m71_model(H), p_m71_prior(H, S, S, counts_rate=0.003125)
    truth = p_m71_prior(H, 0, 100, counts_rate=0.003125)
    c, l, f = truth.sample(num_catalogs=1, device=dev)
    img = model.sample(l, f)[0, 0, :, :, 0].reshape(1, 1, H, H).contiguous()
    counts, locs, fluxes = prior.sample(num_tiles_per_side=1, stratify_by_count=True,
                                        num_catalogs_per_count=N, device=dev)
    tau = torch.full((1, 1), 0.3, device=dev)
    mh = p_m71_mh(100)
    r = [torch.empty(1, 1, N, H * H, device=dev) for _ in range(2)]
    # rate_in must be the images of the state: the first sweep renders them
    locs, fluxes, _ = mh.run(img, counts, locs, fluxes, tau, prior=prior, image_model=model,
                             rate_out=r[0])
    torch.cuda.synchronize()
    x = torch.zeros(1024, device=dev)
    for _ in range(reps):  # baseline: tiny torch kernels
        x.add_(1.0)
    torch.cuda.synchronize()
    cur = 0
    for _ in range(reps):  # persisted rate images (the sampler's default)
        locs, fluxes, _ = mh.run(img, counts, locs, fluxes, tau, prior=prior, image_model=model,
                                 rate_in=r[cur], rate_out=r[1 - cur])
        cur = 1 - cur
    torch.cuda.synchronize()
    x.mul_(1.0)  # marker between the two sequences
    torch.cuda.synchronize()
    for _ in range(reps):  # no rate images (initial render, nothing persisted)
        locs, fluxes, _ = mh.run(img, counts, locs, fluxes, tau, prior=prior, image_model=model)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
