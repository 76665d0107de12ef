"""The reference's MCMC baseline driver (experiments/m71/run_mcmc.py) for a
batch of synthetic 8x8 M71 cutouts: one MHsampler chain per cutout, all
cutouts in one launch (MHsampler.from_tiles), results written in the
driver's per-batch file layout.

    python examples/mcmc_m71_cutouts.py [num_cutouts] [out_dir]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from smcdet_amd.images import M71ImageModel
from smcdet_amd.prior import M71Prior
from smcdet_amd.sampler import MHsampler

P = dict(flux_alpha=0.21411753249015655, flux_lower=0.06291294097900389,
         flux_upper=1804.6791992187502, flux_detection_threshold=0.25165176391601557,
         counts_rate=0.030264640226960182, background=104.1486587524414,
         adu_per_nmgy=241.02658081054688,
         psf_params=[1.107237458229065, 2.0800251960754395, 2.3254318237304688,
                     5.240590572357178, 0.7346734404563904, 0.5114791393280029],
         psf_radius=8, noise_additive=1.0000007072408224e-10,
         noise_multiplicative=1.936462640762329)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    out = sys.argv[2] if len(sys.argv) > 2 else None
    H = 8
    model = M71ImageModel(image_height=H, image_width=H, background=P["background"],
                          psf_radius=P["psf_radius"], adu_per_nmgy=P["adu_per_nmgy"],
                          psf_params=P["psf_params"], noise_additive=P["noise_additive"],
                          noise_multiplicative=P["noise_multiplicative"])
    truth = M71Prior(min_objects=0, max_objects=100, counts_rate=P["counts_rate"],
                     image_height=H, image_width=H, flux_alpha=P["flux_alpha"],
                     flux_lower=P["flux_detection_threshold"], flux_upper=P["flux_upper"], pad=4)
    prior = M71Prior(min_objects=10, max_objects=10, counts_rate=P["counts_rate"],
                     image_height=H, image_width=H, flux_alpha=P["flux_alpha"],
                     flux_lower=P["flux_lower"], flux_upper=P["flux_upper"], pad=4)
    torch.manual_seed(0)
    c, l, f = truth.sample(num_catalogs=B)
    tiles = model.sample(l, f)[0, 0].permute(2, 0, 1).reshape(1, B, H, H).contiguous()
    # run_mcmc.py:71-74: 50,000 samples, burn-in 30,000, every 2nd kept
    s = MHsampler.from_tiles(tiles, prior, model, 0.1, 2.5, P["flux_detection_threshold"],
                             50000, 30000, 2, print_every=10000)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.run()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    mean_count = s.posterior_mean_count(s.pruned_counts)[0]
    print(f"{B} cutouts x 50,000 samples in {dt:.3f} s; posterior mean detectable counts "
          f"{[round(float(x), 2) for x in mean_count[:5]]} ...")
    if out:
        os.makedirs(out, exist_ok=True)
        M = s.locs.shape[2]
        for name, v in (("runtime", torch.full((B,), dt / B)), ("counts", s.counts[0]),
                        ("locs", s.locs[0]), ("fluxes", s.fluxes[0])):
            torch.save(v.cpu(), os.path.join(out, f"{name}_0.pt"))
        print(f"wrote {out}/{{runtime,counts,locs,fluxes}}_0.pt ({M} kept samples per cutout)")


if __name__ == "__main__":
    main()
