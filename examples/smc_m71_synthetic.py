"""The reference's notebook flow (notebooks/smc.ipynb, cells 2-7) on a
synthetic M71 image, run unmodified through the drop-in alias: the imports
below are the reference's own module names.

    python examples/smc_m71_synthetic.py [image_size] [tile_dim] [num_catalogs]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import smcdet_amd

smcdet_amd.install_as_smcdet()

from smcdet.images import M71ImageModel, generate_images  # noqa: E402
from smcdet.kernel import SingleComponentMH  # noqa: E402
from smcdet.prior import M71Prior  # noqa: E402
from smcdet.sampler import SMCsampler  # noqa: E402

# notebooks/smc.ipynb cell 2 (full-precision PSF parameters)
params = dict(flux_alpha=0.21411753249015655, flux_lower=0.06291294097900389,
              flux_upper=1804.6791992187502, flux_detection_threshold=0.25165176391601557,
              counts_rate=0.030264640226960182, background=104.1486587524414,
              adu_per_nmgy=241.02658081054688,
              psf_params=[1.107237458229065, 2.0800251960754395, 2.3254318237304688,
                          5.240590572357178, 0.7346734404563904, 0.5114791393280029],
              psf_radius=8, noise_additive=1.0000007072408224e-10,
              noise_multiplicative=1.936462640762329)


def main():
    image_size = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    tile_dim = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    num_catalogs = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    torch.manual_seed(0)
    model = M71ImageModel(image_height=tile_dim, image_width=tile_dim,
                          background=params["background"], psf_radius=params["psf_radius"],
                          adu_per_nmgy=params["adu_per_nmgy"], psf_params=params["psf_params"],
                          noise_additive=params["noise_additive"],
                          noise_multiplicative=params["noise_multiplicative"])
    full = M71ImageModel(image_height=image_size, image_width=image_size,
                         background=params["background"], psf_radius=params["psf_radius"],
                         adu_per_nmgy=params["adu_per_nmgy"], psf_params=params["psf_params"],
                         noise_additive=params["noise_additive"],
                         noise_multiplicative=params["noise_multiplicative"])
    truth = M71Prior(min_objects=0, max_objects=100, counts_rate=params["counts_rate"],
                     image_height=image_size, image_width=image_size,
                     flux_alpha=params["flux_alpha"],
                     flux_lower=params["flux_detection_threshold"],
                     flux_upper=params["flux_upper"], pad=4)
    res = generate_images(truth, full, params["flux_detection_threshold"], 0, image_size, 1)
    pruned_counts, images = res[3], res[-1]
    print(f"true detectable count: {int(pruned_counts.reshape(-1)[0])}")
    prior = M71Prior(min_objects=10, max_objects=10, counts_rate=params["counts_rate"],
                     image_height=tile_dim, image_width=tile_dim,
                     flux_alpha=params["flux_alpha"], flux_lower=params["flux_lower"],
                     flux_upper=params["flux_upper"], pad=4)
    mh = SingleComponentMH(100, 0.1, 2.5, params["flux_lower"], params["flux_upper"])
    sampler = SMCsampler(image=images[0], tile_dim=tile_dim, Prior=prior, ImageModel=model,
                         MutationKernel=mh, num_catalogs=num_catalogs, ess_threshold_prop=0.5,
                         resample_method="multinomial",
                         flux_detection_threshold=params["flux_detection_threshold"],
                         max_smc_iters=100, print_every=10)
    sampler.run()
    sampler.summarize()


if __name__ == "__main__":
    main()
