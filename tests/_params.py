"""Shared model parameters for the tests (values from the reference's
notebooks/smc.ipynb cell 2 and experiments/basic/generate_images.py:26-60)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

M71 = dict(
    flux_alpha=0.21411753249015655,
    flux_lower=0.06291294097900389,
    flux_upper=1804.6791992187502,
    flux_detection_threshold=0.25165176391601557,
    counts_rate=0.030264640226960182,
    background=104.1486587524414,
    adu_per_nmgy=241.02658081054688,
    psf_params=[1.107237458229065, 2.0800251960754395, 2.3254318237304688,
                5.240590572357178, 0.7346734404563904, 0.5114791393280029],
    psf_radius=8,
    noise_additive=1.0000007072408224e-10,
    noise_multiplicative=1.936462640762329,
)
BASIC_PSF_STDEV = 0.93
BASIC_BACKGROUND = 200.0
_psf_max = 1 / (2 * np.pi * BASIC_PSF_STDEV ** 2)
BASIC_FLUX_SCALE = 5 * np.sqrt(BASIC_BACKGROUND) / _psf_max
BASIC_FLUX_ALPHA = (-np.log(1 - 0.99)) / (
    np.log(50 * np.sqrt(BASIC_BACKGROUND) / _psf_max) - np.log(BASIC_FLUX_SCALE))


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


def tiles_of(img, td):
    nt = img.shape[0] // td
    return img[: nt * td, : nt * td].reshape(nt, td, nt, td).transpose(0, 2, 1, 3)


# ---- oracle-side constructors -------------------------------------------
def o_m71_model(H):
    from oracle import smc_oracle as O
    p = M71
    return O.M71Model(H, H, p["background"], p["psf_radius"], p["adu_per_nmgy"],
                      p["psf_params"], p["noise_additive"], p["noise_multiplicative"])


def o_basic_model(H):
    from oracle import smc_oracle as O
    return O.BasicModel(H, H, BASIC_BACKGROUND, 8, BASIC_PSF_STDEV)


def o_m71_prior(H, smin, smax, counts_rate=M71["counts_rate"], pad=4):
    from oracle import smc_oracle as O
    p = M71
    return O.M71PriorP(smin, smax, counts_rate, H, H, pad, p["flux_alpha"], p["flux_lower"],
                       p["flux_upper"])


def o_basic_prior(H, smin, smax, pad=2):
    from oracle import smc_oracle as O
    return O.ParetoPriorP(smin, smax, H, H, pad, BASIC_FLUX_SCALE * 0.9, BASIC_FLUX_ALPHA)


def o_m71_mh(K):
    from oracle import smc_oracle as O
    return O.MHParams(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])


def o_basic_mh(K):
    from oracle import smc_oracle as O
    return O.MHParams(K, 0.1, 100, BASIC_FLUX_SCALE * 0.9, 1e6)


# fixture name -> (tile_dim, oracle model, oracle prior, oracle mh)
def mh_fixture_setup(name):
    if name == "mh_m71_8x8":
        return 8, o_m71_model(8), o_m71_prior(8, 4, 4), o_m71_mh(20)
    if name == "mh_m71_32x32":
        return 32, o_m71_model(32), o_m71_prior(32, 10, 10), o_m71_mh(10)
    if name == "mh_m71_tiles":
        return 8, o_m71_model(8), o_m71_prior(8, 3, 3), o_m71_mh(10)
    if name == "mh_basic_16x16":
        return 16, o_basic_model(16), o_basic_prior(16, 3, 3), o_basic_mh(20)
    if name == "mh_m71_edge_8x8":
        return 8, o_m71_model(8), o_m71_prior(8, 4, 4), o_m71_mh(30)
    if name == "mh_m71_edge_32x32":
        return 32, o_m71_model(32), o_m71_prior(32, 10, 10), o_m71_mh(24)
    raise KeyError(name)


# the edge fixtures (make_golden.py gen_mh_edge) put location proposals exactly
# on the prior box's upper edge: rejected, then the reference's NaN freeze
MH_EDGE_FIXTURES = ["mh_m71_edge_8x8", "mh_m71_edge_32x32"]
MH_FIXTURES = ["mh_m71_8x8", "mh_m71_32x32", "mh_m71_tiles", "mh_basic_16x16"] + MH_EDGE_FIXTURES


def mala_fixture_setup(name):
    """tests/golden/make_golden.py gen_mala: the MH fixtures' geometries,
    with SingleComponentMALA(K, locs_step, fluxes_step, fluxes_min, fluxes_max)."""
    if name in ("mala_m71_8x8", "mala_m71_8x8_tau1"):
        return 8, o_m71_model(8), o_m71_prior(8, 4, 4), o_m71_mh(20)
    if name == "mala_m71_32x32":
        return 32, o_m71_model(32), o_m71_prior(32, 10, 10), o_m71_mh(10)
    if name == "mala_m71_tiles":
        return 8, o_m71_model(8), o_m71_prior(8, 3, 3), o_m71_mh(10)
    if name == "mala_basic_16x16":
        return 16, o_basic_model(16), o_basic_prior(16, 3, 3), o_basic_mh(20)
    raise KeyError(name)


MALA_FIXTURES = ["mala_m71_8x8", "mala_m71_8x8_tau1", "mala_m71_32x32", "mala_m71_tiles",
                 "mala_basic_16x16"]


# ---- product-side constructors (smcdet_amd) -------------------------------
def p_m71_model(H):
    from smcdet_amd.images import M71ImageModel
    p = M71
    return M71ImageModel(image_height=H, image_width=H, background=p["background"],
                         psf_radius=p["psf_radius"], adu_per_nmgy=p["adu_per_nmgy"],
                         psf_params=p["psf_params"], noise_additive=p["noise_additive"],
                         noise_multiplicative=p["noise_multiplicative"])


def p_basic_model(H):
    from smcdet_amd.images import ImageModel
    return ImageModel(image_height=H, image_width=H, psf_radius=8, psf_stdev=BASIC_PSF_STDEV,
                      background=BASIC_BACKGROUND)


def p_m71_prior(H, smin, smax, counts_rate=M71["counts_rate"], pad=4):
    from smcdet_amd.prior import M71Prior
    p = M71
    return M71Prior(min_objects=smin, max_objects=smax, counts_rate=counts_rate, image_height=H,
                    image_width=H, flux_alpha=p["flux_alpha"], flux_lower=p["flux_lower"],
                    flux_upper=p["flux_upper"], pad=pad)


def p_basic_prior(H, smin, smax, pad=2):
    from smcdet_amd.prior import ParetoStarPrior
    return ParetoStarPrior(min_objects=smin, max_objects=smax, image_height=H, image_width=H,
                           flux_scale=BASIC_FLUX_SCALE * 0.9, flux_alpha=BASIC_FLUX_ALPHA,
                           pad=pad)


def p_m71_mh(K, **kw):
    from smcdet_amd.kernel import SingleComponentMH
    return SingleComponentMH(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"], **kw)


def p_basic_mh(K, **kw):
    from smcdet_amd.kernel import SingleComponentMH
    return SingleComponentMH(K, 0.1, 100, BASIC_FLUX_SCALE * 0.9, 1e6, **kw)


def p_mh_fixture_setup(name, **kw):
    if name == "mh_m71_8x8":
        return 8, p_m71_model(8), p_m71_prior(8, 4, 4), p_m71_mh(20, **kw)
    if name == "mh_m71_32x32":
        return 32, p_m71_model(32), p_m71_prior(32, 10, 10), p_m71_mh(10, **kw)
    if name == "mh_m71_tiles":
        return 8, p_m71_model(8), p_m71_prior(8, 3, 3), p_m71_mh(10, **kw)
    if name == "mh_basic_16x16":
        return 16, p_basic_model(16), p_basic_prior(16, 3, 3), p_basic_mh(20, **kw)
    if name == "mh_m71_edge_8x8":
        return 8, p_m71_model(8), p_m71_prior(8, 4, 4), p_m71_mh(30, **kw)
    if name == "mh_m71_edge_32x32":
        return 32, p_m71_model(32), p_m71_prior(32, 10, 10), p_m71_mh(24, **kw)
    raise KeyError(name)


def p_mala_fixture_setup(name):
    from smcdet_amd.kernel import SingleComponentMALA
    if name in ("mala_m71_8x8", "mala_m71_8x8_tau1"):
        K, H, S = 20, 8, 4
    elif name == "mala_m71_32x32":
        K, H, S = 10, 32, 10
    elif name == "mala_m71_tiles":
        K, H, S = 10, 8, 3
    elif name == "mala_basic_16x16":
        return (16, p_basic_model(16), p_basic_prior(16, 3, 3),
                SingleComponentMALA(20, 0.1, 100, BASIC_FLUX_SCALE * 0.9, 1e6))
    else:
        raise KeyError(name)
    return (H, p_m71_model(H), p_m71_prior(H, S, S),
            SingleComponentMALA(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"]))
