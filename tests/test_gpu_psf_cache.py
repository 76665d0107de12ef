"""The MH sweep's LDS caches.  Small tiles (<= 64 pixels, incremental MH): each wave
keeps its particle's S raw PSF images in LDS, so a move reads the moved
source's old PSF instead of re-evaluating it.  The cached values are the ones
the uncached sweep computes (same operations on the same inputs), so whole
SMC runs are bit-identical with and without the cache
(SMCDET_MH_NO_PSF_CACHE).  A self-consistency regression; the cached sweep's
parity with the reference is pinned by the 8x8 replays of
test_gpu_parity.py (mh_m71_8x8, mh_m71_edge_8x8, mh_m71_tiles and the
recorded SMC runs), which now run through it.
"""
import contextlib

import numpy as np
import pytest
import torch

from tests._params import (M71, p_basic_mh, p_basic_model, p_basic_prior, p_m71_mh, p_m71_model,
                           p_m71_prior)

pytestmark = pytest.mark.gpu
DEV = "cuda"
NO_PSF_CACHE = 2048  # include/smcdet_hip.h
PSF_TABLE = 8192
NO_RCP_CACHE = 4096
DIAG_FLAGS = PSF_TABLE | NO_RCP_CACHE


def _lib_for(flags):
    """The library a variant lives in: the product's own kernels, or -- for the
    diagnostic variants (PSF table, no 1/v cache), which the product refuses --
    the diagnostic build (make diag), in the same process."""
    from smcdet_amd import _hip
    return _hip.diag_library() if flags & DIAG_FLAGS else contextlib.nullcontext()


def _m71_image(H, seed, n_tiles, counts_rate=0.004):
    torch.manual_seed(seed)
    truth = p_m71_prior(H * n_tiles, 0, 40, counts_rate=counts_rate)
    _, l, f = truth.sample(num_catalogs=1, device=DEV)
    return p_m71_model(H * n_tiles).sample(l, f)[0, 0, :, :, 0].contiguous()


def _run(img, td, prior, model, mh, N, seed, cache, by_count=False, flags=0):
    from smcdet_amd.sampler import SMCsampler
    mh.debug_flags = flags | (0 if cache else NO_PSF_CACHE)
    s = SMCsampler(img, td, prior, model, mh, N, 0.5, "systematic",
                   M71["flux_detection_threshold"], 200, print_every=10 ** 9, seed=seed,
                   device=DEV)
    with _lib_for(flags):
        s.run()
        torch.cuda.synchronize()
    return {k: getattr(s, k).detach().cpu().numpy().copy()
            for k in ("temperature", "log_normalizing_constant", "ess", "locs", "fluxes",
                      "counts", "loglik", "mutation_acc_rates")} | {"iter": np.array(s.iter)}


def _assert_same(a, b):
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


@pytest.mark.parametrize("table", [True, False], ids=["psf-table", "exp2"])
@pytest.mark.parametrize("S", [4, 10])
def test_psf_cache_m71_8x8_run_is_bit_identical(S, table):
    """2x2 grid of 8x8 M71 tiles at the real M71 source density, N = 1024,
    K = 50, to temperature 1 (>= 10 SMC iterations, so the cache's accept-path
    updates are compared many times over), with the PSF values from exp2/log2
    (default) and from the opt-in radial table (SMCDET_MH_PSF_TABLE)."""
    img = _m71_image(8, 21 + S, 2, counts_rate=M71["counts_rate"])
    fl = PSF_TABLE if table else 0
    out = [_run(img, 8, p_m71_prior(8, S, S), p_m71_model(8), p_m71_mh(50), 1024, 5, c, flags=fl)
           for c in (True, False)]
    assert out[0]["iter"] >= 10, int(out[0]["iter"])
    _assert_same(*out)


def test_psf_cache_poisson_8x8_run_is_bit_identical():
    """The basic Poisson model on 8x8 tiles (Normal-pdf PSF in the cache)."""
    torch.manual_seed(4)
    model = p_basic_model(16)
    truth = p_basic_prior(16, 0, 3)
    _, l, f = truth.sample(num_catalogs=1, device=DEV)
    img = model.sample(l, f)[0, 0, :, :, 0].contiguous()
    out = [_run(img, 8, p_basic_prior(8, 3, 3), p_basic_model(8), p_basic_mh(40), 512, 9, c)
           for c in (True, False)]
    _assert_same(*out)


@pytest.mark.parametrize("H,N,base", [(32, 1024, 0), (16, 512, 0), (16, 512, PSF_TABLE)])
def test_rcp_cache_m71_run_is_bit_identical(H, N, base):
    """M71 tiles of 65..1024 pixels keep a per-wave image of 1/(s0^2 + eta*rate)
    in LDS (read by the pixel delta instead of formed; on accept the delta's
    own reciprocal of the new rate is stored): whole C2-geometry runs are
    bit-identical with and without it (SMCDET_MH_NO_RCP_CACHE); 16x16 tiles
    also with the opt-in PSF table (SMCDET_MH_PSF_TABLE), which at 32x32 takes
    the LDS the 1/v image needs.  The sweeps without the 1/v image (and the
    table's) are the diagnostic build's: base 0 compares the PRODUCT library's
    sweep with the diagnostic build's uncached one."""
    img = _m71_image(H, 31 + H, 1)
    out = []
    for flags in (base, base | NO_RCP_CACHE):
        from smcdet_amd.sampler import SMCsampler
        mh = p_m71_mh(100)
        mh.debug_flags = flags
        s = SMCsampler(img, H, p_m71_prior(H, 10, 10, counts_rate=0.003125), p_m71_model(H), mh,
                       N, 0.5, "systematic", M71["flux_detection_threshold"], 200,
                       print_every=10 ** 9, seed=13, device=DEV)
        with _lib_for(flags):
            s.run()
            torch.cuda.synchronize()
        out.append({k: getattr(s, k).detach().cpu().numpy().copy()
                     for k in ("temperature", "log_normalizing_constant", "ess", "locs", "fluxes",
                               "loglik", "mutation_acc_rates")} | {"iter": np.array(s.iter)})
    assert out[0]["iter"] >= 2
    _assert_same(*out)


def test_psf_table_sweep_close_to_exp2_sweep():
    """The opt-in radial PSF table (SMCDET_MH_PSF_TABLE) against the default
    exp2/log2 form on one C2-geometry sweep from the same state
    with the same Philox draws: the table's PSF values differ by float32
    rounding (<= 3e-7 relative), so the two sweeps make the same decisions
    except at near ties -- and they are not bit-identical (the table path
    ran; the table is the diagnostic build's, the exp2 form the product's)."""
    from smcdet_amd._rng import PhiloxStream
    H, N, K = 32, 2048, 100
    img = _m71_image(H, 77, 1, counts_rate=0.003125)[None, None].contiguous()
    prior, model = p_m71_prior(H, 10, 10, counts_rate=0.003125), p_m71_model(H)
    torch.manual_seed(8)
    counts, locs, fluxes = prior.sample(num_tiles_per_side=1, stratify_by_count=True,
                                        num_catalogs_per_count=N, device=DEV)
    tau = torch.tensor([[0.02]], device=DEV)
    res = []
    for flags in (PSF_TABLE, 0):
        mh = p_m71_mh(K)
        mh.debug_flags = flags
        mh.rng = PhiloxStream(17)
        with _lib_for(flags):
            lo, fo, _ = mh.run(img, counts, locs, fluxes, tau, prior=prior, image_model=model)
            torch.cuda.synchronize()
        res.append((lo.cpu().numpy(), fo.cpu().numpy(), mh.last_loglik.cpu().numpy()))
    same = np.all(res[0][0] == res[1][0], axis=(-1, -2)) & np.all(res[0][1] == res[1][1], axis=-1)
    assert same.mean() > 0.97, same.mean()
    close = np.abs(res[0][2] - res[1][2])[same]
    assert close.max() < 2e-2, close.max()
    assert not all(np.array_equal(a, b) for a, b in zip(res[0], res[1]))


NO_BLOCK = 16384  # include/smcdet_hip.h


@pytest.mark.parametrize("H,W,R", [(32, 32, 8), (24, 40, 8), (40, 24, 8), (32, 32, 9)])
def test_block_form_sweep_close_to_per_pixel_sweep(H, W, R):
    """The block form of same-anchor M71 steps (the union window's first 16
    rows / columns as a 16x16 block whose Gaussian PSF terms are one rank-4
    MFMA) against the per-pixel form (SMCDET_MH_NO_BLOCK) on one sweep from
    the same state with the same Philox draws: the profile is rounded
    differently (a few ulp), so the decisions agree except at near ties, each
    sweep's log-likelihood equals a fresh evaluation of its final state, each
    persisted rate image equals a fresh render of it, and the two sweeps are
    not bit-identical (the block path ran).  R = 9 (19x19 windows, which the
    block's one-row / one-column strip cannot hold) must take the per-pixel
    form: identical results, rate images and log-likelihoods fresh."""
    from smcdet_amd._rng import PhiloxStream
    from smcdet_amd.images import M71ImageModel
    from smcdet_amd.prior import M71Prior
    N, K = 2048, 100
    p = M71
    model = M71ImageModel(image_height=H, image_width=W, background=p["background"],
                          psf_radius=R, adu_per_nmgy=p["adu_per_nmgy"],
                          psf_params=p["psf_params"], noise_additive=p["noise_additive"],
                          noise_multiplicative=p["noise_multiplicative"])

    def prior(smin, smax, rate):
        return M71Prior(min_objects=smin, max_objects=smax, counts_rate=rate, image_height=H,
                        image_width=W, flux_alpha=p["flux_alpha"], flux_lower=p["flux_lower"],
                        flux_upper=p["flux_upper"], pad=4)

    torch.manual_seed(3)
    _, l, f = prior(0, 40, 0.004).sample(num_catalogs=1, device=DEV)
    img = model.sample(l, f)[0, 0, :, :, 0].contiguous()[None, None]
    pr = prior(10, 10, 0.003125)
    torch.manual_seed(8)
    counts, locs, fluxes = pr.sample(num_tiles_per_side=1, stratify_by_count=True,
                                     num_catalogs_per_count=N, device=DEV)
    tau = torch.tensor([[0.05]], device=DEV)
    res = []
    for flags in (0, NO_BLOCK):
        mh = p_m71_mh(K)
        mh.debug_flags = flags
        mh.rng = PhiloxStream(17)
        rate = torch.empty(1, 1, N, H * W, device=DEV)
        lo, fo, _ = mh.run(img, counts, locs, fluxes, tau, prior=pr, image_model=model,
                           rate_out=rate)
        ll = mh.last_loglik.cpu().numpy()
        np.testing.assert_allclose(ll, model.loglikelihood(img, lo, fo).cpu().numpy(),
                                   rtol=2e-6, atol=2e-3)
        fresh = model.rate(lo, fo)[0, 0].permute(2, 0, 1).reshape(N, H * W)
        np.testing.assert_allclose(rate[0, 0].cpu().numpy(), fresh.cpu().numpy(),
                                   rtol=2e-5, atol=2e-3)
        res.append((lo.cpu().numpy(), fo.cpu().numpy(), ll))
    same = np.all(res[0][0] == res[1][0], axis=(-1, -2)) & np.all(res[0][1] == res[1][1], axis=-1)
    assert same.mean() > 0.97, same.mean()
    # the same final state: log-likelihoods (summed over each sweep's own
    # rate image) as close as each is to a fresh evaluation
    np.testing.assert_allclose(res[0][2][same], res[1][2][same], rtol=4e-6, atol=4e-3)
    identical = all(np.array_equal(a, b) for a, b in zip(res[0], res[1]))
    assert identical == (R != 8), identical
