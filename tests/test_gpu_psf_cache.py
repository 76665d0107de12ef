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
import numpy as np
import pytest
import torch

from tests._params import (M71, p_basic_mh, p_basic_model, p_basic_prior, p_m71_mh, p_m71_model,
                           p_m71_prior)

pytestmark = pytest.mark.gpu
DEV = "cuda"
NO_PSF_CACHE = 2048  # include/smcdet_hip.h


def _m71_image(H, seed, n_tiles):
    torch.manual_seed(seed)
    truth = p_m71_prior(H * n_tiles, 0, 40, counts_rate=0.004)
    _, l, f = truth.sample(num_catalogs=1, device=DEV)
    return p_m71_model(H * n_tiles).sample(l, f)[0, 0, :, :, 0].contiguous()


def _run(img, td, prior, model, mh, N, seed, cache, by_count=False):
    from smcdet_amd.sampler import SMCsampler
    mh.debug_flags = 0 if cache else NO_PSF_CACHE
    s = SMCsampler(img, td, prior, model, mh, N, 0.5, "systematic",
                   M71["flux_detection_threshold"], 200, print_every=10 ** 9, seed=seed,
                   device=DEV)
    s.run()
    torch.cuda.synchronize()
    return {k: getattr(s, k).detach().cpu().numpy().copy()
            for k in ("temperature", "log_normalizing_constant", "ess", "locs", "fluxes",
                      "counts", "loglik", "mutation_acc_rates")} | {"iter": np.array(s.iter)}


def _assert_same(a, b):
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


@pytest.mark.parametrize("S", [4, 10])
def test_psf_cache_m71_8x8_run_is_bit_identical(S):
    """2x2 grid of 8x8 M71 tiles, N = 1024, K = 50, to temperature 1."""
    img = _m71_image(8, 21 + S, 2)
    out = [_run(img, 8, p_m71_prior(8, S, S), p_m71_model(8), p_m71_mh(50), 1024, 5, c)
           for c in (True, False)]
    assert out[0]["iter"] >= 2
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


NO_RCP_CACHE = 4096  # include/smcdet_hip.h


@pytest.mark.parametrize("H,N", [(32, 1024), (16, 512)])
def test_rcp_cache_m71_run_is_bit_identical(H, N):
    """M71 tiles of 65..1024 pixels keep a per-wave image of 1/(s0^2 + eta*rate)
    in LDS (read by the pixel delta instead of formed; on accept the delta's
    own reciprocal of the new rate is stored): whole C2-geometry runs are
    bit-identical with and without it (SMCDET_MH_NO_RCP_CACHE)."""
    img = _m71_image(H, 31 + H, 1)
    out = []
    for flags in (0, NO_RCP_CACHE):
        from smcdet_amd.sampler import SMCsampler
        mh = p_m71_mh(100)
        mh.debug_flags = flags
        s = SMCsampler(img, H, p_m71_prior(H, 10, 10, counts_rate=0.003125), p_m71_model(H), mh,
                       N, 0.5, "systematic", M71["flux_detection_threshold"], 200,
                       print_every=10 ** 9, seed=13, device=DEV)
        s.run()
        torch.cuda.synchronize()
        out.append({k: getattr(s, k).detach().cpu().numpy().copy()
                     for k in ("temperature", "log_normalizing_constant", "ess", "locs", "fluxes",
                               "loglik", "mutation_acc_rates")} | {"iter": np.array(s.iter)})
    assert out[0]["iter"] >= 2
    _assert_same(*out)
