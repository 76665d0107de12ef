"""Tile aggregation beyond the LDS budget: joint tiles
whose image, two rate images and catalog per wave do not fit 160 KiB of LDS
at 4 waves run smcdet_aggregate_sweep's global-memory variant (the caller's
workspace, smcdet_aggregate_workspace), so Aggregate reaches whole images of
up to 256x256 pixels (the reference aggregates to the whole image,
smcdet/aggregate.py:523-593).  Checked against the oracle (oracle/
agg_oracle.py) on 128x64 / 64x128 joint tiles -- l_p, l_c1 + l_c2 and a
replayed sweep on the bridging target -- and end to end: a 128x128 image from
a 4x4 grid of 32x32 tiles (CS-SMC children), aggregated over 4 levels, the
last two through the workspace."""
import contextlib
import io

import numpy as np
import pytest
import torch

from oracle import agg_oracle as A
from oracle import smc_oracle as O
from tests._params import M71
from tests.test_gpu_aggregate import D, N_, mh, o_model, o_prior, p_model, p_prior

pytestmark = pytest.mark.gpu
DEV = "cuda"


def joint_population(H, W, S, N, seed):
    """Count-varying catalogs (0..S sources, compacted) over a joint tile, and
    a synthetic image of a few bright stars."""
    rng = np.random.default_rng(seed)
    counts = rng.integers(0, S + 1, (1, 1, N)).astype(np.float32)
    mask = np.arange(S) < counts[..., None]
    locs = np.stack([rng.uniform(-4, H + 4, (1, 1, N, S)), rng.uniform(-4, W + 4, (1, 1, N, S))],
                    -1).astype(np.float32) * mask[..., None]
    fluxes = (rng.uniform(0.5, 20.0, (1, 1, N, S)) * mask).astype(np.float32)
    tl = torch.tensor(np.stack([rng.uniform(4, H - 4, 6), rng.uniform(4, W - 4, 6)], -1),
                      dtype=torch.float32).reshape(1, 1, 1, 6, 2)
    tf = torch.tensor(rng.uniform(5, 30, 6), dtype=torch.float32).reshape(1, 1, 1, 6)
    torch.manual_seed(seed)
    img = p_model(H, W).sample(tl.to(DEV), tf.to(DEV))[0, 0, :, :, 0]
    return N_(img)[None, None], counts, locs, fluxes


@pytest.mark.parametrize("axis", [0, 1])
def test_large_joint_tile_sweep_vs_oracle(axis):
    from smcdet_amd import _hip
    from smcdet_amd.aggregate import aggregate_sweep
    H, W = (128, 64) if axis == 0 else (64, 128)
    S, N, K = 24, 32, 12
    d, c, l, f = joint_population(H, W, S, N, 20 + axis)
    prior, model, k = p_prior(H, W, 0, S), p_model(H, W), mh(K)
    k.locs_min, k.locs_max = prior.loc_prior.low, prior.loc_prior.high
    need = _hip.lib().smcdet_aggregate_workspace(_hip.ref(model._cmodel()), 1, N, S)
    assert need == N * (2 * H * W + 3 * S)  # the global-memory variant runs
    tau0 = D(np.full((1, 1), 0.3, np.float32))
    _, lo, fo, lp, lc, _ = aggregate_sweep(model, prior, k, axis, D(d), tau0, D(c), D(l), D(f),
                                           num_iters=0)
    np.testing.assert_array_equal(N_(lo), l)
    olp, olc = A.parent_child_loglik(d, c, l, f, o_model(H, W), axis)
    np.testing.assert_allclose(N_(lp), olp, rtol=3e-6, atol=3e-3)
    np.testing.assert_allclose(N_(lc), olc, rtol=3e-6, atol=3e-3)
    # a replayed sweep on the bridging target at tau = 0.4
    rng = np.random.default_rng(30 + axis)
    cnt = np.maximum(c, 1).astype(np.int64)
    comp = np.minimum((rng.random((K,) + c.shape) * cnt).astype(np.int32), cnt - 1).astype(np.int32)
    uloc = rng.random((K,) + c.shape + (2,)).astype(np.float32)
    uflux = rng.random((K,) + c.shape).astype(np.float32)
    uacc = rng.random((K,) + c.shape).astype(np.float32)
    tau = np.full((1, 1), 0.4, np.float32)
    ol, of, oacc, marg = A.agg_mh_sweep(d, c, l, f, tau, o_prior(H, W, S), o_model(H, W), axis,
                                        O.MHParams(K, 0.1, 2.5, M71["flux_lower"],
                                                   M71["flux_upper"]),
                                        comp, uloc, uflux, uacc, trace=True)
    rp = dict(comp=torch.as_tensor(comp), uloc=torch.as_tensor(uloc),
              uflux=torch.as_tensor(uflux), uacc=torch.as_tensor(uacc))
    ws = torch.zeros(2, device=DEV, dtype=torch.int32)
    co, lo, fo, lp, lc, acc = aggregate_sweep(model, prior, k, axis, D(d), D(tau), D(c), D(l),
                                              D(f), replay=rp, acc_workspace=ws)
    clear = np.all(np.abs(np.nan_to_num(marg, nan=0.0)) > 1e-3, axis=0)
    assert clear.mean() > 0.8, clear.mean()
    assert oacc.any() and (~oacc).any()
    np.testing.assert_array_equal(N_(co), c)
    np.testing.assert_allclose(N_(lo)[clear], ol[clear], rtol=0, atol=5e-5)
    np.testing.assert_allclose(N_(fo)[clear], of[clear], rtol=3e-5, atol=1e-5)
    olp, olc = A.parent_child_loglik(d, c, ol, of, o_model(H, W), axis)
    np.testing.assert_allclose(N_(lp)[clear], olp[clear], rtol=3e-6, atol=3e-3)
    np.testing.assert_allclose(N_(lc)[clear], olc[clear], rtol=3e-6, atol=3e-3)
    assert int(ws.abs().sum()) == 0


def test_aggregate_to_128x128_image():
    """CS-SMC on the 4x4 32x32 tiles of a 128x128 M71 image (counts 0..3,
    partition boxes), then Aggregate.run over 4 levels to one 128x128
    population (joint tiles 64x32 and 64x64 in LDS, 128x64 and 128x128
    through the workspace).  The final state's parent log-likelihood is the
    oracle's, the evidence is finite, every source lies in the image's padded
    box, and the detected stars cover the truth's bright ones."""
    from smcdet_amd.aggregate import Aggregate
    from smcdet_amd.cssmc import CountStratifiedSMC
    H, tile, N, K = 128, 32, 256, 20
    rng = np.random.default_rng(5)
    # eight bright stars, well inside their 32x32 tiles
    cells = rng.choice(16, 8, replace=False)
    tl = torch.tensor([[(c // 4) * 32 + rng.uniform(8, 24), (c % 4) * 32 + rng.uniform(8, 24)]
                       for c in cells], dtype=torch.float32).reshape(1, 1, 1, 8, 2)
    tf = torch.tensor(rng.uniform(15, 40, 8), dtype=torch.float32).reshape(1, 1, 1, 8)
    torch.manual_seed(5)
    img = p_model(H, H).sample(tl.to(DEV), tf.to(DEV))[0, 0, :, :, 0].contiguous()
    kp = p_prior(tile, tile, 0, 3, counts_rate=0.001, pad=2, pad_mode="partition")
    kids = CountStratifiedSMC(img, tile, kp, p_model(tile, tile), mh(K), N, 0.5, "systematic",
                              M71["flux_detection_threshold"], 200, print_every=10 ** 9,
                              num_catalogs=N, seed=21, device=DEV)
    with contextlib.redirect_stdout(io.StringIO()):
        kids.run()
    agg = Aggregate(kp, p_model(tile, tile), mh(K), kids.tiled_image, kids.counts, kids.locs,
                    kids.fluxes, kids.weights, kids.log_normalizing_constant,
                    M71["flux_detection_threshold"], "systematic", 0.5, print_every=10 ** 9,
                    seed=22, device=DEV)
    with contextlib.redirect_stdout(io.StringIO()):
        agg.run()
    assert agg.num_aggregation_levels == 4 and len(agg.iters_per_level) == 4
    assert (agg.numH, agg.numW, agg.dimH, agg.dimW) == (1, 1, H, H)
    assert np.isfinite(float(agg.log_evidence))
    lo, fl = N_(agg.locs), N_(agg.fluxes)
    pres = fl != 0
    assert (lo[pres] >= -2).all() and (lo[pres] < H + 2).all()
    # the final population's l_p against the oracle (a subset of particles)
    sub = slice(0, 16)
    c = N_(agg.counts)[:, :, sub]
    ll = agg.ImageModel.loglikelihood(agg.data, agg.locs[:, :, sub].contiguous(),
                                      agg.fluxes[:, :, sub].contiguous())
    ref = O.loglikelihood(N_(agg.data), lo[:, :, sub], fl[:, :, sub], o_model(H, H))
    np.testing.assert_allclose(N_(ll), ref, rtol=4e-6, atol=5e-3)
    assert c.max() <= 48
    det = float(agg.pruned_counts.float().mean())
    assert 7.0 <= det <= 12.0, det


def test_poisson_64x64_joint_tile_reduced_waves_vs_oracle():
    """The basic (Poisson) image model has no global-memory sweep: a 64x64
    joint tile (image + lgamma(x+1), and per wave two rate images and the
    catalog: 160 KiB at 4 waves is exceeded for any S) runs the LDS sweep at
    the largest wave count that fits, no workspace.  l_p, l_c and
    a replayed sweep on the bridging target against the oracle.  Tolerance
    rtol 1e-5: a 4,096-pixel Poisson sum carries the float32 lgamma(x + 1)
    roundings (the reference's own float32 Poisson.log_prob does too) --
    ~0.2 nats, the same for every particle, against the float64 oracle."""
    from smcdet_amd import _hip
    from smcdet_amd.aggregate import aggregate_sweep
    from smcdet_amd.images import ImageModel
    from smcdet_amd.prior import ParetoStarPrior
    from tests._params import BASIC_BACKGROUND, BASIC_FLUX_ALPHA, BASIC_FLUX_SCALE, BASIC_PSF_STDEV
    H = W = 64
    S, N, K, axis = 8, 24, 10, 0
    model = ImageModel(image_height=H, image_width=W, psf_radius=8, psf_stdev=BASIC_PSF_STDEV,
                       background=BASIC_BACKGROUND)
    prior = ParetoStarPrior(min_objects=0, max_objects=S, image_height=H, image_width=W,
                            flux_scale=BASIC_FLUX_SCALE * 0.9, flux_alpha=BASIC_FLUX_ALPHA, pad=2)
    om = O.BasicModel(H, W, BASIC_BACKGROUND, 8, BASIC_PSF_STDEV)
    op = O.ParetoPriorP(0, S, H, W, 2, BASIC_FLUX_SCALE * 0.9, BASIC_FLUX_ALPHA)
    from smcdet_amd.kernel import SingleComponentMH
    k = SingleComponentMH(K, 0.1, 100.0, BASIC_FLUX_SCALE * 0.9, 1e6)
    k.locs_min, k.locs_max = prior.loc_prior.low, prior.loc_prior.high
    assert _hip.lib().smcdet_aggregate_workspace(_hip.ref(model._cmodel()), 1, N, S) == 0
    rng = np.random.default_rng(41)
    c = rng.integers(1, S + 1, (1, 1, N)).astype(np.float32)
    mask = np.arange(S) < c[..., None]
    l = np.stack([rng.uniform(-2, H + 2, (1, 1, N, S)), rng.uniform(-2, W + 2, (1, 1, N, S))],
                 -1).astype(np.float32) * mask[..., None]
    f = (rng.uniform(400, 3000, (1, 1, N, S)) * mask).astype(np.float32)
    tl = np.stack([rng.uniform(6, H - 6, 5), rng.uniform(6, W - 6, 5)], -1).reshape(1, 1, 1, 5, 2)
    tf = rng.uniform(800, 4000, 5).reshape(1, 1, 1, 5)
    rate = O.render_rate(tl, tf, om)[0, 0, :, :, 0]
    d = rng.poisson(rate).astype(np.float32)[None, None]
    tau0 = D(np.full((1, 1), 0.3, np.float32))
    _, lo, _, lp, lc, _ = aggregate_sweep(model, prior, k, axis, D(d), tau0, D(c), D(l), D(f),
                                          num_iters=0)
    np.testing.assert_array_equal(N_(lo), l)
    olp, olc = A.parent_child_loglik(d, c, l, f, om, axis)
    np.testing.assert_allclose(N_(lp), olp, rtol=1e-5, atol=3e-3)
    np.testing.assert_allclose(N_(lc), olc, rtol=1e-5, atol=3e-3)
    comp = np.minimum((rng.random((K,) + c.shape) * c).astype(np.int32), c.astype(np.int32) - 1)
    uloc = rng.random((K,) + c.shape + (2,)).astype(np.float32)
    uflux = rng.random((K,) + c.shape).astype(np.float32)
    uacc = rng.random((K,) + c.shape).astype(np.float32)
    tau = np.full((1, 1), 0.4, np.float32)
    ol, of, oacc, marg = A.agg_mh_sweep(d, c, l, f, tau, op, om, axis,
                                        O.MHParams(K, 0.1, 100.0, BASIC_FLUX_SCALE * 0.9, 1e6),
                                        comp, uloc, uflux, uacc, trace=True)
    rp = dict(comp=torch.as_tensor(comp.astype(np.int32)), uloc=torch.as_tensor(uloc),
              uflux=torch.as_tensor(uflux), uacc=torch.as_tensor(uacc))
    ws = torch.zeros(2, device=DEV, dtype=torch.int32)
    co, lo, fo, lp, lc, acc = aggregate_sweep(model, prior, k, axis, D(d), D(tau), D(c), D(l),
                                              D(f), replay=rp, acc_workspace=ws)
    clear = np.all(np.abs(np.nan_to_num(marg, nan=0.0)) > 1e-3, axis=0)
    assert clear.mean() > 0.7, clear.mean()
    assert oacc.any() and (~oacc).any()
    np.testing.assert_allclose(N_(lo)[clear], ol[clear], rtol=0, atol=5e-5)
    np.testing.assert_allclose(N_(fo)[clear], of[clear], rtol=3e-5, atol=1e-3)
    olp, olc = A.parent_child_loglik(d, c, ol, of, om, axis)
    np.testing.assert_allclose(N_(lp)[clear], olp[clear], rtol=1e-5, atol=3e-3)
    np.testing.assert_allclose(N_(lc)[clear], olc[clear], rtol=1e-5, atol=3e-3)
    assert int(ws.abs().sum()) == 0
