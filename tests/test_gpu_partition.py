"""Per-tile location boxes (Prior pad_mode="partition", SMCDET ABI 12): the
tiles' prior boxes partition the padded image (padding only on its outer
edges).  Prior draws, prior log-probabilities and MH sweeps under replayed
draws against the oracle with each tile's own box, and tile aggregation in
this mode against a single large-tile sampler on the same image (DESIGN.md
§9: the exact variant; evidence included)."""
import numpy as np
import pytest
import torch

from oracle import smc_oracle as O
from tests._params import M71, golden, o_m71_model

pytestmark = pytest.mark.gpu
DEV = "cuda"


def N_(t):
    return t.detach().cpu().numpy()


def p_prior(H, smin, smax, pad, mode, rate=M71["counts_rate"]):
    from smcdet_amd.prior import M71Prior
    p = M71
    return M71Prior(min_objects=smin, max_objects=smax, counts_rate=rate, image_height=H,
                    image_width=H, flux_alpha=p["flux_alpha"], flux_lower=p["flux_lower"],
                    flux_upper=p["flux_upper"], pad=pad, pad_mode=mode)


def p_model(H):
    from smcdet_amd.images import M71ImageModel
    p = M71
    return M71ImageModel(image_height=H, image_width=H, background=p["background"],
                         psf_radius=p["psf_radius"], adu_per_nmgy=p["adu_per_nmgy"],
                         psf_params=p["psf_params"], noise_additive=p["noise_additive"],
                         noise_multiplicative=p["noise_multiplicative"])


def o_prior(H, smin, smax, pad, box):
    p = M71
    return O.M71PriorP(smin, smax, p["counts_rate"], H, H, pad, p["flux_alpha"], p["flux_lower"],
                       p["flux_upper"], box=tuple(float(v) for v in box))


def test_partition_boxes_layout():
    from smcdet_amd.prior import partition_boxes
    b = N_(partition_boxes((2, 3), 8, 8, 2))
    assert b.shape == (6, 4)
    # corner tile (0, 0): padded on top and left; middle of the top row: top only
    np.testing.assert_array_equal(b[0], [-2, -2, 8, 8])
    np.testing.assert_array_equal(b[1], [-2, 0, 8, 8])
    np.testing.assert_array_equal(b[5], [0, 0, 10, 10])
    # the boxes tile the padded 16x24 image exactly
    area = ((b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])).sum()
    assert area == (16 + 4) * (24 + 4)


def test_prior_sample_and_log_prob_in_tile_boxes():
    """Stratified prior draws land in each tile's own box (and use the outer
    padding), and log_prob with the boxes equals the oracle's per-tile prior
    (uniform density over the box, Poisson mean of the box area)."""
    from smcdet_amd._rng import PhiloxStream
    pr = p_prior(8, 0, 4, 2, "partition")
    boxes = pr.tile_boxes((2, 2), DEV)
    c, l, f = pr.sample_stratified(2, 256, device=DEV, rng=PhiloxStream(3), tiles_shape=(2, 2),
                                   tile_boxes=boxes)
    lc, ll, lf, b = N_(c), N_(l).reshape(4, -1, 4, 2), N_(f).reshape(4, -1, 4), N_(boxes)
    pres = np.arange(4) < lc.reshape(4, -1)[..., None]
    for t in range(4):
        h, w = ll[t][..., 0][pres[t]], ll[t][..., 1][pres[t]]
        assert (h >= b[t, 0]).all() and (h < b[t, 2]).all()
        assert (w >= b[t, 1]).all() and (w < b[t, 3]).all()
    assert (ll[0][..., 0][pres[0]] < 0).any()       # tile (0,0) uses the top padding
    assert not (ll[3][..., 0][pres[3]] < 0).any()   # tile (1,1) has none on top
    lp = N_(pr.log_prob(c, l, f, tile_boxes=boxes)).reshape(4, -1)
    for t in range(4):
        op = o_prior(8, 0, 4, 2, b[t])
        ref = O.log_prior(lc.reshape(4, -1)[t], ll[t], lf[t], op)
        np.testing.assert_allclose(lp[t], ref, rtol=2e-6, atol=2e-4)


def test_mh_sweep_with_tile_boxes_vs_oracle():
    """The MH sweep with per-tile boxes under replayed draws: every tile's
    particles against the oracle run with that tile's box -- including
    proposals clamped onto an interior upper edge (rejected, then frozen)."""
    from smcdet_amd.kernel import SingleComponentMH
    d = golden("agg_m71_pieces.npz")
    data = d["data"]                                   # [2,2,8,8]
    pr = p_prior(8, 4, 4, 2, "partition")
    boxes = N_(pr.tile_boxes((2, 2), DEV))
    rng = np.random.default_rng(21)
    N, S, K = 64, 4, 20
    locs = np.empty((2, 2, N, S, 2), np.float32)
    for t in range(4):
        lo, hi = boxes[t, :2], boxes[t, 2:]
        locs.reshape(4, N, S, 2)[t] = lo + rng.random((N, S, 2)) * (hi - lo)
    # sources hugging the interior upper edges: h -> 8 in the top row, w -> 8 left column
    locs[0, :, :8, 0, 0] = 7.999
    locs[:, 0, 8:16, 1, 1] = 7.999
    fluxes = (1.0 + 9.0 * rng.random((2, 2, N, S))).astype(np.float32)
    counts = np.full((2, 2, N), float(S), np.float32)
    comp = rng.integers(0, S, (K, 2, 2, N)).astype(np.int32)
    comp[:3, 0, :, :8] = 0
    comp[:3, :, 0, 8:16] = 1
    uloc = rng.random((K, 2, 2, N, 2)).astype(np.float32)
    uloc[:3, 0, :, :8, 0] = 0.9999999                  # onto the upper edge 8
    uloc[:3, :, 0, 8:16, 1] = 0.9999999
    uflux = rng.random((K, 2, 2, N)).astype(np.float32)
    uacc = rng.random((K, 2, 2, N)).astype(np.float32)
    tau = np.full((2, 2), 0.3, np.float32)
    mh = SingleComponentMH(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    rp = {k: torch.as_tensor(v) for k, v in
          dict(comp=comp, uloc=uloc, uflux=uflux, uacc=uacc).items()}
    T_ = lambda x: torch.as_tensor(x, device=DEV)  # noqa: E731
    lo, fo, acc = mh.run(T_(data), T_(counts), T_(locs), T_(fluxes), T_(tau), prior=pr,
                         image_model=p_model(8), replay=rp, tile_boxes=T_(boxes))
    lo, fo = N_(lo), N_(fo)
    omh = O.MHParams(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    frozen = 0
    for t in range(4):
        h, w = divmod(t, 2)
        sl = lambda x: np.ascontiguousarray(x[:, h:h + 1, w:w + 1])  # noqa: E731
        ol, of, oa, loga, oacc = O.mh_sweep(
            data[h:h + 1, w:w + 1], counts[h:h + 1, w:w + 1], locs[h:h + 1, w:w + 1],
            fluxes[h:h + 1, w:w + 1], tau[h:h + 1, w:w + 1], o_prior(8, 4, 4, 2, boxes[t]),
            o_m71_model(8), omh, sl(comp), sl(uloc), sl(uflux), sl(uacc), trace=True)
        margin = np.abs(np.nan_to_num(loga - np.log(sl(uacc).astype(np.float64)), nan=1.0))
        clear = (margin > 1e-3).all(0)[0, 0]
        frozen += int(np.isnan(loga[-1]).sum())
        np.testing.assert_allclose(lo[h, w][clear], ol[0, 0][clear], rtol=0, atol=2e-5)
        np.testing.assert_allclose(fo[h, w][clear], of[0, 0][clear], rtol=3e-5, atol=1e-4)
        assert clear.mean() > 0.9
    assert frozen > 0  # some interior-edge hits froze their particle


def test_aggregate_partition_mode_padded_evidence():
    """Children sampled with partition boxes (pad 2 on the image's outer edges
    only), aggregated, against the single 16x16 tile with pad 2 -- the same
    prior.  On the boundary-star image, where the padded-tile ("tile" mode)
    aggregate is ~64 nats high, the log evidence agrees within 5 nats; counts
    within 0.6 or 3 pooled SE and flux within 3% as before.  3 seeds, 8192
    particles per count, K = 200."""
    from tests.test_gpu_aggregate import _agg_vs_big, count_tol
    img = torch.as_tensor(golden("agg_m71_pieces.npz")["image"], device=DEV)
    m = _agg_vs_big(img, pad=2, mode="partition")
    assert abs(m["agg_lz"] - m["big_lz"]) < 5.0, m
    assert abs(m["agg_count"] - m["big_count"]) < count_tol(m, 0.6), m
    assert abs(m["agg_flux"] / m["big_flux"] - 1) < 0.03, m
