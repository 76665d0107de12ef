"""The aggregation oracle (oracle/agg_oracle.py) against the pieces of the
reference's Aggregate that run at HEAD (tests/golden/agg_m71_pieces.npz,
make_golden.py gen_agg): drop_sources_from_overlap, join, unjoin, log_target,
sort_by_count, temper and update_weights (smcdet/aggregate.py:105-483), on
synthetic count-varying populations over a 2x2 grid of 8x8 M71 tiles."""
import numpy as np
import pytest

from oracle import agg_oracle as A
from oracle import smc_oracle as O
from tests._params import M71, golden

G = golden("agg_m71_pieces.npz")


def joint_model(axis):
    H, W = (16, 8) if axis == 0 else (8, 16)
    p = M71
    return O.M71Model(H, W, p["background"], p["psf_radius"], p["adu_per_nmgy"], p["psf_params"],
                      p["noise_additive"], p["noise_multiplicative"])


def joint_prior(axis, smax):
    H, W = (16, 8) if axis == 0 else (8, 16)
    p = M71
    return O.M71PriorP(0, smax, p["counts_rate"], H, W, 4, p["flux_alpha"], p["flux_lower"],
                       p["flux_upper"])


def compact_ref(locs, fluxes):
    """The reference zeroes dropped sources in place: compact by flux != 0."""
    keep = fluxes != 0
    _, l, f = A.compact(keep, locs, fluxes)
    return l, f


@pytest.mark.parametrize("axis", [0, 1])
def test_drop_sources_from_overlap(axis):
    c, l, f = A.drop_sources_from_overlap(axis, G["counts"], G["locs"], G["fluxes"], 8)
    np.testing.assert_array_equal(c, G[f"drop{axis}_counts"])
    rl, rf = compact_ref(G[f"drop{axis}_locs"], G[f"drop{axis}_fluxes"])
    np.testing.assert_array_equal(l, rl)
    np.testing.assert_array_equal(f, rf)
    # something was dropped on both sides of the shared boundary
    assert (c < G["counts"]).any()


@pytest.mark.parametrize("axis", [0, 1])
def test_join(axis):
    c, l, f = A.drop_sources_from_overlap(axis, G["counts"], G["locs"], G["fluxes"], 8)
    d, jc, jl, jf = A.join(axis, G["data"], c, l, f, 8)
    np.testing.assert_array_equal(d, G[f"join{axis}_data"])
    np.testing.assert_array_equal(jc, G[f"join{axis}_counts"])
    np.testing.assert_allclose(jl, G[f"join{axis}_locs"], rtol=0, atol=0)
    np.testing.assert_array_equal(jf, G[f"join{axis}_fluxes"])
    assert jl.shape[-2] == max(1, int(jc.max()))


@pytest.mark.parametrize("axis", [0, 1])
def test_unjoin_inverts_join(axis):
    d, jc, jl, jf = (G[f"join{axis}_{k}"] for k in ("data", "counts", "locs", "fluxes"))
    ud, uc, ul, uf = A.unjoin(axis, d, jc, jl, jf, 16)
    np.testing.assert_array_equal(ud, G[f"unjoin{axis}_data"])
    np.testing.assert_array_equal(uc, G[f"unjoin{axis}_counts"])
    np.testing.assert_allclose(ul, G[f"unjoin{axis}_locs"], rtol=0, atol=2e-6)
    np.testing.assert_array_equal(uf, G[f"unjoin{axis}_fluxes"])
    np.testing.assert_array_equal(ud, G["data"])  # the children are the original tiles


@pytest.mark.parametrize("axis", [0, 1])
def test_log_target(axis):
    d, jc, jl, jf = (G[f"join{axis}_{k}"] for k in ("data", "counts", "locs", "fluxes"))
    lt = A.agg_log_target(d, jc, jl, jf, G[f"logtarget{axis}_tau"], joint_prior(axis, jl.shape[-2]),
                          joint_model(axis), axis)
    ref = G[f"logtarget{axis}"]
    # float64 restatement vs the reference's float32 sums over 128 pixels
    np.testing.assert_allclose(lt, ref, rtol=2e-6, atol=2e-3)


@pytest.mark.parametrize("axis", [0, 1])
def test_loglik_diff_and_groups(axis):
    d = G[f"join{axis}_data"]
    c, l, f = (G[f"sorted{axis}_{k}"] for k in ("counts", "locs", "fluxes"))
    lp, lc = A.parent_child_loglik(d, c, l, f, joint_model(axis), axis)
    np.testing.assert_allclose(lp - lc, G[f"loglik_diff{axis}"], rtol=1e-5, atol=5e-3)
    oc, _, _, groups = A.sort_by_count(G[f"join{axis}_counts"], G[f"join{axis}_locs"],
                                       G[f"join{axis}_fluxes"])
    np.testing.assert_array_equal(oc, c)
    ref_groups = G[f"groups{axis}"]
    for h in range(oc.shape[0]):
        for w in range(oc.shape[1]):
            g = ref_groups[h, w]
            assert groups[h][w] == g[g > 0].tolist()


@pytest.mark.parametrize("axis", [0, 1])
def test_temper_and_update_weights(axis):
    """Two tempering steps over the count groups: the tile increment (the
    minimum of the groups' brentq roots), within-group weights, group log
    evidences and the overall weights of the reference."""
    ref_groups = G[f"groups{axis}"]
    groups = [[g[g > 0].tolist() for g in row] for row in ref_groups]
    lnc = [[G[f"lnc_in{axis}"][h, w][:len(groups[h][w])].tolist()
            for w in range(len(groups[h]))] for h in range(len(groups))]
    tau = np.zeros(ref_groups.shape[:2], np.float32)
    for step, key in ((1, f"loglik_diff{axis}"), (2, f"loglik_diff{axis}_2")):
        ld = G[key]
        new_tau, _ = A.temper_groups(ld, groups, tau, 0.5)
        np.testing.assert_allclose(new_tau, G[f"tau{axis}_{step}"], rtol=0, atol=2e-6)
        wi, W, lnc = A.update_weights_groups(ld, groups, new_tau, tau, lnc)
        np.testing.assert_allclose(wi, G[f"w_intra{axis}_{step}"], rtol=2e-4, atol=1e-7)
        np.testing.assert_allclose(W, G[f"weights{axis}_{step}"], rtol=2e-4, atol=1e-7)
        for h in range(len(groups)):
            for w in range(len(groups[h])):
                np.testing.assert_allclose(lnc[h][w],
                                           G[f"lnc{axis}_{step}"][h, w][:len(groups[h][w])],
                                           rtol=1e-6, atol=1e-3)
        tau = new_tau


def test_merge_log_evidence():
    """Repaired merge (aggregate.py:362-422): group j of the
    joined population gets log Z_c1 + log Z_c2 + log(n_j / N), so the
    groups' evidences sum (in probability) to the product of the children's."""
    lnc_children = [[[-10.0, -12.0], [-11.0]], [[-9.5], [-13.0, -13.5, -20.0]]]
    counts = np.array([[[0, 0, 1, 2, 2, 2, 3, 3], [1, 1, 1, 1, 2, 2, 2, 5]]], np.float32)
    out = A.merge_log_evidence(lnc_children, counts, axis=0)

    def lse(v):
        v = np.asarray(v)
        return v.max() + np.log(np.exp(v - v.max()).sum())
    for w in range(2):
        tot = lse(lnc_children[0][w]) + lse(lnc_children[1][w])
        np.testing.assert_allclose(lse(out[0][w]), tot, rtol=0, atol=1e-9)
        assert len(out[0][w]) == len(np.unique(counts[0, w]))


def test_agg_mh_sweep_moves_only_present_sources():
    """Replayed sweep at a joint 16x8 tile: components past the count never
    move; count-0 particles stay put; accepted moves change the target."""
    axis = 0
    d, jc, jl, jf = (G[f"join{axis}_{k}"] for k in ("data", "counts", "locs", "fluxes"))
    d, jc, jl, jf = d[:, :, ...], jc[:, :, :8], jl[:, :, :8], jf[:, :, :8]
    rng = np.random.default_rng(1)
    K = 12
    S = jl.shape[-2]
    comp = np.minimum((rng.random((K,) + jc.shape) * np.maximum(jc, 1)).astype(np.int32),
                      np.maximum(jc, 1).astype(np.int32) - 1)
    uloc = rng.random((K,) + jc.shape + (2,)).astype(np.float32)
    uflux = rng.random((K,) + jc.shape).astype(np.float32)
    uacc = rng.random((K,) + jc.shape).astype(np.float32)
    mh = O.MHParams(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    l2, f2, acc, _ = A.agg_mh_sweep(d, jc, jl, jf, np.full(jc.shape[:2], 0.4, np.float32),
                                 joint_prior(axis, S), joint_model(axis), axis, mh, comp, uloc,
                                 uflux, uacc, trace=True)
    past = ~A.present(jc, S)
    np.testing.assert_array_equal(l2[past], jl[past])
    np.testing.assert_array_equal(f2[past], jf[past])
    np.testing.assert_array_equal(l2[jc == 0], jl[jc == 0])
    assert acc.any() and not acc.all()
