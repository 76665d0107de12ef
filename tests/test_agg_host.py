"""Host-side catalog bookkeeping of smcdet_amd.aggregate (drop / join /
unjoin as torch ops, run once per aggregation level) against the oracle and
the reference's own outputs (tests/golden/agg_m71_pieces.npz)."""
import numpy as np
import pytest
import torch

from oracle import agg_oracle as A
from smcdet_amd.aggregate import compact, drop_overlap, join_tiles, unjoin_tiles
from tests._params import golden

G = golden("agg_m71_pieces.npz")


def T(x):
    return torch.as_tensor(np.asarray(x))


@pytest.mark.parametrize("axis", [0, 1])
def test_drop_join_unjoin_match_reference(axis):
    c, l, f = drop_overlap(axis, T(G["locs"]), T(G["fluxes"]), 8)
    np.testing.assert_array_equal(c.numpy(), G[f"drop{axis}_counts"])
    d, jc, jl, jf = join_tiles(axis, T(G["data"]), l, f, 8)
    smax = max(1, int(jc.max()))
    np.testing.assert_array_equal(d.numpy(), G[f"join{axis}_data"])
    np.testing.assert_array_equal(jc.numpy(), G[f"join{axis}_counts"])
    np.testing.assert_array_equal(jl[..., :smax, :].numpy(), G[f"join{axis}_locs"])
    np.testing.assert_array_equal(jf[..., :smax].numpy(), G[f"join{axis}_fluxes"])
    ud, uc, ul, uf = unjoin_tiles(axis, d, jl[..., :smax, :], jf[..., :smax], 16)
    np.testing.assert_array_equal(ud.numpy(), G[f"unjoin{axis}_data"])
    np.testing.assert_array_equal(uc.numpy(), G[f"unjoin{axis}_counts"])
    np.testing.assert_allclose(ul.numpy(), G[f"unjoin{axis}_locs"], rtol=0, atol=2e-6)
    np.testing.assert_array_equal(uf.numpy(), G[f"unjoin{axis}_fluxes"])


@pytest.mark.parametrize("axis", [0, 1])
def test_multi_joint_grid_matches_oracle(axis):
    """A 4x4 grid (two joint tiles along the axis): the torch bookkeeping and
    the oracle agree, and unjoin pairs each joint tile with its own children
    (the layout the reference gets wrong)."""
    rng = np.random.default_rng(3 + axis)
    N, S = 16, 3
    counts = rng.integers(0, S + 1, (4, 4, N)).astype(np.float32)
    mask = A.present(counts, S)
    locs = (rng.uniform(-4, 12, (4, 4, N, S, 2)) * mask[..., None]).astype(np.float32)
    fluxes = (rng.uniform(0.5, 9, (4, 4, N, S)) * mask).astype(np.float32)
    data = rng.normal(100, 5, (4, 4, 8, 8)).astype(np.float32)
    oc, ol, of = A.drop_sources_from_overlap(axis, counts, locs, fluxes, 8)
    c, l, f = drop_overlap(axis, T(locs), T(fluxes), 8)
    np.testing.assert_array_equal(c.numpy(), oc)
    np.testing.assert_array_equal(l.numpy(), ol)
    od, ojc, ojl, ojf = A.join(axis, data, oc, ol, of, 8)
    d, jc, jl, jf = join_tiles(axis, T(data), l, f, 8)
    smax = ojl.shape[-2]
    np.testing.assert_array_equal(d.numpy(), od)
    np.testing.assert_array_equal(jc.numpy(), ojc)
    np.testing.assert_array_equal(jl[..., :smax, :].numpy(), ojl)
    ud, uc, ul, uf = unjoin_tiles(axis, d, jl[..., :smax, :], jf[..., :smax], 16)
    oud, ouc, oul, ouf = A.unjoin(axis, od, ojc, ojl, ojf, 16)
    np.testing.assert_array_equal(ud.numpy(), oud)
    np.testing.assert_array_equal(ud.numpy(), data)  # children back at their own positions
    np.testing.assert_array_equal(uc.numpy(), ouc)
    np.testing.assert_allclose(ul.numpy(), oul, rtol=0, atol=1e-6)
    # every kept source of child (i, j) comes back to child (i, j)
    np.testing.assert_array_equal(np.sort(uf.numpy(), -1)[..., -S:], np.sort(of, -1))
    assert (np.sort(uf.numpy(), -1)[..., :-S] == 0).all()


def test_compact_is_stable():
    keep = torch.tensor([[False, True, False, True, True]])
    locs = torch.arange(10, dtype=torch.float32).reshape(1, 5, 2)
    fl = torch.tensor([[1.0, 2.0, 3.0, 4.0, 5.0]])
    c, l, f = compact(keep, locs, fl)
    assert c.tolist() == [3.0]
    assert f.tolist() == [[2.0, 4.0, 5.0, 0.0, 0.0]]
    assert l[0, :3, 0].tolist() == [2.0, 6.0, 8.0]
