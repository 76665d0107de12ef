"""The drop-in distributions (smcdet_amd/distributions.py) against the
reference's own outputs: tests/golden/distributions.npz was written by
tests/golden/make_golden.py::gen_distributions from smcdet/distributions.py
(TruncatedDiagonalMVN :22-58 sampled with recorded uniforms, its log_prob and
log-mass in the box; TruncatedPareto :61-89 sampled and scored).  The drop-in
classes, fed the recorded uniforms, reproduce every value bit for bit (CPU,
float32)."""
import numpy as np
import torch

from smcdet_amd.distributions import DiscreteUniform, TruncatedDiagonalMVN, TruncatedPareto
from tests._params import M71, golden


def _t(d, k):
    return torch.from_numpy(np.ascontiguousarray(d[k]))


def test_truncated_mvn_loc_and_flux_match_reference_outputs():
    d = golden("distributions.npz")
    cases = (("loc", torch.tensor(0.1), -4 * torch.ones(2), torch.tensor([36.0, 36.0])),
             ("flux", 2.5 * torch.ones(1), M71["flux_lower"] * torch.ones(1),
              M71["flux_upper"] * torch.ones(1)))
    for name, sig, lb, ub in cases:
        dist = TruncatedDiagonalMVN(_t(d, name + "_mu"), sig, lb, ub)
        np.testing.assert_array_equal(dist.log_prob_in_box.numpy(), d[name + "_logZ"])
        x = dist.sample(u=_t(d, name + "_u"))
        np.testing.assert_array_equal(x.numpy(), d[name + "_x"])
        np.testing.assert_array_equal(dist.log_prob(_t(d, name + "_x")).numpy(),
                                      d[name + "_logprob_x"])


def test_truncated_pareto_matches_reference_outputs():
    d = golden("distributions.npz")
    tp = TruncatedPareto(M71["flux_alpha"], M71["flux_lower"], M71["flux_upper"])
    f = tp.sample([500], device="cpu", u=_t(d, "tpareto_u"))
    np.testing.assert_array_equal(f.numpy(), d["tpareto_x"])
    np.testing.assert_array_equal(tp.log_prob(_t(d, "tpareto_x")).numpy(), d["tpareto_logprob"])


def test_out_of_support_values_raise_as_the_reference():
    tp = TruncatedPareto(M71["flux_alpha"], M71["flux_lower"], M71["flux_upper"])
    try:
        tp.log_prob(torch.tensor([M71["flux_lower"] * 0.5]))
    except AssertionError:
        pass
    else:
        raise AssertionError("TruncatedPareto.log_prob accepted a value below its support")
    du = DiscreteUniform(0, 3)
    lp = du.log_prob(torch.tensor([0, 3, 4]))
    assert torch.isfinite(lp[:2]).all() and lp[2] == float("-inf")
    np.testing.assert_allclose(lp[:2].numpy(), np.log(0.25), rtol=1e-7)
