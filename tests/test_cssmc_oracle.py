"""Count-stratified SMC (manuscript.tex:314-356): the oracle's combination
step against the reference's own fixed-count runs (tests/golden/stats_cssmc.json,
make_golden.py cssmc), and the host-side count prior.  CPU only."""
import json
import os

import numpy as np
import pytest

from oracle import smc_oracle as O
from tests._params import GOLDEN, o_basic_prior, o_m71_prior, p_basic_prior, p_m71_prior

STATS = os.path.join(GOLDEN, "stats_cssmc.json")


def _stats():
    if not os.path.exists(STATS):
        pytest.skip("stats_cssmc.json not generated")
    with open(STATS) as f:
        return json.load(f)


def test_log_count_prior_matches_reference_poisson():
    d = _stats()
    cfg = d["config"]
    lp = O.log_count_prior(o_m71_prior(8, cfg["smin"], cfg["smax"]))
    np.testing.assert_allclose(lp, cfg["log_count_prior"], rtol=1e-6, atol=1e-6)


def test_product_log_count_prior_matches_oracle():
    from smcdet_amd.cssmc import log_count_prior
    np.testing.assert_allclose(log_count_prior(p_m71_prior(8, 0, 6)).numpy(),
                               O.log_count_prior(o_m71_prior(8, 0, 6)), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(log_count_prior(p_basic_prior(16, 1, 3)).numpy(),
                               O.log_count_prior(o_basic_prior(16, 1, 3)), rtol=1e-6)


def test_count_posterior_reproduces_reference_runs():
    d = _stats()
    lp = np.array(d["config"]["log_count_prior"])
    for r in d["runs"]:
        np.testing.assert_allclose(O.count_posterior(np.array(r["logZ"]), lp),
                                   r["count_posterior"], rtol=1e-12, atol=1e-15)
    # the empty-catalog stratum: log Z_0 is the likelihood of the background alone
    assert all(r["logZ"][0] == d["config"]["loglik_empty"] for r in d["runs"])


def test_count_posterior_draw_systematic_allocation():
    rng = np.random.default_rng(0)
    T, NS, N, n_out = 4, 5, 64, 1000
    probs = O.count_posterior(rng.normal(0, 2, (T, NS)), np.zeros(NS))
    idx = O.count_posterior_draw(probs, rng.random(T).astype(np.float32),
                                 rng.random((T, n_out)).astype(np.float32), N)
    k = idx // N
    for t in range(T):
        c = np.bincount(k[t], minlength=NS)
        # systematic resampling: each stratum gets floor or ceil of n_out * p
        assert np.all(np.abs(c - n_out * probs[t]) <= 1.0 + 1e-9), (c, n_out * probs[t])
        assert np.all(np.diff(k[t]) >= 0)
    assert idx.min() >= 0 and idx.max() < NS * N
