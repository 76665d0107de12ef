"""tests/_stats.py on the two recorded C2 K = 100 targets (CPU, fixtures only).

Pins the facts the count-posterior gate's variance floor rests on: the
reference's 20 runs against the 648 float64 oracle runs put bin 2 (two
detectable stars, carried by the lower log Z mode) 4.2 pooled SE apart with the
20 runs' own variance, inside 3 SE once the reference side's per-run variance
is floored at the oracle's; the other bins and the pruned flux agree within
2 SE either way.  Total variation between a 20-run mean histogram and the
target is noise-dominated (0.077), which is why the TV gate is against the
648-run target only.
"""
import json
import os

import numpy as np

from tests._params import GOLDEN
from tests._stats import count_posterior_compare, hist_var


def _runs(which):
    with open(os.path.join(GOLDEN, f"stats_{which}.json")) as f:
        return json.load(f)["runs"]


def test_count_posterior_targets_agree_with_floor():
    ref, orc = _runs("c2_moderate_4096_k100"), _runs("c2_moderate_4096_k100_oracle")
    plain = count_posterior_compare(ref, orc)
    z = np.array(plain["bin_z"])
    assert abs(z[2]) > 4.0                       # the rare-bin underestimate
    assert np.all(np.abs(np.delete(z, 2)) < 2.0)
    assert abs(plain["pruned_flux_z"]) < 2.0
    assert 0.06 < plain["total_variation"] < 0.09
    # the gate's orientation (GPU runs = a, reference = b): the reference's
    # variance floored at the oracle's; here the oracle stands in for "a"
    floored = count_posterior_compare(orc, ref, var_floor=hist_var(orc))
    assert floored["max_abs_bin_z"] <= 3.0
    # and the oracle against itself: zero
    same = count_posterior_compare(orc, orc)
    assert same["total_variation"] == 0.0 and same["max_abs_bin_z"] == 0.0
