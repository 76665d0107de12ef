"""north_star's "log Z and ESS within 1%" at C2, resolved by sample size and
recomputable here: the per-run summaries of 65,536 GPU runs of SMCsampler at
C2 (final library, `SMCDET_LAW_DUMP=... python scripts/c2_law.py 65536` on an
MI355X; profiles/r06/law/) against every run of the float64 oracle target
(tests/golden/stats_c2_moderate_4096_k100_oracle.json).  The 95% interval of
each relative mean difference must lie inside +-1% (scripts/c2_law.py
`compare`), and the count posterior must meet the test_c2_count_posterior
gates (TV <= 0.05, every bin and the pruned flux within 3 SE)."""
import io
import json
import os
import sys
from contextlib import redirect_stdout

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DUMP = os.path.join(ROOT, "profiles", "r06", "law", "c2_law_65536.npz")


@pytest.mark.skipif(not os.path.exists(DUMP), reason="GPU law record not in this tree")
def test_c2_law_within_one_percent_against_the_oracle_target():
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import c2_law
    argv, sys.argv = sys.argv, ["c2_law.py", "--recompute", DUMP]
    try:
        buf = io.StringIO()
        with redirect_stdout(buf):
            c2_law.main()
    finally:
        sys.argv = argv
    out = json.loads(buf.getvalue())
    assert out["gpu_runs"] == 65536 and out["oracle_runs"] >= 5291
    res = out["vs_oracle"]
    for key in ("logZ", "final_ess", "iters"):
        lo, hi = res[key]["rel_diff_95"]
        assert -0.01 < lo and hi < 0.01, (key, res[key])
    cp = res["count_posterior"]
    assert cp["total_variation"] <= 0.05 and cp["max_abs_bin_z"] <= 3.0, cp
    assert abs(cp["pruned_flux_z"]) <= 3.0, cp
