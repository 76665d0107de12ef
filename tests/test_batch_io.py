"""Batch result files (smcdet_amd.batch): the layout the reference's drivers
write with torch.save (experiments/m71/run_smc.py:173-181), read back with
weights_only loading.  CPU only (no kernels)."""
import os

import torch

from smcdet_amd.batch import RESULT_FIELDS, load_batch_results, save_batch_results


def test_save_load_round_trip(tmp_path):
    B, N, S = 3, 16, 4
    g = torch.Generator().manual_seed(0)
    res = {"runtime": torch.rand(B, generator=g), "num_iters": torch.tensor([5.0, 7.0, 6.0]),
           "counts": torch.randint(0, S + 1, (B, N), generator=g).float(),
           "locs": torch.rand(B, N, S, 2, generator=g), "fluxes": torch.rand(B, N, S, generator=g),
           "posterior_predictive_total_flux": torch.rand(B, N, generator=g),
           "log_normalizing_constant": torch.randn(B, generator=g)}
    paths = save_batch_results(res, str(tmp_path), 4)
    names = sorted(os.path.basename(p) for p in paths)
    # the reference drivers' file names for batch index 4
    for f in RESULT_FIELDS:
        assert f"{f}_4.pt" in names
    back = load_batch_results(str(tmp_path), 4, fields=tuple(res))
    for k, v in res.items():
        assert torch.equal(back[k], v), k
