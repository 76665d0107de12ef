"""Edge cases of the HIP path the reference's own runs do not exercise:
particle counts that do not fill the last workgroup, a single source,
non-power-of-two N through the division-based resampling path, a one-pixel
tile, and both resampling methods on multi-tile grids.  Each run must finish
at temperature 1 with finite evidence, valid ancestors and in-box states."""
import numpy as np
import pytest
import torch

from tests._params import M71, p_m71_mh, p_m71_model, p_m71_prior

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("H,S,N,method,tiles", [
    (8, 1, 37, "systematic", 1),
    (8, 3, 1000, "multinomial", 2),
    (16, 2, 777, "systematic", 2),
    (4, 2, 64, "systematic", 1),
])
def test_small_and_ragged_runs(H, S, N, method, tiles):
    from smcdet_amd.sampler import SMCsampler
    torch.manual_seed(H * 1000 + N)
    model = p_m71_model(H)
    truth = p_m71_prior(H, 0, 100)  # prior.py:46 indexes counts by the Poisson draw
    img = torch.empty(tiles * H, tiles * H, device=DEV)
    for a in range(tiles):
        for b in range(tiles):
            c, l, f = truth.sample(num_catalogs=1, device=DEV)
            img[a * H:(a + 1) * H, b * H:(b + 1) * H] = model.sample(l, f)[0, 0, :, :, 0]
    prior = p_m71_prior(H, S, S)
    s = SMCsampler(img, H, prior, model, p_m71_mh(20), N, 0.5, method,
                   M71["flux_detection_threshold"], 100, print_every=10 ** 9)
    s.run()
    assert bool((s.temperature == 1).all())
    assert bool(torch.isfinite(s.log_normalizing_constant).all())
    assert s.locs.shape == (tiles, tiles, N, S, 2)
    lo, hi = -4.0, H + 4.0
    assert float(s.locs.min()) >= lo and float(s.locs.max()) <= hi
    f = s.fluxes
    assert float(f.min()) >= np.float32(M71["flux_lower"]) * (1 - 1e-6)
    assert float(f.max()) <= np.float32(M71["flux_upper"]) * (1 + 1e-6)
    assert s.pruned_counts.max() <= S
    it = s.iters_per_tile
    assert int(it.min()) >= 0 and int(it.max()) == s.iter
