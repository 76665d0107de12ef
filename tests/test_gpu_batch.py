"""Batched independent images on the GPU (smcdet_amd.batch).

* Independent stopping changes only what happens to an image after it has
  reached temperature 1: with the same seed, lockstep and independent runs
  draw identical random streams, so every image's log Z and finishing
  iteration agree exactly, and the last image to finish has bit-identical
  particles; images that finished earlier are frozen (independent) or keep
  being mutated at temperature 1 (lockstep).
* A batch of copies of the reference's statistics image reproduces the
  reference's single-image log Z distribution (20 reference runs).
"""
import json
import os

import numpy as np
import pytest
import torch

from tests._params import GOLDEN, M71, p_m71_mh, p_m71_model, p_m71_prior

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _images(B, H, seed):
    torch.manual_seed(seed)
    model = p_m71_model(H)
    truth = p_m71_prior(H, 0, 20)
    ims = []
    for b in range(B):
        c, l, f = truth.sample(num_catalogs=1, device=DEV)
        ims.append(model.sample(l, f)[0, 0, :, :, 0])
    return torch.stack(ims)


def _run(images, stopping, seed, N=256, K=20, S=4):
    from smcdet_amd.batch import BatchSMC
    H = images.shape[-1]
    bs = BatchSMC(images, p_m71_prior(H, S, S), p_m71_model(H), p_m71_mh(K), N, 0.5,
                  "systematic", M71["flux_detection_threshold"], 100, stopping=stopping,
                  seed=seed, device=DEV)
    return bs.run()


def test_independent_vs_lockstep_same_streams():
    images = _images(6, 8, 3)
    a = _run(images, "lockstep", 11)
    b = _run(images, "independent", 11)
    ra, rb = a.results(), b.results()
    assert a.sampler.iter == b.sampler.iter
    np.testing.assert_array_equal(ra["num_iters"].cpu().numpy(), rb["num_iters"].cpu().numpy())
    np.testing.assert_array_equal(ra["log_normalizing_constant"].cpu().numpy(),
                                  rb["log_normalizing_constant"].cpu().numpy())
    it = rb["num_iters"].cpu().numpy()
    assert it.min() >= 0 and it.max() == a.sampler.iter
    last = np.nonzero(it == it.max())[0]
    early = np.nonzero(it < it.max())[0]
    for t in last:
        assert torch.equal(ra["locs"][t], rb["locs"][t])
    # finished images kept being mutated in lockstep mode only
    for t in early:
        assert not torch.equal(ra["locs"][t], rb["locs"][t])
    assert bool((b.sampler.temperature == 1).all())


def test_batch_logz_matches_reference_stats():
    with open(os.path.join(GOLDEN, "stats_m71.json")) as f:
        ref = json.load(f)
    cfg = ref["config"]
    img = torch.tensor(ref["image"], dtype=torch.float32, device=DEV)
    lz = []
    for seed in range(3):
        images = img[None].repeat(10, 1, 1).contiguous()
        bs = _run(images, "independent", 100 + seed, N=cfg["N"], K=cfg["K"], S=cfg["S"])
        r = bs.results()
        lz += r["log_normalizing_constant"].cpu().tolist()
        assert r["counts"].shape == (10, cfg["N"])
        assert r["posterior_predictive_total_flux"].shape == (10, cfg["N"])
    lz = np.array(lz)
    lz_ref = np.array([r["logZ"] for r in ref["runs"]])
    se = np.sqrt(lz.var(ddof=1) / len(lz) + lz_ref.var(ddof=1) / len(lz_ref))
    assert abs(lz.mean() - lz_ref.mean()) <= 3 * se, (lz.mean(), lz_ref.mean(), se)
    assert abs(lz.mean() - lz_ref.mean()) <= 0.01 * abs(lz_ref.mean())


def test_speculative_loop_equals_synchronous_loop():
    """SMCsampler.run() enqueues each SMC iteration before reading the
    previous loop condition (kernels predicated on the device-side count of
    unfinished tiles) and rolls back the one no-op iteration at the end: the
    result must equal the synchronous loop's exactly."""
    from smcdet_amd.sampler import SMCsampler
    images = _images(4, 8, 7)
    outs = []
    for speculative in (True, False):
        s = SMCsampler.from_tiles(images.reshape(1, 4, 8, 8), p_m71_prior(8, 4, 4),
                                  p_m71_model(8), p_m71_mh(20), 256, 0.5, "systematic",
                                  M71["flux_detection_threshold"], 100, print_every=10 ** 9,
                                  seed=13, device=DEV)
        if not speculative:
            s._keep_going = s._keep_going  # an instance hook selects the synchronous loop
        assert s._can_speculate() == speculative
        s.run()
        outs.append(s)
    a, b = outs
    assert a.iter == b.iter
    for k in ("locs", "fluxes", "counts", "log_normalizing_constant", "temperature", "ess",
              "weights", "pruned_counts", "iters_per_tile"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    assert a.rng.offset == b.rng.offset
