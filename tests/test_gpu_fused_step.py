"""The fused SMC step (smcdet_mh_sweep_step): the MH sweep's last workgroup
per tile runs temper -> reweight -> next resampling indices (tile.h) in the
same launch.  It plays the tile kernel's 512-thread layout on its 256
threads, so every temperature, weight, ESS, log Z and index equals the
two-launch path's bit for bit: checked here step by step and on whole runs
(C2 geometry at N = 4096 / 1024 / 512, a multi-tile grid, multinomial and
non-power-of-two systematic resampling, independent stopping through the
speculative loop).  The two-launch path itself is pinned to the reference by
the recorded-run replays (test_gpu_parity.py; its "mh-step" variant drives
the replay through SMCsampler._step, whose 8x8 tiles take the two-launch
form of smcdet_mh_sweep_step).
"""
import numpy as np
import pytest
import torch

from tests._params import M71, p_m71_mh, p_m71_model, p_m71_prior

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _image(H, seed, n_tiles=1):
    torch.manual_seed(seed)
    model = p_m71_model(H * n_tiles)
    truth = p_m71_prior(H * n_tiles, 0, 40, counts_rate=0.004)
    c, l, f = truth.sample(num_catalogs=1, device=DEV)
    return model.sample(l, f)[0, 0, :, :, 0].contiguous()


def _sampler(img, td, N, S, K, seed, method="systematic", stopping="lockstep", fused_step=True):
    from smcdet_amd.sampler import SMCsampler
    s = SMCsampler(img, td, p_m71_prior(td, S, S), p_m71_model(td), p_m71_mh(K), N, 0.5, method,
                   M71["flux_detection_threshold"], 200, print_every=10 ** 9, seed=seed,
                   device=DEV, stopping=stopping)
    s.fused_step = fused_step
    return s


def _state(s):
    keys = ("temperature", "temperature_prev", "log_normalizing_constant", "ess", "weights",
            "weights_log_unnorm", "locs", "fluxes", "counts", "loglik")
    out = {k: getattr(s, k).detach().cpu().numpy().copy() for k in keys}
    if s._pending_idx is not None:
        from smcdet_amd import _hip
        out["idx"] = _hip.as_index(s._pending_idx).cpu().numpy().copy()
    return out


def _steps(s, n):
    s.initialize()
    s._temper_reweight(with_resample=True)
    trace = []
    for _ in range(n):
        idx, s._pending_idx = s._pending_idx, None
        s._step(idx)
        torch.cuda.synchronize()
        trace.append(_state(s))
    return trace


def _assert_same(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        for k in x:
            np.testing.assert_array_equal(x[k], y[k], err_msg=f"step {i}: {k}")


@pytest.mark.parametrize("N", [4096, 1024, 512])
def test_fused_step_equals_split_step_c2(N):
    """C2 geometry (one 32x32 tile, S = 10, K = 100): every output of 6 SMC
    iterations is identical for the fused and the two-launch step.  A
    self-consistency regression, not parity evidence (the reference parity
    of the tile pass at N = 4096 is test_gpu_parity.py::
    test_tile_pass_4096_vs_reference)."""
    from smcdet_amd import _hip
    img = _image(32, 5)
    a = _sampler(img, 32, N, 10, 100, 77, fused_step=True)
    assert a._step_fusable()
    assert _hip.lib().smcdet_mh_sweep_step_fused(_hip.ref(a.ImageModel._cmodel()), N, 10, 0) == 1
    b = _sampler(img, 32, N, 10, 100, 77, fused_step=False)
    _assert_same(_steps(a, 6), _steps(b, 6))


def test_fused_step_equals_split_step_tiles_multinomial():
    """2x2 grid of 16x16 tiles, multinomial resampling, N = 768 (not a power
    of two: the systematic pass's general count path, masked slots)."""
    img = _image(16, 6, n_tiles=2)
    for method in ("multinomial", "systematic"):
        a = _sampler(img, 16, 768, 6, 40, 91, method=method, fused_step=True)
        b = _sampler(img, 16, 768, 6, 40, 91, method=method, fused_step=False)
        _assert_same(_steps(a, 5), _steps(b, 5))


def test_fused_run_equals_split_run_independent_stopping():
    """Whole runs to temperature 1 (speculative loop, independent stopping:
    finished tiles frozen by the tail's SMCDET_SMC_FREEZE_DONE path)."""
    img = _image(16, 8, n_tiles=2)
    res = []
    for fused in (True, False):
        s = _sampler(img, 16, 512, 6, 30, 5, stopping="independent", fused_step=fused)
        s.run()
        res.append((s.iter, s.iters_per_tile.cpu().numpy(), s.log_normalizing_constant.cpu().numpy(),
                    s.locs.cpu().numpy(), s.pruned_counts.cpu().numpy()))
    assert res[0][0] == res[1][0]
    for x, y in zip(res[0][1:], res[1][1:]):
        np.testing.assert_array_equal(x, y)


def test_small_tiles_take_the_two_launch_path():
    """8x8 tiles (the small-tile sweep at 7 waves per SIMD) cannot host the
    tile pass's buffer: smcdet_mh_sweep_step launches the tile kernel after
    the sweep, with the same results."""
    from smcdet_amd import _hip
    img = _image(8, 9, n_tiles=2)
    a = _sampler(img, 8, 1024, 10, 30, 3, fused_step=True)
    assert _hip.lib().smcdet_mh_sweep_step_fused(_hip.ref(a.ImageModel._cmodel()), 1024, 10, 0) == 0
    b = _sampler(img, 8, 1024, 10, 30, 3, fused_step=False)
    _assert_same(_steps(a, 4), _steps(b, 4))


def test_launch_timing_on_dispatch_events():
    """smcdet_launch_timing (bench.py's kernel time): each timed sweep launch
    of the two-launch step gets its own positive duration, the pool stops at
    its size, and timing leaves the results unchanged."""
    from smcdet_amd import _hip
    img = _image(32, 5)
    a = _sampler(img, 32, 1024, 10, 50, 77, fused_step=False)
    b = _sampler(img, 32, 1024, 10, 50, 77, fused_step=False)
    _hip.launch_timing(2)
    try:
        ta = _steps(a, 3)
        ms = _hip.launch_timing_read(3)
    finally:
        _hip.launch_timing(0)
    assert len(ms) == 2 and all(0.0 < x < 1000.0 for x in ms)
    _assert_same(ta, _steps(b, 3))


@pytest.mark.parametrize("stopping,N,fused", [("lockstep", 1024, False),
                                              ("independent", 1024, False),
                                              ("lockstep", 1000, False),
                                              ("lockstep", 1001, False),
                                              ("independent", 1024, True)])
def test_ancestor_bins_equal_indices(stopping, N, fused):
    """The step's tile pass hands the next systematic resampling to the next
    sweep as bins + offset (AncestorBins, ABI 16), whose waves search their
    own ancestors: the same indices and the same run, bit for bit, as the
    int64 index hand-over (SMCsampler.ancestor_bins = False); N = 1000: the
    search's division form for N not a power of two; N = 1001: bins_out + t*N
    not 16-byte aligned (the tile pass's scalar store path);
    fused: the bins written by the sweep's in-kernel tail (one launch)."""
    from smcdet_amd.sampler import SMCsampler
    out = []
    for bins in (True, False):
        torch.manual_seed(3)
        H = 32
        s = SMCsampler(_image(H, 5), H, p_m71_prior(H, 10, 10, counts_rate=0.003125),
                       p_m71_model(H), p_m71_mh(30), N, 0.5, "systematic",
                       M71["flux_detection_threshold"], 200, print_every=10 ** 9, seed=21,
                       device=DEV, stopping=stopping)
        s.ancestor_bins = bins
        s.fused_step = fused
        s.run()
        torch.cuda.synchronize()
        out.append({k: getattr(s, k).detach().cpu().numpy().copy()
                    for k in ("temperature", "log_normalizing_constant", "ess", "locs", "fluxes",
                              "counts", "weights")} | {"iter": np.array(s.iter)})
    assert out[0]["iter"] >= 5
    for k in out[0]:
        np.testing.assert_array_equal(out[0][k], out[1][k], err_msg=k)


@pytest.mark.parametrize("N", [4096, 1000, 7, 64, 65, 16384])
def test_bins_index_vs_oracle(N):
    """smcdet_bins_index (the sweep's 64-ary ancestor search, its first level
    from the chunk-end array) against the oracle's bucketize of the same
    weights and offsets: random, degenerate (one particle, a block of zero
    weights) and uniform weights."""
    from oracle import smc_oracle as O
    from smcdet_amd import _hip
    rng = np.random.default_rng(N)
    W = np.stack([rng.random(N), np.eye(1, N, rng.integers(N))[0],
                  np.where(np.arange(N) % 7 < 3, 0.0, rng.random(N)), np.ones(N)])
    W = (W / W.sum(1, keepdims=True)).astype(np.float32)
    T = W.shape[0]
    U = rng.random(T).astype(np.float32)
    U[-1] = 0.0  # an offset of exactly 0
    bins = np.cumsum(W.astype(np.float64), axis=1).astype(np.float32)  # the tile pass's bins
    # the first search level's chunk ends (ABI 17): entry l = bins[min((l+1)c, N) - 1]
    c = -(-N // 64)
    ends = np.minimum((np.arange(64) + 1) * c, N) - 1
    coarse = bins[:, ends]
    buf = torch.tensor(np.concatenate([bins.ravel(), U, coarse.ravel()]), device=DEV)
    idx = torch.empty(T, N, device=DEV, dtype=torch.int64)
    _hip.check(_hip.lib().smcdet_bins_index(_hip.ptr(buf), T, N, _hip.ptr(idx),
                                            _hip.stream_of(idx)), "bins_index")
    ref = O.systematic_resample_index(W.reshape(1, T, N), U.reshape(1, T)).reshape(T, N)
    np.testing.assert_array_equal(idx.cpu().numpy(), ref)
