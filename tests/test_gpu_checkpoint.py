"""Checkpoint / resume and the progress lines of the speculative
SMC loop."""
import contextlib
import io

import pytest
import torch

from tests._params import M71, p_m71_mh, p_m71_model, p_m71_prior

pytestmark = pytest.mark.gpu
H, S, N, K = 16, 4, 256, 20


def _image():
    torch.manual_seed(3)
    model = p_m71_model(H)
    c, l, f = p_m71_prior(H, 0, 100, counts_rate=0.01).sample(num_catalogs=1, device="cuda")
    return model.sample(l, f)[0, 0, :, :, 0]


def _sampler(img, seed=5, print_every=10 ** 9):
    from smcdet_amd.sampler import SMCsampler
    return SMCsampler(img, H, p_m71_prior(H, S, S), p_m71_model(H), p_m71_mh(K), N, 0.5,
                      "systematic", M71["flux_detection_threshold"], 200,
                      print_every=print_every, seed=seed)


RESULTS = ("counts", "locs", "fluxes", "weights", "ess", "log_normalizing_constant",
           "temperature", "pruned_counts", "pruned_locs", "pruned_fluxes", "iters_per_tile")


@pytest.mark.parametrize("with_rate", [True, False])
def test_resume_from_checkpoint(with_rate):
    """state_dict() taken after SMC iteration 6 of a run, loaded into a fresh
    sampler and resumed: the same result as the uninterrupted run -- bit for
    bit with the rate images in the checkpoint; without them the resumed
    sweep re-renders its rate images (float32 rounding differs from the
    incrementally maintained ones), so only the run's course is compared."""
    img = _image()
    saved = {}
    a = _sampler(img)

    def hook(s):
        if s.iter == 6:
            saved["st"] = s.state_dict(with_rate_images=with_rate)

    a.on_iteration = hook
    with contextlib.redirect_stdout(io.StringIO()):
        a.run()
    st = saved["st"]
    assert st["iter"] == 6 and ("rate_image" in st) == with_rate
    # the checkpoint is a copy: the run went on without changing it
    assert not torch.equal(st["temperature"], a.temperature)

    b = _sampler(img, seed=999)  # the seed comes from the checkpoint's stream state
    b.load_state_dict(st)
    with contextlib.redirect_stdout(io.StringIO()):
        b.resume()
    assert b.iter == a.iter
    if with_rate:
        for k in RESULTS:
            assert torch.equal(getattr(a, k), getattr(b, k)), k
    else:
        assert float(b.temperature.min()) == 1.0
        assert abs(float(b.log_normalizing_constant) - float(a.log_normalizing_constant)) < \
            0.05 * abs(float(a.log_normalizing_constant))


def test_uninterrupted_run_equals_speculative_run():
    """on_iteration forces the synchronous loop; the default run() enqueues
    iterations speculatively.  Same draws, same result."""
    img = _image()
    a, b = _sampler(img), _sampler(img)
    b.on_iteration = lambda s: None
    with contextlib.redirect_stdout(io.StringIO()):
        a.run()
        b.run()
    for k in RESULTS:
        assert torch.equal(getattr(a, k), getattr(b, k)), k


def test_progress_lines_match_synchronous_loop():
    """The speculative loop prints an iteration's progress line only once the
    iteration is known to run (the reference prints after its loop check), with
    the values of the previous iteration: the same lines as the synchronous
    loop, and none for the rolled-back no-op iteration."""
    img = _image()
    outs = []
    for sync in (False, True):
        s = _sampler(img, print_every=2)
        if sync:
            s.on_iteration = lambda s: None
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            s.run()
        outs.append([ln for ln in buf.getvalue().splitlines() if ln.startswith("iteration")])
        last = s.iter
    assert outs[0] == outs[1]
    assert len(outs[0]) == last // 2


def test_fused_resume_from_unfused_checkpoint():
    """a checkpoint taken from a fused=False run carries no pending
    resampling indices; loading it into a fused sampler draws them from the
    restored weights at the stream offset the unfused resample() would use,
    so the resumed fused run ends exactly where the uninterrupted unfused run
    does (rate images off in both: the fused and unfused schedules then
    consume the same draws in the same order)."""
    from smcdet_amd.sampler import SMCsampler
    img = _image()

    def make(fused, seed=5):
        return SMCsampler(img, H, p_m71_prior(H, S, S), p_m71_model(H), p_m71_mh(K), N, 0.5,
                          "systematic", M71["flux_detection_threshold"], 200,
                          print_every=10 ** 9, seed=seed, fused=fused, persist_rate_images=False)

    saved = {}
    a = make(False)

    def hook(s):
        if s.iter == 4:
            saved["st"] = s.state_dict(with_rate_images=False)

    a.on_iteration = hook
    with contextlib.redirect_stdout(io.StringIO()):
        a.run()
    st = saved["st"]
    assert "_pending_idx" not in st
    b = make(True, seed=999)
    b.load_state_dict(st)
    assert b._pending_idx is not None
    with contextlib.redirect_stdout(io.StringIO()):
        b.resume()
    assert b.iter == a.iter
    for k in ("log_normalizing_constant", "temperature", "pruned_counts", "locs", "fluxes"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
