"""The MH sweep's PSF window cache (smcdet_mh_t.psf_cache, ABI 16) is an
evaluation shortcut, not an approximation: a moved source's old PSF is loaded
from the window the sweep stored when the source reached its location, and
that value is the one it would recompute (same psf_raw arithmetic at the same
arguments).  So every output of a sweep -- states, log-likelihoods, rate
images, acceptance -- must be bit-identical with and without the cache, for
the slot variants the geometry selects (tile sizes, window clipping at the
tile edges, anchors that move, jumps beyond the register slots), with
ancestor gathers and count-stratified component draws.  The reference's own
decisions are checked with the cache on by every replay test
(test_gpu_parity.py, test_gpu_teacher.py), since it is the default."""
import pytest
import torch

from smcdet_amd._rng import PhiloxStream
from tests._params import M71, p_m71_mh, p_m71_model, p_m71_prior

pytestmark = pytest.mark.gpu


def _state(H, S, N, seed, dev, spread=8):
    g = torch.Generator().manual_seed(seed)
    counts = torch.full((1, 1, N), float(S), device=dev)
    locs = (torch.rand(1, 1, N, S, 2, generator=g) * (H + spread) - spread / 2).to(dev)
    al, lo, hi = M71["flux_alpha"], M71["flux_lower"], M71["flux_upper"]
    u = torch.rand(1, 1, N, S, generator=g, dtype=torch.float64)
    fl = ((hi ** al - u * hi ** al + u * lo ** al) / (lo ** al * hi ** al)) ** (-1 / al)
    return counts, locs, fl.float().clamp(lo, hi).to(dev)


def _image(H, dev, seed=3):
    model = p_m71_model(H)
    truth = p_m71_prior(H, 4, 4)
    torch.manual_seed(seed)
    c, l, f = truth.sample(num_catalogs=1, device=dev)
    return model, model.sample(l, f)[0, 0, :, :, 0].reshape(1, 1, H, H).contiguous()


def _sweep(cache, img, model, prior, counts, locs, fluxes, tau, K, locs_stdev, *, rate_in=None,
           ancestors=None, by_count=False, seed=5):
    mh = p_m71_mh(K)
    mh.locs_stdev = torch.tensor(locs_stdev)
    mh.psf_cache = cache
    mh.component_by_count = by_count
    mh.rng = PhiloxStream(seed)
    H = img.shape[-1]
    r_out = torch.empty(1, 1, locs.shape[2], H * H, device=locs.device)
    out = mh.run(img, counts, locs, fluxes, tau, prior=prior, image_model=model, rate_in=rate_in,
                 rate_out=r_out, ancestors=ancestors)
    return out, r_out, mh


@pytest.mark.parametrize("H,S,N,K,sd", [
    (32, 10, 1024, 100, 0.1),   # C2 geometry (register render, 5-slot union windows)
    (32, 10, 512, 40, 1.5),     # anchors move on most proposals: union windows, 6 slots
    (16, 15, 512, 60, 0.1),     # 16x16 tiles (4 px per lane), S = 15 (the map's limit)
    (48, 6, 256, 40, 3.0),      # LDS-render instantiation; jumps beyond the register slots
    (12, 3, 256, 50, 0.7),      # windows clipped on every side
])
def test_psf_cache_bit_identical(H, S, N, K, sd):
    dev = torch.device("cuda", 0)
    model, img = _image(H, dev)
    prior = p_m71_prior(H, S, S)
    counts, locs, fluxes = _state(H, S, N, seed=H + S, dev=dev)
    tau = torch.full((1, 1), 0.4, device=dev)
    # a state with persisted rate images, as the sampler's sweeps start
    r_in = torch.empty(1, 1, N, H * H, device=dev)
    p_m71_mh(0).run(img, counts, locs, fluxes, tau, prior=prior, image_model=model, rate_out=r_in)
    anc = torch.randint(0, N, (1, 1, N), device=dev, generator=torch.Generator(device=dev)
                        .manual_seed(9))
    for kw in (dict(), dict(rate_in=r_in), dict(rate_in=r_in, ancestors=anc)):
        (l0, f0, a0), r0, m0 = _sweep(False, img, model, prior, counts, locs, fluxes, tau, K, sd,
                                      **kw)
        (l1, f1, a1), r1, m1 = _sweep(True, img, model, prior, counts, locs, fluxes, tau, K, sd,
                                      **kw)
        assert m1._psf_ws, "the cache was not used"
        assert torch.equal(l0, l1) and torch.equal(f0, f1)
        assert torch.equal(m0.last_loglik, m1.last_loglik)
        assert torch.equal(r0, r1)
        assert torch.equal(a0, a1)
        moved = (l1 != (locs if "ancestors" not in kw else locs[:, :, anc[0, 0]])).any(-1)
        assert moved.float().mean() > 0.3  # the sweep did move sources


def test_psf_cache_bit_identical_by_count():
    """Count-stratified populations (CS-SMC strata padded to S sources): the
    component is drawn from 0..count-1; count 0 never moves."""
    dev = torch.device("cuda", 0)
    H, S, N = 32, 6, 512
    model, img = _image(H, dev)
    prior = p_m71_prior(H, 0, S)
    _, locs, fluxes = _state(H, S, N, seed=4, dev=dev)
    counts = (torch.arange(N, device=dev) % (S + 1)).float().reshape(1, 1, N)
    tau = torch.full((1, 1), 0.7, device=dev)
    (l0, f0, a0), r0, m0 = _sweep(False, img, model, prior, counts, locs, fluxes, tau, 50, 0.1,
                                  by_count=True)
    (l1, f1, a1), r1, m1 = _sweep(True, img, model, prior, counts, locs, fluxes, tau, 50, 0.1,
                                  by_count=True)
    assert torch.equal(l0, l1) and torch.equal(f0, f1) and torch.equal(r0, r1)
    assert torch.equal(m0.last_loglik, m1.last_loglik)
