"""The drop-in boundary on the CPU (no GPU calls): the reference's module
names resolve to this package after install_as_smcdet(), and the mutation
kernels keep the reference's constructor signatures and public attributes
(smcdet/kernel.py:7-24, :133-145)."""
import sys

import pytest
import torch


@pytest.fixture
def alias():
    saved = {k: v for k, v in sys.modules.items() if k == "smcdet" or k.startswith("smcdet.")}
    import smcdet_amd
    smcdet_amd.install_as_smcdet()
    yield
    for k in [k for k in sys.modules if k == "smcdet" or k.startswith("smcdet.")]:
        del sys.modules[k]
    sys.modules.update(saved)


def test_reference_imports_resolve(alias):
    from smcdet.images import ImageModel, M71ImageModel  # noqa: F401
    from smcdet.kernel import SingleComponentMALA, SingleComponentMH
    from smcdet.prior import M71Prior, ParetoStarPrior  # noqa: F401
    from smcdet.sampler import SMCsampler
    import smcdet_amd.kernel as K
    import smcdet_amd.sampler as Sm
    assert SingleComponentMH is K.SingleComponentMH
    assert SingleComponentMALA is K.SingleComponentMALA
    assert SMCsampler is Sm.SMCsampler


def test_mh_attributes():
    from smcdet_amd.kernel import SingleComponentMH
    mh = SingleComponentMH(100, 0.1, 2.5, 0.06, 1800.0)
    assert mh.num_iters == 100
    assert mh.locs_stdev.shape == () and float(mh.locs_stdev) == pytest.approx(0.1)
    assert mh.fluxes_stdev.shape == (1,) and float(mh.fluxes_stdev) == 2.5
    assert mh.fluxes_min.shape == (1,) and mh.fluxes_max.shape == (1,)
    assert mh.locs_min is None and mh.locs_max is None


def test_mala_attributes_and_abi_fields():
    from smcdet_amd.kernel import SingleComponentMALA
    k = SingleComponentMALA(50, 0.1, 2.5, 0.06, 1800.0)
    assert k.num_iters == 50
    assert isinstance(k.locs_step, torch.Tensor) and k.locs_step.shape == ()
    assert isinstance(k.fluxes_step, torch.Tensor) and k.fluxes_step.shape == ()
    assert float(k.locs_step) == pytest.approx(0.1) and float(k.fluxes_step) == 2.5
    assert k.fluxes_min.shape == (1,) and float(k.fluxes_max) == 1800.0
    assert k.locs_min is None and k.locs_max is None
    # the C ABI's proposal-scale fields carry the step sizes

    class _Box:
        class loc_prior:
            low = torch.tensor(-4.0)
            high = torch.tensor([12.0, 12.0])

    c = k._cmh(_Box)
    assert c.num_iters == 50
    assert c.locs_stdev == pytest.approx(0.1) and c.fluxes_stdev == 2.5
    assert (c.locs_min_h, c.locs_max_w) == (-4.0, 12.0)
    assert k._entry == "smcdet_mala_sweep"


def test_unsupported_shapes_fail_at_construction():
    """tiles over 64x64 pixels, more than 64 sources or
    more than 16,384 particles per tile raise ValueError naming the limit when
    the sampler is built, before any kernel launch (the reference tiles any
    image, smcdet/sampler.py:25-31)."""
    from smcdet_amd.images import M71ImageModel
    from smcdet_amd.kernel import SingleComponentMH
    from smcdet_amd.prior import M71Prior
    from smcdet_amd.sampler import MHsampler, SMCsampler

    def make(H, S):
        model = M71ImageModel(image_height=H, image_width=H, background=104.0, psf_radius=8,
                              adu_per_nmgy=241.0, psf_params=[1.1, 2.1, 2.3, 5.2, 0.73, 0.51],
                              noise_additive=1e-10, noise_multiplicative=1.94)
        prior = M71Prior(min_objects=S, max_objects=S, counts_rate=0.003, image_height=H,
                         image_width=H, flux_alpha=0.2, flux_lower=0.06, flux_upper=1800.0,
                         pad=4)
        return model, prior

    from smcdet_amd.kernel import SingleComponentMALA
    mh = SingleComponentMH(10, 0.1, 2.5, 0.06, 1800.0)
    img = torch.zeros(128, 128)
    model, prior = make(128, 10)
    # SMC with SingleComponentMH and the M71 model runs tiles up to 256x256
    # (global-memory sweep); MALA and the MCMC chains keep
    # the LDS budget
    with pytest.raises(ValueError, match="16384 pixels.*4096"):
        SMCsampler(img, 128, prior, model, SingleComponentMALA(10, 0.1, 2.5, 0.06, 1800.0), 512,
                   0.5, "systematic", 0.25, 10)
    with pytest.raises(ValueError, match="4096"):
        MHsampler(img, 128, prior, model, 0.1, 2.5, 0.25, 100, 10)
    model, prior = make(300, 10)
    with pytest.raises(ValueError, match="90000 pixels.*65536"):
        SMCsampler(torch.zeros(300, 300), 300, prior, model, mh, 512, 0.5, "systematic", 0.25,
                   10)
    model, prior = make(32, 80)
    with pytest.raises(ValueError, match="max_objects = 80 > 64"):
        SMCsampler(torch.zeros(32, 32), 32, prior, model, mh, 512, 0.5, "systematic", 0.25, 10)
    model, prior = make(32, 10)
    with pytest.raises(ValueError, match="20000 particles per tile > 16384"):
        SMCsampler(torch.zeros(32, 32), 32, prior, model, mh, 20000, 0.5, "systematic", 0.25, 10)
    # independent stopping lives in the fused step's
    # kernels; the method-by-method schedule refuses it at construction
    with pytest.raises(ValueError, match="independent.*fused"):
        SMCsampler(torch.zeros(32, 32), 32, prior, model, mh, 512, 0.5, "systematic", 0.25, 10,
                   fused=False, stopping="independent")


def test_struct_caches_follow_rebinding():
    """_cmh / _cmodel / _cprior are cached per object (the per-step host
    path) and rebuilt when a parameter attribute is rebound; the struct is
    shared, so Aggregate's num_iters override works on a copy."""
    from smcdet_amd import _hip
    from smcdet_amd.images import M71ImageModel
    from smcdet_amd.kernel import SingleComponentMH
    from tests._params import p_m71_model, p_m71_prior
    k = SingleComponentMH(100, 0.1, 2.5, 0.06, 1800.0)
    prior = p_m71_prior(16, 0, 4)
    c1 = k._cmh(prior)
    assert k._cmh(prior) is c1
    k.locs_stdev = torch.tensor(0.2)
    c2 = k._cmh(prior)
    assert c2 is not c1 and c2.locs_stdev == pytest.approx(0.2)
    k.num_iters = 7
    assert k._cmh(prior).num_iters == 7
    cp = _hip.MHC.from_buffer_copy(k._cmh(prior))
    cp.num_iters = 0
    assert k._cmh(prior).num_iters == 7
    model = p_m71_model(16)
    assert isinstance(model, M71ImageModel)
    m1 = model._cmodel()
    assert model._cmodel() is m1 and m1.H == 16
    model.image_height = 32
    assert model._cmodel().H == 32
    p1 = prior._cprior()
    assert prior._cprior() is p1
    prior.max_objects = 9
    assert prior._cprior().max_objects == 9


def test_ancestor_bins_buffer_layout():
    """AncestorBins (ABI 17): per tile N running sums, then the T offsets, then
    per tile the 64 chunk ends of the search's first level -- the
    SMCDET_BINS_FLOATS(T, N) = T*N + 65*T floats the header names; as_index
    passes int64 index tensors through."""
    import re

    from smcdet_amd import _hip
    b = _hip.AncestorBins.empty((2, 3, 100), torch.device("cpu"))
    assert b.shape == (2, 3, 100) and b.buf.dtype == torch.float32
    assert b.buf.numel() == 6 * 100 + 65 * 6
    hdr = open(_hip.SOURCES[-1]).read()
    m = re.search(r"#define SMCDET_BINS_FLOATS\(T, N\) \(\(size_t\)\(T\) \* \(size_t\)\(N\) \+ "
                  r"\(size_t\)\(T\) \* (\d+)u\)", hdr)
    assert m and int(m.group(1)) == 65
    idx = torch.zeros(1, 1, 4, dtype=torch.int64)
    assert _hip.as_index(idx) is idx and _hip.as_index(None) is None
