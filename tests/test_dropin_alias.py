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
