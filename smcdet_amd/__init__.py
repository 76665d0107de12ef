"""smcdet_amd — MI355X (gfx950) native SMC star-detection sampler.

Drop-in for the hot path of timwhite0/smcdet: the modules `sampler`,
`kernel`, `images`, `prior`, `distributions` keep the reference's classes
and signatures; the per-particle work runs as hand-written HIP kernels behind
the C ABI in include/smcdet_hip.h (libsmcdet_hip.so, loaded by ctypes).
"""
import importlib
import sys

from . import _hip  # noqa: F401

__version__ = "0.1.0"

_DROP_IN = ("sampler", "kernel", "images", "prior", "distributions", "aggregate")


def install_as_smcdet():
    """Registers this package under the reference's module names (`smcdet`,
    `smcdet.sampler`, ...) so that an unmodified driver doing
    `from smcdet.sampler import SMCsampler` runs on the HIP path."""
    pkg = sys.modules[__name__]
    sys.modules["smcdet"] = pkg
    for name in _DROP_IN:
        sys.modules[f"smcdet.{name}"] = importlib.import_module(f"{__name__}.{name}")
    return pkg
