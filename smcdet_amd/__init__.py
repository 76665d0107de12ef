"""smcdet_amd — MI355X (gfx950) native SMC star-detection sampler.

Drop-in for the hot path of timwhite0/smcdet: the modules `sampler`,
`kernel`, `images`, `prior`, `distributions` keep the reference's classes
and signatures; the per-particle work runs as hand-written HIP kernels behind
the C ABI in include/smcdet_hip.h (libsmcdet_hip.so, loaded by ctypes).
"""
from . import _hip  # noqa: F401

__version__ = "0.1.0"
