"""The C-ABI library loads on a host without a GPU and exports every entry
point include/smcdet_hip.h declares; the ctypes structs match the header
layout; argument validation fails loudly (no compute is launched)."""
import ctypes
import os
import re

import pytest

from smcdet_amd import _hip

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "smcdet_hip.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(smcdet_[a-z_0-9]+)\s*\(", txt)))


def test_every_header_symbol_is_exported_and_bound():
    names = header_functions()
    assert len(names) >= 15
    L = _hip.lib()
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_hip.EXPORTS), set(names) ^ set(_hip.EXPORTS)


def header_arity():
    """name -> number of parameters, from the header's declarations."""
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(smcdet_[a-z_0-9]+)\s*\(([^;{]*?)\)\s*;", txt, re.S):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_ctypes_signatures_match_header_arity():
    """Every binding passes exactly as many arguments as the header declares
    (a mismatch would shift pointers into the wrong parameters)."""
    arity = header_arity()
    for name, (args, _) in _hip._SIGS.items():
        assert arity[name] == len(args), (name, arity[name], len(args))


def test_version_and_abi():
    assert _hip.lib().smcdet_abi_version() == _hip.ABI_VERSION
    assert "gfx950" in _hip.version()


def test_struct_layouts_match_header():
    # sizes of the POD structs as the header declares them (all 4-byte fields)
    assert ctypes.sizeof(_hip.ImageModelC) == 4 * 4 + 4 * 2 + 6 * 4 + 3 * 4
    assert ctypes.sizeof(_hip.PriorC) == 3 * 4 + 7 * 4
    assert ctypes.sizeof(_hip.MHC) == 4 + 8 * 4
    assert ctypes.sizeof(_hip.ReplayC) == 6 * ctypes.sizeof(ctypes.c_void_p)


def test_invalid_arguments_fail_loudly_without_gpu():
    L = _hip.lib()
    rc = L.smcdet_loglik(None, None, None, None, 1, 1, 1, None, None)
    assert rc == -1
    assert b"null" in L.smcdet_last_error()
    m = _hip.ImageModelC()
    m.model, m.H, m.W, m.psf_radius = 1, 300, 300, 8  # 90,000 px > 65,536
    rc = L.smcdet_loglik(ctypes.byref(m), ctypes.c_void_p(1), ctypes.c_void_p(2),
                         ctypes.c_void_p(3), 1, 1, 1, ctypes.c_void_p(4), None)
    assert rc == -2
    # above 4,096 px only the M71 model has the global-memory paths
    m.model, m.H, m.W = 2, 100, 100
    rc = L.smcdet_loglik(ctypes.byref(m), ctypes.c_void_p(1), ctypes.c_void_p(2),
                         ctypes.c_void_p(3), 1, 1, 1, ctypes.c_void_p(4), None)
    assert rc == -2 and b"M71" in L.smcdet_last_error()
    # the LDS-resident kernels (MALA, MCMC chains, aggregation) keep 4,096 px
    m.model = 1
    rc = L.smcdet_mala_sweep(ctypes.byref(m), *([0] * 25))
    assert rc in (-1, -2)
    with pytest.raises(RuntimeError, match="failed"):
        _hip.check(rc, "smcdet_loglik")


def test_product_refuses_host_tensors():
    import torch
    with pytest.raises(RuntimeError, match="HIP device"):
        _hip.dev_f32(torch.zeros(3), "x")


def test_build_provenance():
    """smcdet_version() carries the sha1 of the sources the library was built
    from (Makefile SRC_HASH); it must equal the hash of the sources here, and
    the Makefile must hash the same files in the same order as _hip.SOURCES."""
    import re
    mk = open(os.path.join(os.path.dirname(_hip._HERE), "Makefile")).read()
    srcs = re.search(r"^SRCS := (.*)$", mk, re.M).group(1).replace("$(CSRC)", "smcdet_amd/csrc")
    hdrs = re.search(r"^HDRS := (.*)$", mk, re.M).group(1).replace("$(CSRC)", "smcdet_amd/csrc")
    listed = (srcs + " " + hdrs).split()
    assert [os.path.relpath(p, os.path.dirname(_hip._HERE)) for p in _hip.SOURCES] == listed
    assert _hip.built_hash() == _hip.source_hash()


def test_launch_timing_pool_without_gpu():
    """smcdet_launch_timing: negative sizes are refused, 0 disables (no HIP
    call), and reading an empty pool reports no timed launches."""
    L = _hip.lib()
    assert L.smcdet_launch_timing(-1) == -1
    assert L.smcdet_launch_timing(0) == 0
    assert _hip.launch_timing_read(4) == []


def test_alias_check_rejects_shared_output_pointer():
    """an output pointer equal to another argument's (a
    freed temporary reused by the caching allocator) is rejected before the
    launch; the header's in-place pairs pass."""
    import ctypes

    import pytest

    from smcdet_amd import _hip
    P = ctypes.c_void_p
    # smcdet_resample_index(weights, T, N, method, seed, offset, u, idx, stream)
    ok = (P(0x1000), 1, 8, 1, 0, 0, None, P(0x2000), P(0x9))
    _hip.check_aliases("smcdet_resample_index", ok)
    bad = (P(0x1000), 1, 8, 1, 0, 0, P(0x2000), P(0x2000), P(0x9))
    with pytest.raises(ValueError, match="argument 7"):
        _hip.check_aliases("smcdet_resample_index", bad)
    # the stream is not compared
    _hip.check_aliases("smcdet_resample_index", (P(0x1000), 1, 8, 1, 0, 0, None, P(0x2000),
                                                 P(0x2000)))
    # MH sweep: locs_in == locs_out (no ancestor gather) is the header's in-place form
    args = [None] * 27
    args[10] = args[13] = P(0x3000)
    args[21] = P(0x4000)
    _hip.check_aliases("smcdet_mh_sweep", tuple(args))
    args[22] = P(0x4000)  # acc_rate aliasing loglik_out
    with pytest.raises(ValueError):
        _hip.check_aliases("smcdet_mh_sweep", tuple(args))


def test_ptr_keeps_temporaries_alive():
    import gc

    import torch

    from smcdet_amd import _hip
    t = torch.empty(4)
    addr = t.data_ptr()
    import weakref
    r = weakref.ref(t)
    p = _hip.ptr(t)
    del t
    gc.collect()
    assert r() is not None and p.value == addr


def test_ptr_temporaries_released_after_the_call():
    """ptr()'s temporaries live until the library call they are
    arguments of returns, and no longer (no step's buffers are held across
    steps); many steps' worth of conversions stay bounded."""
    import gc
    import weakref

    import torch

    from smcdet_amd import _hip
    L = _hip.lib()
    refs = []
    for _ in range(300):  # > the old 256-entry ring
        t = torch.empty(8)
        refs.append(weakref.ref(t))
        _hip.ptr(t)
        del t
        gc.collect()
        assert refs[-1]() is not None  # alive until a call
        L.smcdet_launch_timing(0)        # any entry point (no GPU work)
        gc.collect()
        assert refs[-1]() is None        # released once the call returned
    assert all(r() is None for r in refs)
    # the bound for conversions that never reach a call
    for _ in range(_hip._KEEP_MAX + 10):
        _hip.ptr(torch.empty(1))
    assert len(_hip._kept()) <= _hip._KEEP_MAX
    L.smcdet_launch_timing(0)
    assert len(_hip._kept()) == 0


def test_checked_wrapper_forwards_argtypes():
    """Attribute writes on an entry point reach the ctypes function (ADVICE r5:
    scripts/trace_phases.py sets argtypes through _hip.lib()); checked on a
    libc function so the library's own signatures stay untouched."""
    import ctypes

    from smcdet_amd import _hip
    raw = ctypes.CDLL(None).strlen
    w = _hip._Checked(raw, "smcdet_test_strlen")
    w.argtypes = [ctypes.c_char_p]
    w.restype = ctypes.c_size_t
    assert raw.argtypes == [ctypes.c_char_p] and raw.restype is ctypes.c_size_t
    assert w(b"graft") == 5


def _mh_call(L, flags):
    """smcdet_mh_sweep with valid descriptors and placeholder device pointers
    (never dereferenced: the calls below stop at argument validation, or at
    the launch on a machine without a GPU)."""
    m = _hip.ImageModelC()
    m.model, m.H, m.W, m.psf_radius = 1, 32, 32, 8
    m.background, m.adu_per_nmgy, m.psf_norm = 100.0, 1.0, 1.0
    m.psf_params[:] = [1.0, 2.0, 2.0, 5.0, 0.5, 0.5]
    m.noise_additive, m.noise_multiplicative = 1e-10, 1.9
    p = _hip.PriorC()
    p.kind, p.min_objects, p.max_objects = 1, 10, 10
    p.loc_low, p.loc_high_h, p.loc_high_w = -4.0, 36.0, 36.0
    p.poisson_mean, p.flux_alpha, p.flux_lower, p.flux_upper = 5.0, 0.2, 0.06, 1800.0
    mh = _hip.MHC()
    mh.num_iters, mh.locs_stdev, mh.fluxes_stdev = 1, 0.1, 2.5
    mh.fluxes_min, mh.fluxes_max = 0.06, 1800.0
    mh.locs_min_h = mh.locs_min_w = -4.0
    mh.locs_max_h = mh.locs_max_w = 36.0
    P = [ctypes.c_void_p(0x100000 * (i + 1)) for i in range(16)]
    return L.smcdet_mh_sweep(ctypes.byref(m), ctypes.byref(p), ctypes.byref(mh), P[0], P[1],
                             1, 64, 10, None, P[2], P[3], P[4], P[5], P[6], P[7], None, None,
                             1, 0, None, flags, P[8], P[9], P[10], None, None, None)


def test_product_refuses_diagnostic_flags_and_diag_build_takes_them():
    """The product library compiles only the dispatched MH variants and refuses
    the diagnostic ones (ablations 256/512, scalar slots 1024, PSF table 8192,
    no 1/v cache 4096: include/smcdet_hip.h) before any device work; the
    diagnostic build (make diag) gets past that check."""
    L = _hip.lib()
    assert not _hip.is_diag(L)
    for flag in (256, 512, 1024, 4096, 8192):
        rc = _mh_call(L, flag)
        assert rc == -2, (flag, rc)
        assert b"diagnostic build" in L.smcdet_last_error(), flag
    if not os.path.exists(_hip.DIAG_LIB_PATH):
        pytest.skip("diagnostic build not made")
    with _hip.diag_library() as D:
        assert _hip.lib() is D and _hip.is_diag(D)
        for flag in (256, 1024, 4096):
            _mh_call(D, flag)
            assert b"diagnostic build" not in D.smcdet_last_error(), flag
    assert _hip.lib() is L
