"""ctypes binding of the gfx950 C ABI (include/smcdet_hip.h).

The library `libsmcdet_hip.so` is built in-tree by `make` (or
`__graft_entry__.build()`).  There is no fallback: if the library is missing
or the tensors are not float32 CUDA(HIP) tensors, the call raises.
"""
from __future__ import annotations

import ctypes
import functools
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SMCDET_HIP_LIB", os.path.join(_HERE, "libsmcdet_hip.so"))

SMCDET_MODEL_M71 = 1
SMCDET_MODEL_POISSON = 2
SMCDET_PRIOR_M71 = 1
SMCDET_PRIOR_PARETO = 2
SMCDET_RESAMPLE_MULTINOMIAL = 0
SMCDET_RESAMPLE_SYSTEMATIC = 1
SMCDET_MH_FULL_RECOMPUTE = 1
SMCDET_MH_COMPONENT_BY_COUNT = 2
SMCDET_MH_SKIP_DONE = 4
ABI_VERSION = 18
SMCDET_SMC_FREEZE_DONE = 1
SMCDET_SMC_TWO_LAUNCH = 2

# Shapes the kernels support (checked by the C ABI too; the samplers raise
# ValueError at construction with these named, SMCsampler/MHsampler.__init__):
MAX_TILE_PIXELS = 4096      # H*W: the tile image + one rate image per wave in LDS (64x64)
# SingleComponentMH SMC with the M71 model above MAX_TILE_PIXELS: the global-memory
# sweep (tile image L2-resident, rate images in HBM), up to 256x256
MAX_TILE_PIXELS_GLOBAL = 65536
MAX_SOURCES = 64            # S = Prior.max_objects: one source per lane
MAX_PARTICLES = 16384       # N per tile: the tile kernel holds 32 log-likelihoods per thread
MAX_TILES = 65535           # T: the MH grid's y dimension
MAX_PSF_RADIUS = 64
MAX_AGG_SOURCES = 4096      # sources of an aggregated (joint) tile (LDS or workspace catalog)


def check_limits(H, W, S, N=None, T=None, R=None, where="sampler", global_ok=False):
    """ValueError naming the limit a configuration exceeds (the reference has
    none: smcdet/sampler.py:25-31 tiles any image).  global_ok: the caller
    runs the global-memory paths above MAX_TILE_PIXELS (SingleComponentMH with
    the M71 image model, up to MAX_TILE_PIXELS_GLOBAL)."""
    if global_ok and H * W > MAX_TILE_PIXELS:
        if H * W > MAX_TILE_PIXELS_GLOBAL:
            raise ValueError(f"{where}: a {H}x{W} tile has {H * W} pixels, above the "
                             f"{MAX_TILE_PIXELS_GLOBAL} (256x256) of the global-memory sweep")
    elif H * W > MAX_TILE_PIXELS:
        raise ValueError(f"{where}: a {H}x{W} tile has {H * W} pixels; this path keeps the "
                         f"tile and one rate image per wavefront in LDS, at most "
                         f"{MAX_TILE_PIXELS} pixels (64x64) -- use tile_dim <= 64 (SMC with "
                         f"SingleComponentMH and M71ImageModel runs tiles up to 256x256)")
    if S > MAX_SOURCES:
        raise ValueError(f"{where}: max_objects = {S} > {MAX_SOURCES} (one source per lane of a "
                         "64-wide wavefront)")
    if N is not None and N > MAX_PARTICLES:
        raise ValueError(f"{where}: {N} particles per tile > {MAX_PARTICLES}")
    if T is not None and T > MAX_TILES:
        raise ValueError(f"{where}: {T} tiles > {MAX_TILES}")
    if R is not None and not 0 <= R <= MAX_PSF_RADIUS:
        raise ValueError(f"{where}: psf_radius {R} outside 0..{MAX_PSF_RADIUS}")


c_f = ctypes.c_float
c_i = ctypes.c_int32
c_p = ctypes.c_void_p
c_u64 = ctypes.c_uint64
c_i64 = ctypes.c_int64
c_u32 = ctypes.c_uint32
c_d = ctypes.c_double


class ImageModelC(ctypes.Structure):
    _fields_ = [("model", c_i), ("H", c_i), ("W", c_i), ("psf_radius", c_i),
                ("background", c_f), ("adu_per_nmgy", c_f), ("psf_params", c_f * 6),
                ("psf_norm", c_f), ("noise_additive", c_f), ("noise_multiplicative", c_f)]


class PriorC(ctypes.Structure):
    _fields_ = [("kind", c_i), ("min_objects", c_i), ("max_objects", c_i), ("loc_low", c_f),
                ("loc_high_h", c_f), ("loc_high_w", c_f), ("poisson_mean", c_f),
                ("flux_alpha", c_f), ("flux_lower", c_f), ("flux_upper", c_f)]


class MHC(ctypes.Structure):
    _fields_ = [("num_iters", c_i), ("locs_stdev", c_f), ("fluxes_stdev", c_f),
                ("fluxes_min", c_f), ("fluxes_max", c_f), ("locs_min_h", c_f),
                ("locs_min_w", c_f), ("locs_max_h", c_f), ("locs_max_w", c_f)]


class ReplayC(ctypes.Structure):
    """smcdet_mh_replay_t: recorded draws, plus the optional decision trace
    (log alpha and accept flag per [k, t, n]) the MH sweep writes."""
    _fields_ = [("comp", c_p), ("uloc", c_p), ("uflux", c_p), ("uacc", c_p),
                ("trace_loga", c_p), ("trace_accept", c_p)]


class SmcTailC(ctypes.Structure):
    """smcdet_smc_tail_t: the temper / reweight / resample-index half of a
    fused SMC iteration (smcdet_mh_sweep_step)."""
    _fields_ = [("temperature_prev", c_p), ("log_weights_unnorm", c_p), ("weights", c_p),
                ("ess", c_p), ("log_norm_const", c_p), ("ess_threshold", c_d),
                ("resample_method", c_i), ("flags", c_u32), ("seed", c_u64), ("offset", c_u64),
                ("idx", c_p), ("resample_u", c_p), ("finished_iter", c_p), ("live", c_p),
                ("live_host", c_p), ("iter", c_i), ("reserved", c_i),
                ("anc_bins", c_p), ("bins_out", c_p)]


_SIGS = {
    "smcdet_version": ([], ctypes.c_char_p),
    "smcdet_abi_version": ([], c_i),
    "smcdet_host_alloc": ([ctypes.c_size_t, c_p, c_p], c_i),
    "smcdet_host_free": ([c_p], c_i),
    "smcdet_launch_timing": ([c_i], c_i),
    "smcdet_launch_timing_read": ([c_p, c_i, c_p], c_i),
    "smcdet_launch_timing_starts": ([c_p, c_i, c_p], c_i),
    "smcdet_launch_timing_tiles": ([c_i], c_i),
    "smcdet_last_error": ([], ctypes.c_char_p),
    "smcdet_loglik": ([c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_p, c_p], c_i),
    "smcdet_render": ([c_p, c_p, c_p, c_i, c_i, c_i, c_p, c_p], c_i),
    "smcdet_psf_dense": ([c_p, c_p, c_i, c_i, c_i, c_p, c_p], c_i),
    "smcdet_sample_image": ([c_p, c_p, c_i64, c_u64, c_u64, c_p, c_p], c_i),
    "smcdet_log_prior": ([c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_p, c_p, c_p], c_i),
    "smcdet_prior_sample": ([c_p, c_i, c_i, c_u64, c_u64, c_p, c_p, c_p, c_p, c_p, c_p, c_p],
                            c_i),
    "smcdet_mh_sweep": ([c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p,
                         c_p, c_p, c_p, c_u64, c_u64, c_p, c_u32, c_p, c_p, c_p, c_p, c_p, c_p],
                        c_i),
    "smcdet_mh_sweep_step": ([c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p,
                              c_p, c_p, c_p, c_p, c_u64, c_u64, c_p, c_u32, c_p, c_p, c_p, c_p,
                              c_p, c_p, c_p], c_i),
    "smcdet_mh_sweep_step_fused": ([c_p, c_i, c_i, c_u32], c_i),
    "smcdet_mala_sweep": ([c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p,
                           c_p, c_p, c_p, c_u64, c_u64, c_p, c_u32, c_p, c_p, c_p, c_p, c_p],
                          c_i),
    "smcdet_mh_chain": ([c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_p, c_p, c_p, c_i, c_i, c_i, c_i,
                         c_i, c_u64, c_u64, c_p, c_p, c_p, c_p, c_p, c_p], c_i),
    "smcdet_temper": ([c_p, c_p, c_p, c_i, c_i, c_d, c_p], c_i),
    "smcdet_update_weights": ([c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_p], c_i),
    "smcdet_resample_index": ([c_p, c_i, c_i, c_i, c_u64, c_u64, c_p, c_p, c_p], c_i),
    "smcdet_temper_reweight": ([c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_d, c_i, c_u64,
                                c_u64, c_p, c_u32, c_p, c_i, c_p, c_p, c_p, c_p], c_i),
    "smcdet_gather": ([c_p, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p], c_i),
    "smcdet_bins_index": ([c_p, c_i, c_i, c_p, c_p], c_i),
    "smcdet_count_posterior": ([c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_u64, c_u64, c_p,
                                c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p], c_i),
    "smcdet_prune": ([c_p, c_p, c_i, c_i, c_i, c_f, c_f, c_p, c_p, c_p, c_p], c_i),
    "smcdet_aggregate_sweep": ([c_p, c_p, c_p, c_i, c_p, c_p, c_i, c_i, c_i, c_p, c_p, c_p, c_p,
                                c_p, c_p, c_p, c_u64, c_u64, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                c_p], c_i),
    "smcdet_aggregate_workspace": ([c_p, c_i, c_i, c_i], c_i64),
    "smcdet_aggregate_temper": ([c_p, c_p, c_p, c_i, c_i, c_i, c_p, c_p, c_p, c_d, c_p, c_p],
                                c_i),
    "smcdet_aggregate_reweight": ([c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p,
                                   c_p, c_p, c_u64, c_u64, c_p, c_p, c_p], c_i),
}
EXPORTS = tuple(_SIGS)

# Output arguments (0-based positions) of each entry point, and the in-place
# pairs the header allows (an input buffer that is also the output: the MH /
# MALA / aggregation sweeps without an ancestor gather, a sampled image
# written over its rate image).  Every call through lib() rejects any other
# output pointer that equals another argument's pointer: two arguments in one
# buffer is what a freed temporary reused by the caching allocator looks like
# (round 3: test_tile_pass_4096_vs_reference read every weight as 1/N).
_SWEEP_OUTS = (12, 13, 14, 16, 21, 22, 23)
_SWEEP_INPLACE = ((9, 12), (10, 13), (11, 14), (15, 16))
_OUTS = {
    "smcdet_loglik": ((7,), ()),
    "smcdet_render": ((6,), ()),
    "smcdet_psf_dense": ((5,), ()),
    "smcdet_sample_image": ((5,), ((1, 5),)),
    "smcdet_log_prior": ((8,), ()),
    "smcdet_prior_sample": ((8, 9, 10), ()),
    "smcdet_mh_sweep": (_SWEEP_OUTS, _SWEEP_INPLACE),
    "smcdet_mh_sweep_step": (_SWEEP_OUTS, _SWEEP_INPLACE),
    "smcdet_mala_sweep": (_SWEEP_OUTS, _SWEEP_INPLACE),
    "smcdet_mh_chain": ((8, 9, 18, 19, 20, 21), ()),
    "smcdet_temper": ((1, 2), ()),
    "smcdet_update_weights": ((3, 4, 5, 6), ()),
    "smcdet_resample_index": ((7,), ()),
    "smcdet_temper_reweight": ((1, 2, 3, 4, 5, 6, 13, 15, 17), ()),
    "smcdet_gather": ((7, 8, 9), ()),
    "smcdet_bins_index": ((3,), ()),
    "smcdet_count_posterior": ((16, 17, 18, 19, 20), ()),
    "smcdet_prune": ((7, 8, 9), ()),
    "smcdet_aggregate_sweep": ((13, 14, 15, 19, 20, 21, 22, 24), ((10, 13), (11, 14), (12, 15))),
    "smcdet_aggregate_temper": ((10,), ()),
    "smcdet_aggregate_reweight": ((10, 11, 12, 13, 17), ()),
}


def _addr(a):
    if isinstance(a, ctypes.c_void_p):
        return a.value or 0
    if isinstance(a, int) and not isinstance(a, bool):
        return a
    return 0


def check_aliases(name, args):
    """ValueError if an output argument of `name` shares its pointer with
    another argument (other than the header's in-place pairs); the stream (last
    argument) is not compared."""
    spec = _OUTS.get(name)
    if spec is None:
        return
    addrs = [_addr(a) for a in args[:-1]]
    nz = [a for a in addrs if a]
    if len(set(nz)) == len(nz):
        return  # no pointer repeats (the common case: one set() on the host path)
    outs, inplace = spec
    ok = {frozenset(pq) for pq in inplace}
    for o in outs:
        if o >= len(addrs) or not addrs[o]:
            continue
        for i, v in enumerate(addrs):
            if i != o and v == addrs[o] and frozenset((i, o)) not in ok:
                raise ValueError(
                    f"{name}: argument {o} (an output) and argument {i} are the same device "
                    f"pointer 0x{v:x}; every buffer passed to the C ABI must be its own "
                    "allocation and stay referenced until the launch's stream has passed it "
                    "(a freed temporary reused by PyTorch's caching allocator looks like this; "
                    "INTEGRATION.md §4)")


class _Checked:
    """An entry point that checks its pointer arguments before the call."""

    def __init__(self, fn, name):
        self._fn, self._name = fn, name

    def __call__(self, *args):
        try:
            check_aliases(self._name, args)
            return self._fn(*args)
        finally:
            # the launch is enqueued: the argument temporaries ptr() kept may
            # go (their blocks are reused in stream order, after the launch)
            _release_kept()

    def __getattr__(self, k):
        return getattr(self._fn, k)

    def __setattr__(self, k, v):
        # argtypes / restype (e.g. scripts/trace_phases.py) belong to the
        # ctypes function itself, not to this wrapper
        if k in ("_fn", "_name"):
            object.__setattr__(self, k, v)
        else:
            setattr(self._fn, k, v)


class _Lib:
    """libsmcdet_hip.so with alias-checked entry points (check_aliases);
    anything else is the CDLL's own attribute."""

    def __init__(self, cdll):
        self._cdll = cdll
        for name in _OUTS:
            if hasattr(cdll, name):
                setattr(self, name, _Checked(getattr(cdll, name), name))

    def __getattr__(self, k):
        # every other entry point also releases ptr()'s temporaries after the
        # call (check_aliases has no spec for it and returns at once)
        fn = getattr(self._cdll, k)
        if k.startswith("smcdet_") and callable(fn):
            w = _Checked(fn, k)
            setattr(self, k, w)
            return w
        return fn


_lib = None

# the library's sources in the Makefile's SRCS + HDRS order: their sha1 is
# compiled into smcdet_version() ("src <sha1>")
_REPO = os.path.dirname(_HERE)
SOURCES = tuple(os.path.join(_REPO, p) for p in (
    "smcdet_amd/csrc/common.hip", "smcdet_amd/csrc/model_kernels.hip",
    "smcdet_amd/csrc/mh_kernel.hip", "smcdet_amd/csrc/mala_kernel.hip",
    "smcdet_amd/csrc/chain_kernel.hip", "smcdet_amd/csrc/smc_kernels.hip",
    "smcdet_amd/csrc/agg_kernel.hip", "smcdet_amd/csrc/device.h", "smcdet_amd/csrc/render.h",
    "smcdet_amd/csrc/mcmc.h", "smcdet_amd/csrc/tile.h", "include/smcdet_hip.h"))


def cached_struct(build):
    """Memoises a per-object C struct builder (`_cmodel`, `_cprior`): the
    struct is rebuilt only when one of the object's instance attributes is
    rebound (keyed on the attributes' identities; the cache keeps those
    objects alive, so an identity cannot be reused).  The tensors and lists
    the builders read are treated as read-only, as the reference does.  Saves
    the per-call float conversions on the sampler's per-step host path.  The
    struct is shared: a caller that changes a field works on a copy
    (`type(c).from_buffer_copy(c)`)."""
    slot = "_cs_" + build.__qualname__
    if os.environ.get("SMCDET_NO_STRUCT_CACHE"):  # (diagnostic: rebuild on every call)
        return build

    @functools.wraps(build)
    def wrapper(self):
        vals = tuple(v for k, v in vars(self).items() if not k.startswith("_cs_"))
        key = tuple(map(id, vals))
        hit = self.__dict__.get(slot)
        if hit is not None and hit[0] == key:
            return hit[1]
        c = build(self)
        self.__dict__[slot] = (key, c, vals)
        return c
    return wrapper


def source_hash():
    """sha1 of SOURCES as they are on disk (None if any is missing)."""
    import hashlib
    h = hashlib.sha1()
    for p in SOURCES:
        if not os.path.exists(p):
            return None
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def built_hash(L=None):
    v = (L or lib()).smcdet_version().decode()
    return v.rsplit("src ", 1)[-1] if "src " in v else None


def _load(path):
    """A checked _Lib over the library at `path` (signatures bound, sources
    hash checked unless SMCDET_ALLOW_STALE=1)."""
    if not os.path.exists(path):
        raise RuntimeError(
            f"smcdet_amd: HIP library not found at {path}; build it with `make` "
            "(or __graft_entry__.build())")
    L = ctypes.CDLL(path)
    stale_ok = os.environ.get("SMCDET_ALLOW_STALE") == "1"
    for name, (args, res) in _SIGS.items():
        if stale_ok and not hasattr(L, name):
            continue  # an older library in a same-box A/B (entry point absent)
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if not stale_ok:
        src, built = source_hash(), built_hash(L)
        if src is not None and built != src:
            raise RuntimeError(
                f"smcdet_amd: {path} was built from sources with sha1 {built}, the "
                f"sources here hash to {src}: rebuild with `make`")
    return _Lib(L)


# the diagnostic build (make diag): the product's kernels plus the A/B and
# timing-only MH variants the product refuses (PSF table, scalar slots,
# ablations, no 1/v cache); reached only inside diag_library()
DIAG_LIB_PATH = os.path.join(_HERE, "libsmcdet_hip_diag.so")
_diag = None
_override = threading.local()


def lib():
    """Load libsmcdet_hip.so once.  Raises if it is missing (there is no
    fallback) or if it was built from other sources than the ones next to it
    (a stale library; SMCDET_ALLOW_STALE=1 skips that check).  Inside
    diag_library() (this thread): the diagnostic build instead."""
    global _lib
    o = getattr(_override, "lib", None)
    if o is not None:
        return o
    if _lib is None:
        _lib = _load(LIB_PATH)
    return _lib


def is_diag(L=None) -> bool:
    return ", diag)" in (L or lib()).smcdet_version().decode()


class diag_library:
    """Context manager: library calls of this thread go to the diagnostic
    build (tests of the A/B variants against the product's kernels; the
    product library refuses their flags).  Raises if it is not built."""

    def __enter__(self):
        global _diag
        if _diag is None:
            _diag = _load(DIAG_LIB_PATH)
            if not is_diag(_diag):
                raise RuntimeError(f"{DIAG_LIB_PATH} is not a diagnostic build")
        self._prev = getattr(_override, "lib", None)
        _override.lib = _diag
        return _diag

    def __exit__(self, *exc):
        _override.lib = self._prev
        return False


def version() -> str:
    return lib().smcdet_version().decode()


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().smcdet_last_error().decode()
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def launch_timing(max_launches: int):
    """Time the next max_launches sweep launches on their own dispatch packets
    (smcdet_launch_timing; 0 disables)."""
    check(lib().smcdet_launch_timing(int(max_launches)), "smcdet_launch_timing")


def launch_timing_read(max_launches: int):
    """Durations (ms) of the sweep launches timed since launch_timing()."""
    buf = (ctypes.c_float * max(int(max_launches), 1))()
    n = c_i(0)
    check(lib().smcdet_launch_timing_read(ctypes.addressof(buf), int(max_launches),
                                          ctypes.byref(n)), "smcdet_launch_timing_read")
    return [float(buf[i]) for i in range(min(n.value, int(max_launches)))]


def launch_timing_starts(max_launches: int):
    """Start times (ms after the first) of the sweep launches timed since
    launch_timing()."""
    buf = (ctypes.c_float * max(int(max_launches), 1))()
    n = c_i(0)
    check(lib().smcdet_launch_timing_starts(ctypes.addressof(buf), int(max_launches),
                                            ctypes.byref(n)), "smcdet_launch_timing_starts")
    return [float(buf[i]) for i in range(min(n.value, int(max_launches)))]


def launch_timing_tiles(on: bool):
    """Also time the per-tile temper / reweight / resampling launches, in launch
    order with the sweeps (smcdet_launch_timing_tiles)."""
    check(lib().smcdet_launch_timing_tiles(1 if on else 0), "smcdet_launch_timing_tiles")


# ptr() keeps the tensors it converts alive until the next library call made
# through lib() returns (per thread), so a temporary passed as
# `ptr(torch.tensor(...))` outlives the call it is an argument of -- its block
# cannot be handed to the next temporary of the same argument list -- and is
# released right after that call: no step's buffers are held beyond it.
# _KEEP_MAX bounds the list for code that converts without calling.
_KEEP_MAX = 4096
_tls = threading.local()


def _kept():
    k = getattr(_tls, "kept", None)
    if k is None:
        k = _tls.kept = []
    return k


def _release_kept():
    k = getattr(_tls, "kept", None)
    if k:
        k.clear()


def ptr(t):
    if t is None:
        return None
    k = _kept()
    if len(k) >= _KEEP_MAX:
        del k[:_KEEP_MAX // 2]
    k.append(t)
    return ctypes.c_void_p(t.data_ptr())


def stream_of(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def dev_f32(t, name):
    """Validates a float32 contiguous HIP tensor (no silent host fallback)."""
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if not t.is_cuda:
        raise RuntimeError(f"{name} must live on a HIP device (got {t.device}); "
                           "smcdet_amd runs only on MI355X (gfx950)")
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32 (got {t.dtype})")
    return t.contiguous()


def ref(x):
    return ctypes.byref(x)


class AncestorBins:
    """The next systematic resampling as the MH sweep reads it
    (smcdet_smc_tail_t.anc_bins / bins_out, ABI 16/17): per tile the running
    sum of the weights (float32), then the T offsets U, then per tile the 64
    chunk ends of the search's first level -- SMCDET_BINS_FLOATS(T, N) =
    T*N + 65*T float32.  Each wave of the next sweep searches its own
    ancestor, so the tile pass skips the index search.  to_index() gives the
    [numH, numW, N] int64 indices (the same ones, bit for bit)."""

    def __init__(self, buf, shape):
        self.buf = buf
        self.shape = tuple(shape)  # (numH, numW, N)

    @staticmethod
    def empty(shape, device):
        nH, nW, N = shape
        return AncestorBins(torch.empty(nH * nW * (N + 65), device=device,
                                        dtype=torch.float32), shape)

    def to_index(self):
        nH, nW, N = self.shape
        idx = torch.empty(self.shape, device=self.buf.device, dtype=torch.int64)
        check(lib().smcdet_bins_index(ptr(self.buf), nH * nW, N, ptr(idx), stream_of(idx)),
              "smcdet_bins_index")
        return idx

    @property
    def device(self):
        return self.buf.device


def as_index(x):
    """Resampling indices of x (an int64 tensor, or AncestorBins), or None."""
    return x.to_index() if isinstance(x, AncestorBins) else x


class HostInts:
    """n int32 in pinned, device-mapped host memory (smcdet_host_alloc):
    `dev(i)` is the device address of element i, `[i]` reads it on the host."""

    def __init__(self, n):
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        check(lib().smcdet_host_alloc(4 * n, ctypes.byref(h), ctypes.byref(d)),
              "smcdet_host_alloc")
        self._h, self._d, self.n = h, d, n
        self._view = (ctypes.c_int32 * n).from_address(h.value)

    def dev(self, i):
        return ctypes.c_void_p(self._d.value + 4 * i)

    def __getitem__(self, i):
        return int(self._view[i])

    def __setitem__(self, i, v):
        self._view[i] = int(v)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib is not None:
            _lib.smcdet_host_free(h)
            self._h = None
