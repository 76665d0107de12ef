#!/usr/bin/env python
"""Per-phase cycle counts of the MH sweep and tile kernels from the profiling
build (make trace -> libsmcdet_hip_trace.so, -DSMCDET_TRACE): lane 0 of the
first 256 waves (MH) / tiles (tile kernel) stores s_memtime at phase
boundaries.  Runs the bench workload (C2) for a few SMC steps and reports the
mean cycles per phase of the last step."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["SMCDET_HIP_LIB"] = os.path.join(ROOT, "smcdet_amd", "libsmcdet_hip_trace.so")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from smcdet_amd import _hip  # noqa: E402
from smcdet_amd.sampler import SMCsampler  # noqa: E402

MH_PHASES = ["stage image", "state + tn caches", "initial render", "MH loop", "write back"]
TILE_PHASES = ["load ll + max", "f(top)", "brentq", "weights", "cumsum", "bins store (or index search)"]


def read_raw(name):
    buf = (ctypes.c_ulonglong * (256 * 16))()
    fn = getattr(_hip.lib(), name)
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert fn(ctypes.addressof(buf), 256 * 16) == 0
    return np.frombuffer(buf, dtype=np.uint64).reshape(256, 16).astype(np.float64)


def read(name, cols):
    buf = (ctypes.c_ulonglong * (256 * 16))()
    fn = getattr(_hip.lib(), name)
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert fn(ctypes.addressof(buf), 256 * 16) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(256, 16)[:, :cols].astype(np.float64)
    return np.diff(t, axis=1)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    H, S, Np, K = 32, 10, 4096, 100
    model, prior, truth = bench.make_models(H, S)
    from smcdet_amd.kernel import SingleComponentMH as MH
    image = bench.synthetic_image(model, truth, H, 1, 1000, dev, max_sources=S)
    mh = MH(K, 0.1, 2.5, bench.M71["flux_lower"], bench.M71["flux_upper"])
    s = SMCsampler(image, H, prior, model, mh, Np, 0.5, "systematic",
                   bench.M71["flux_detection_threshold"], 10 ** 9, print_every=10 ** 9,
                   seed=12345, device=dev)
    s.initialize()
    s._temper_reweight(with_resample=True)
    out = {}
    for i in range(steps):
        idx, s._pending_idx = s._pending_idx, None
        s._step(idx)  # (two launches: the sweep, then the tile kernel)
        torch.cuda.synchronize()
        mh_d = read("smcdet_trace_read_mh", 6)
        tile_d = read("smcdet_trace_read_tile", len(TILE_PHASES) + 1)[:1]
        # the weights phase's sub-steps (columns 7, 8 lie between 3 and 4)
        tr = read_raw("smcdet_trace_read_tile")[0]
        weights_sub = {"exp + partial sums": tr[7] - tr[3], "double reduction": tr[8] - tr[7],
                       "divide + store": tr[4] - tr[8]}
        out[f"step{i}"] = {
            "tau": float(s.temperature.min()),
            "mh_cycles_mean": dict(zip(MH_PHASES, mh_d.mean(0).round(0).tolist())),
            "mh_cycles_max": dict(zip(MH_PHASES, mh_d.max(0).round(0).tolist())),
            "tile_cycles": dict(zip(TILE_PHASES, tile_d[0].round(0).tolist())),
            "tile_weights_cycles": weights_sub,
        }
    # wave lifetimes of the last MH sweep: start/end (s_memrealtime, 100 MHz),
    # s_memtime ticks, HW_ID (CU/SIMD placement)
    buf = (ctypes.c_ulonglong * (8192 * 8))()
    fn = _hip.lib().smcdet_trace_read_waves
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    idx, s._pending_idx = s._pending_idx, None
    s._step(idx)
    torch.cuda.synchronize()
    assert fn(ctypes.addressof(buf), 8192 * 8) == 0
    w = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 8)[:Np].astype(np.float64)
    t0 = w[:, 0].min()
    start, end = (w[:, 0] - t0) * 10e-3, (w[:, 1] - t0) * 10e-3  # microseconds
    life = end - start
    hw = w[:, 4].astype(np.uint64)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = se * 32 + sh * 16 + cu
    per_cu = np.bincount(key.astype(np.int64), minlength=256)
    clk = (w[:, 3] - w[:, 2]) / np.maximum(life, 1e-9) / 1e3  # memtime ticks per ns
    npos, nacc, xcc = w[:, 5], w[:, 6], w[:, 7]
    order = np.argsort(life)
    dec = np.array_split(order, 10)
    out["waves_by_lifetime_decile"] = [
        {"life_us": float(life[d].mean()), "positions": float(npos[d].mean()),
         "accepts": float(nacc[d].mean())} for d in dec]
    out["corr_life_positions"] = float(np.corrcoef(life, npos)[0, 1])
    out["corr_life_accepts"] = float(np.corrcoef(life, nacc)[0, 1])
    out["life_by_xcc"] = {int(x): float(life[xcc == x].mean()) for x in np.unique(xcc)}
    # per-SIMD view: do the waves sharing a SIMD finish together, and do the
    # SIMDs carry equal work?
    xid = (xcc.astype(np.uint64) & 7).astype(np.int64)
    sid = (xid * 256 + key.astype(np.int64)) * 4 + simd.astype(np.int64)
    simd_stats = []
    for v in np.unique(sid):
        m = sid == v
        simd_stats.append((m.sum(), end[m].min(), end[m].max(), npos[m].sum()))
    st = np.array(simd_stats, dtype=np.float64)
    # placement hypothesis: workgroup b (4 waves) lands on CU slot b % 256 and
    # wave w of it on SIMD w, so SIMD-mates are waves (b + 256 k, w)
    wave_idx = np.arange(len(sid))
    b_of, w_of = wave_idx // 4, wave_idx % 4
    hyp = (b_of % 256) * 4 + w_of
    ok = 0
    for v in np.unique(sid):
        m = np.nonzero(sid == v)[0]
        ok += int(len(np.unique(hyp[m])) == 1)
    out["placement_hypothesis_simds_matching"] = f"{ok}/{len(np.unique(sid))}"
    out["placement_sample"] = [[int(i), int(xid[i]), int(se[i]), int(sh[i]), int(cu[i]),
                                int(simd[i])] for i in list(range(0, 16)) + [1024, 1025, 2048]]
    out["per_simd"] = {
        "n_simds": int(len(st)), "waves_per_simd_pctl": np.percentile(st[:, 0], [0, 50, 100]).tolist(),
        "first_end_us_pctl": np.percentile(st[:, 1], [0, 10, 50, 90, 100]).round(1).tolist(),
        "last_end_us_pctl": np.percentile(st[:, 2], [0, 10, 50, 90, 100]).round(1).tolist(),
        "within_simd_spread_us_pctl": np.percentile(st[:, 2] - st[:, 1], [0, 10, 50, 90, 100]).round(1).tolist(),
        "positions_sum_pctl": np.percentile(st[:, 3], [0, 10, 50, 90, 100]).round(0).tolist(),
        "corr_last_end_positions": float(np.corrcoef(st[:, 2], st[:, 3])[0, 1]),
    }
    out["waves"] = {
        "kernel_span_us": float(end.max()), "start_us_pctl": np.percentile(start, [0, 50, 90, 99, 100]).round(1).tolist(),
        "end_us_pctl": np.percentile(end, [0, 10, 50, 90, 100]).round(1).tolist(),
        "life_us_pctl": np.percentile(life, [0, 10, 50, 90, 100]).round(1).tolist(),
        "memtime_GHz_median": float(np.median(clk)),
        "distinct_cu_keys": int((per_cu > 0).sum()), "waves_per_cu_key_max": int(per_cu.max()),
        "hist_start_10us": np.histogram(start, bins=np.arange(0, end.max() + 10, 10))[0].tolist(),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
