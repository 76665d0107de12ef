#!/usr/bin/env python
"""Benchmark: MH particle-steps/sec on 4096-particle 32x32 synthetic M71 tiles.

Workload (BASELINE.json configs[1]): one 32x32 tile per GPU,
S = 10 sources per catalog, N = 4096 particles, SingleComponentMH with 100
iterations per SMC step, M71 image model/prior (notebooks/smc.ipynb params,
counts_rate 5/(40*40)), systematic resampling, rho = 0.5.

A timed "step" is one full SMC iteration of the hot path on resident device
data: the fused MH sweep (ancestor gather + 100 MH iterations + fresh
log-likelihood) and the per-tile temper + reweight + resampling-index launch.
particle-steps per step = N * 100 per tile.  Multi-GPU: one process per GPU,
each rank owns its own tile(s) (weak scaling, no data-path collective); the
timed region is bracketed by barrier + synchronize and the MAX over ranks is
reported.  value = all ranks' particle-steps / that time.  The default run
also times BASELINE configs[2] (C3: 64 tiles split over the ranks, strong
scaling) with the same bracket and reports it as `c3_strong` (--no-c3 skips).

Roofline objects: `roofline` (HBM, as BASELINE.json asks): algorithmic bytes
of the MH launch = 248 B per particle-step (state read+write
24*S B + log-target cache 8 B) x N x K over the MH kernel's average
duration, timed with HIP events on the launch stream.  `compute` gives the
binding resource (FP32 VALU + transcendental) with SURVEY §8d's algorithmic
68.0 kFLOP / 13.6 k transcendentals per particle-step of the reference's full
re-render.  `cpu_baseline`: the C restatement (oracle/mh_oracle.c, float64,
OpenMP) timed on this host's cores on a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

M71 = dict(flux_alpha=0.21411753249015655, flux_lower=0.06291294097900389,
           flux_upper=1804.6791992187502, flux_detection_threshold=0.25165176391601557,
           background=104.1486587524414, adu_per_nmgy=241.02658081054688,
           psf_params=[1.107237458229065, 2.0800251960754395, 2.3254318237304688,
                       5.240590572357178, 0.7346734404563904, 0.5114791393280029],
           psf_radius=8, noise_additive=1.0000007072408224e-10,
           noise_multiplicative=1.936462640762329)
COUNTS_RATE_C2 = 5.0 / (40 * 40)
M71_COUNTS_RATE = 0.030264640226960182  # notebooks/smc.ipynb cell 2
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md (spec)
C3_TILES = 64               # BASELINE configs[2]: 64 32x32 tiles over the node
FP32_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md (vector FP32, spec)
B_ALG_PER_STEP = 248        # SURVEY §8d, S=10
F_ALG_PER_STEP = 68.0e3     # SURVEY §8d, S=10, 32x32
# rocprofv3 PMC summary of the C2 MH launch (scripts/profile.sh + scripts/pmc_summary.py):
# FETCH_SIZE / WRITE_SIZE (HBM traffic), SQ VALU counts, GRBM_GUI_ACTIVE (effective clock),
# and the sha1 of the library sources it was measured on
PMC_FILE = "pmc_mh_r06.json"
# the same for the C4 / C5 MH launches (the default run's `c4` / `c5` legs)
PMC_FILES = {"c2": PMC_FILE, "c4": "pmc_mh_c4_r06.json", "c5": "pmc_mh_c5_r06.json"}
# The VALU issue costs on gfx950, measured at the MH sweeps' occupancies
# (scripts/probe/issue_probe.hip: per-SIMD s_memtime spans of 16 independent
# chains per wave, profiles/r06/issue_probe.txt): SIMD cycles per
# wave-instruction at 4 waves per SIMD (the 32x32 sweep) and 7 (the 8x8
# sweep).  Transcendentals are NOT co-issued (a 6 fma : 1 exp mix costs more
# than the sum of its parts), and v_pk_* f32 ops cost ~1.85 plain ones.
ISSUE_MODEL = {
    "cycles": {"4": {"plain": 2.68, "packed": 4.94, "trans": 8.58},
               "7": {"plain": 2.40, "packed": 4.45, "trans": 8.33}},
    "floor": "plain x (VALU - TRANS) + trans x TRANS: packed ops counted as plain, so a lower "
             "bound on the SIMD cycles the counted stream needs",
    "probe": "profiles/r06/issue_probe.txt"}
SIMDS = 256 * 4


def waves_per_simd(tile):
    """The MH sweep's occupancy: 7 waves per SIMD for tiles of <= 64 pixels
    (mh_waves_per_eu<1>), 4 otherwise."""
    return 7 if tile * tile <= 64 else 4


def issue_floor(per_step, tile, clk_ghz, mh_ms, launch_steps):
    """The calibrated issue floor of the PMC-counted VALU stream against the
    SIMD cycles the launch had (at its measured clock), per particle-step."""
    w = str(waves_per_simd(tile))
    c = ISSUE_MODEL["cycles"][w]
    valu = per_step["SQ_INSTS_VALU"]
    trans = per_step.get("SQ_INSTS_VALU_TRANS_F32") or 0.0
    floor = c["plain"] * (valu - trans) + c["trans"] * trans
    avail = SIMDS * clk_ghz * 1e9 * mh_ms * 1e-3 / launch_steps
    return {"waves_per_simd": int(w), "valu_wave_insts_per_particle_step": valu,
            "trans_wave_insts_per_particle_step": trans,
            "floor_cycles_per_particle_step": floor,
            "available_cycles_per_particle_step": avail, "clock_ghz": clk_ghz,
            "issue_frac": floor / avail, "cycles_per_valu_inst": avail / valu,
            "costs": c}


# the reference itself (torch CPU, smcdet/kernel.py) on the same workload, SURVEY §6 (build
# container, 8 cores; the reference does not travel to the GPU box)
REFERENCE_CPU = {"value": 8466.0, "unit": "particle-steps/sec", "cores": 8, "kind": "reference",
                 "sample": "reference SingleComponentMH, 32x32, N=4096, S=10, 10 iterations at "
                           "tau=0.3, torch 2.10 CPU float32 (SURVEY.md §6)"}
# Cross-calibration of the port against the reference on the same 8 cores, the
# same state and configuration (scripts/cpu_crosscal.py in the build container,
# profiles/r06/cpu_crosscal.json): the port's particle-steps/s over the
# reference's.  Converts the box's port figure to a reference-equivalent one.
CROSSCAL_FILE = "profiles/r06/cpu_crosscal.json"


# --host-rehearsal: the multi-rank bookkeeping on the CPU (gloo, stub sampler)
REHEARSAL = False


def _sync():
    """torch.cuda.synchronize(), or nothing in a CPU host rehearsal."""
    if not REHEARSAL:
        torch.cuda.synchronize()


class RehearsalSampler:
    """The SMCsampler surface bench.py drives (initialize, _temper_reweight,
    _step, the state tensors and _T), on the CPU with no kernel: a step sleeps
    1 ms per tile and rank, so ranks finish at different times and the MAX
    over ranks is what the line reports.  For tests/test_bench_host.py's
    2-rank gloo torchrun of bench.py (--host-rehearsal)."""

    def __init__(self, T, N, S, rank):
        self._T, self.N, self.S, self.rank = T, N, S, rank
        self.device = torch.device("cpu")
        self.fused_step = False
        self.temperature = torch.zeros(1, T)
        self.ess = torch.full((1, T), float(N))
        self.mutation_acc_rates = torch.zeros(1, T)
        self.counts = torch.full((1, T, N), float(S))
        self.locs = torch.zeros(1, T, N, S, 2)
        self.fluxes = torch.ones(1, T, N, S)
        self.weights = torch.full((1, T, N), 1.0 / N)
        self.log_normalizing_constant = torch.zeros(1, T)
        self._pending_idx = None
        self.steps_run = 0

    def initialize(self):
        pass

    def _step_fusable(self):
        return False

    def _temper_reweight(self, with_resample=True):
        self._pending_idx = torch.arange(self.N).repeat(1, self._T, 1)

    def _step(self, idx):
        time.sleep(1e-3 * self._T * (1 + self.rank))
        self.steps_run += 1
        self._temper_reweight(True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # c2 (default, the headline): one 32x32 tile per GPU.  c4 / c5 are the
    # BASELINE.json configs[3] / [4] run as extra lines: batches of 8x8 M71
    # tiles (N=4096, S=10) and count-stratified SMC over 8x8 tiles (counts
    # 0..6, 8192 particles per count), per GPU.
    # mcmc: the reference's MCMC baseline (MHsampler, experiments/m71/
    # run_mcmc.py: 8x8 M71 cutouts, S=10, 50,000 samples, burn-in 30,000,
    # every 2nd kept), one chain per image, a batch of images per GPU
    # agg: tile aggregation (smcdet/aggregate.py): CS-SMC on the
    # 4x4 8x8 tiles of a 32x32 image (partition boxes, pad 2, counts 0..6),
    # then Aggregate over 4 levels to one 32x32 population; one image per GPU
    ap.add_argument("--workload", choices=["c2", "c4", "c5", "mcmc", "agg"], default="c2")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--particles", type=int, default=4096)
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--sources", type=int, default=10)
    ap.add_argument("--mh-iters", type=int, default=100)
    ap.add_argument("--tiles-per-gpu", type=int, default=1)
    # c2 strong scaling (BASELINE configs[2], C3: 64 tiles over the GPUs): this
    # many 32x32 tiles in total, split contiguously over the ranks; tile g is
    # drawn from seed 1000 + g whatever the rank count
    ap.add_argument("--total-tiles", type=int, default=0)
    ap.add_argument("--full-recompute", action="store_true")
    # mutation kernel: SingleComponentMH (the headline) or SingleComponentMALA
    # (smcdet/kernel.py:133-275) on the same workload, as an extra line
    ap.add_argument("--kernel", choices=["mh", "mala"], default="mh")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # skip the untimed complete run() (wall time to temperature 1), e.g. under
    # a profiler whose kernel averages should cover the timed steps only
    ap.add_argument("--no-full-run", action="store_true")
    # skip the untimed comparison with the reference's recorded runs
    ap.add_argument("--no-vs-ref", action="store_true")
    # A/B: the temper/reweight/resample pass inside the sweep's launch
    # (SMCsampler.fused_step) instead of the default two back-to-back launches
    ap.add_argument("--fused-step", action="store_true")
    # A/B: the tile pass writes int64 resampling indices instead of handing
    # bins to the next sweep (SMCsampler.ancestor_bins = False)
    ap.add_argument("--ancestor-indices", action="store_true")
    # no kernel-timing pass after the timed region (the roofline then uses the
    # step time as the kernel time)
    ap.add_argument("--no-kernel-timing", action="store_true")
    # skip the C3 strong-scaling leg (c3_leg) of the default C2 run
    ap.add_argument("--no-c3", action="store_true")
    # skip the untimed step-spread passes
    ap.add_argument("--no-spread", action="store_true")
    # skip the C4 / C5 / C3-rank-share legs of the default C2 run
    ap.add_argument("--no-legs", action="store_true")
    # seconds of back-to-back untimed steps before the warmup steps (then the
    # sampler restarts from a fresh initialisation): the chip's clock ramps
    # up over its first ~60 busy steps after idle, which the W = 5 warmup
    # steps do not cover (scripts/warmup_probe.py); 0 = off
    ap.add_argument("--prewarm-s", type=float, default=2.0)
    # diagnostic MH flags (A/B timing: e.g. 2048 = SMCDET_MH_NO_PSF_CACHE)
    ap.add_argument("--mh-debug-flags", type=int, default=0)
    # CPU rehearsal of the multi-rank bookkeeping (gloo, RehearsalSampler: no
    # GPU, no kernel): shard sizes, the barrier + MAX-over-ranks timing, the
    # rank-0-only line / vs_reference / cpu_baseline, the catalog gather
    ap.add_argument("--host-rehearsal", action="store_true")
    return ap.parse_args()


def mutation_kernel(args, K, full_recompute=False):
    from smcdet_amd.kernel import SingleComponentMALA, SingleComponentMH
    p = M71
    if args.kernel == "mala":
        return SingleComponentMALA(K, 0.1, 2.5, p["flux_lower"], p["flux_upper"])
    mh = SingleComponentMH(K, 0.1, 2.5, p["flux_lower"], p["flux_upper"],
                           full_recompute=full_recompute)
    mh.debug_flags = args.mh_debug_flags
    return mh


def make_models(H, S):
    from smcdet_amd.images import M71ImageModel
    from smcdet_amd.prior import M71Prior
    p = M71
    model = M71ImageModel(image_height=H, image_width=H, background=p["background"],
                          psf_radius=p["psf_radius"], adu_per_nmgy=p["adu_per_nmgy"],
                          psf_params=p["psf_params"], noise_additive=p["noise_additive"],
                          noise_multiplicative=p["noise_multiplicative"])
    prior = M71Prior(min_objects=S, max_objects=S, counts_rate=COUNTS_RATE_C2, image_height=H,
                     image_width=H, flux_alpha=p["flux_alpha"], flux_lower=p["flux_lower"],
                     flux_upper=p["flux_upper"], pad=4)
    truth = M71Prior(min_objects=0, max_objects=100, counts_rate=COUNTS_RATE_C2, image_height=H,
                     image_width=H, flux_alpha=p["flux_alpha"],
                     flux_lower=p["flux_detection_threshold"], flux_upper=p["flux_upper"], pad=4)
    return model, prior, truth


def synthetic_image(model, truth, H, tiles_per_side, seed, dev, max_sources):
    """Synthetic M71 truth tiles (generate_images, images.py:178-228), drawn on
    device; draws with more than max_sources sources are rejected."""
    torch.manual_seed(seed)
    img = torch.empty(tiles_per_side * H, tiles_per_side * H, device=dev)
    for a in range(tiles_per_side):
        for b in range(tiles_per_side):
            while True:
                c, l, f = truth.sample(num_catalogs=1, device=dev)
                if int(c.max()) <= max_sources:
                    break
            img[a * H:(a + 1) * H, b * H:(b + 1) * H] = model.sample(l, f)[0, 0, :, :, 0]
    return img


def synthetic_tiles(model, truth, H, tile_ids, dev, max_sources):
    """[1, len(tile_ids), H, H] synthetic M71 tiles, tile g from seed 1000 + g."""
    out = torch.empty(1, len(tile_ids), H, H, device=dev)
    for i, g in enumerate(tile_ids):
        torch.manual_seed(1000 + g)
        while True:
            c, l, f = truth.sample(num_catalogs=1, device=dev)
            if int(c.max()) <= max_sources:
                break
        out[0, i] = model.sample(l, f)[0, 0, :, :, 0]
    return out


def shard(total, world, rank):
    """Contiguous block of range(total) owned by `rank` (as distributed.shard_tiles)."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return list(range(lo, lo + base + (1 if rank < rem else 0)))


def cpu_baseline(args, image_tile, seconds):
    """C restatement of the reference MH sweep (float64 full re-render per
    step, OpenMP over particles) on a bounded sample of the same workload."""
    import numpy as np

    from oracle import c_oracle
    from oracle import smc_oracle as O
    H, S = args.tile, args.sources
    p = M71
    model = O.M71Model(H, H, p["background"], p["psf_radius"], p["adu_per_nmgy"],
                       p["psf_params"], p["noise_additive"], p["noise_multiplicative"])
    prior = O.M71PriorP(S, S, COUNTS_RATE_C2, H, H, 4, p["flux_alpha"], p["flux_lower"],
                        p["flux_upper"])
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    threads = max(1, min(threads, os.cpu_count() or 1))
    rng = np.random.default_rng(0)
    n = max(64, 32 * threads)
    locs = (rng.random((1, 1, n, S, 2)) * (H + 8) - 4).astype(np.float32)
    fl = O.trunc_pareto_sample(rng.random((1, 1, n, S)), p["flux_alpha"], p["flux_lower"],
                               p["flux_upper"]).astype(np.float32)
    counts = np.full((1, 1, n), S, np.float32)
    img = image_tile.reshape(1, 1, H, H)
    c_oracle.lib()
    sweep = c_oracle.mala_sweep if args.kernel == "mala" else c_oracle.mh_sweep
    # calibrate K so the timed sample takes ~`seconds`
    K = 2
    while True:
        mh = O.MHParams(K, 0.1, 2.5, p["flux_lower"], p["flux_upper"])
        t0 = time.perf_counter()
        sweep(img, counts, locs, fl, 0.3, prior, model, mh, seed=1, threads=threads)
        dt = time.perf_counter() - t0
        if dt > seconds / 4 or K >= 4096:
            break
        K *= 2
    K = max(1, int(K * seconds / max(dt, 1e-6)))
    mh = O.MHParams(K, 0.1, 2.5, p["flux_lower"], p["flux_upper"])
    t0 = time.perf_counter()
    sweep(img, counts, locs, fl, 0.3, prior, model, mh, seed=2, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": n * K / dt, "unit": "particle-steps/sec", "cores": threads, "kind": "port",
            "sample": f"oracle/mh_oracle.c float64 full re-render, {n} particles x {K} "
                      f"{args.kernel.upper()} iterations, {H}x{H} tile, S={S}, tau=0.3 "
                      f"({dt:.1f} s)"}


def build_sampler(args, dev, rank):
    """(sampler, particle-steps per SMC step, workload description)."""
    p = M71
    if REHEARSAL:
        H, S, Np, K = args.tile, args.sources, args.particles, args.mh_iters
        world = int(os.environ.get("WORLD_SIZE", "1"))
        ids = shard(args.total_tiles, world, rank) if args.total_tiles > 0 else [rank]
        T = len(ids)
        return RehearsalSampler(T, Np, S, rank), None, T * Np * K, torch.zeros(H, H), dict(
            workload=f"host rehearsal: {T} stub tile(s) on rank {rank} of {world}",
            total_tiles=args.total_tiles, tiles_per_gpu=T, particles=Np, tile=H, sources=S,
            mh_iters=K, kernel=args.kernel, tile_ids=ids)
    from smcdet_amd.sampler import SMCsampler
    if args.workload == "c2" and args.total_tiles > 0:
        H, S, Np, K = args.tile, args.sources, args.particles, args.mh_iters
        world = int(os.environ.get("WORLD_SIZE", "1"))
        ids = shard(args.total_tiles, world, rank)
        if not ids:
            raise SystemExit(f"rank {rank}: no tiles ({args.total_tiles} over {world} ranks)")
        model, prior, truth = make_models(H, S)
        tiles = synthetic_tiles(model, truth, H, ids, dev, S)
        mh = mutation_kernel(args, K, args.full_recompute)
        s = SMCsampler.from_tiles(tiles, prior, model, mh, Np, 0.5, "systematic",
                                  p["flux_detection_threshold"], 10 ** 9, print_every=10 ** 9,
                                  seed=12345 + rank, device=dev)
        T = len(ids)
        return s, mh, T * Np * K, tiles[0, 0], dict(
            workload=f"C3: {args.total_tiles} x {H}x{H} tiles over {world} GPU(s) ({T} on rank "
                     f"{rank}), S={S}, N={Np}, {K} {args.kernel.upper()} iters per SMC step, "
                     "systematic, rho=0.5", total_tiles=args.total_tiles, tiles_per_gpu=T,
            particles=Np, tile=H, sources=S, mh_iters=K, kernel=args.kernel)
    if args.workload == "c2":
        H, S, Np, K = args.tile, args.sources, args.particles, args.mh_iters
        tps = int(round(args.tiles_per_gpu ** 0.5))
        model, prior, truth = make_models(H, S)
        image = synthetic_image(model, truth, H, tps, 1000 + rank, dev, max_sources=S)
        mh = mutation_kernel(args, K, args.full_recompute)
        s = SMCsampler(image, H, prior, model, mh, Np, 0.5, "systematic",
                       p["flux_detection_threshold"], 10 ** 9, print_every=10 ** 9,
                       seed=12345 + rank, device=dev)
        T = tps * tps
        return s, mh, T * Np * K, image[:H, :H], dict(
            workload=f"C2: {T} x {H}x{H} tile(s)/GPU, S={S}, N={Np}, {K} {args.kernel.upper()} "
                     "iters per SMC step, systematic, rho=0.5", tiles_per_gpu=T, particles=Np,
            tile=H, sources=S, mh_iters=K, kernel=args.kernel)
    # 8x8 M71 tiles at the real M71 source density (experiments/m71synthetic/
    # generate_images.py:27-67: truth from M71Prior(0, 100))
    from smcdet_amd.images import M71ImageModel
    from smcdet_amd.prior import M71Prior
    H, K, B = 8, args.mh_iters, max(1, args.tiles_per_gpu)
    model = M71ImageModel(image_height=H, image_width=H, background=p["background"],
                          psf_radius=p["psf_radius"], adu_per_nmgy=p["adu_per_nmgy"],
                          psf_params=p["psf_params"], noise_additive=p["noise_additive"],
                          noise_multiplicative=p["noise_multiplicative"])
    truth = M71Prior(min_objects=0, max_objects=100, counts_rate=M71_COUNTS_RATE, image_height=H,
                     image_width=H, flux_alpha=p["flux_alpha"],
                     flux_lower=p["flux_detection_threshold"], flux_upper=p["flux_upper"], pad=4)
    torch.manual_seed(2000 + rank)
    c, l, f = truth.sample(num_catalogs=B, device=dev)
    images = model.sample(l, f)[0, 0].permute(2, 0, 1).contiguous()       # [B, 8, 8]
    mh = mutation_kernel(args, K)
    if args.workload == "c4":
        S, Np = 10, 4096
        prior = M71Prior(min_objects=S, max_objects=S, counts_rate=M71_COUNTS_RATE,
                         image_height=H, image_width=H, flux_alpha=p["flux_alpha"],
                         flux_lower=p["flux_lower"], flux_upper=p["flux_upper"], pad=4)
        s = SMCsampler.from_tiles(images.reshape(1, B, H, H), prior, model, mh, Np, 0.5,
                                  "systematic", p["flux_detection_threshold"], 10 ** 9,
                                  10 ** 9, seed=12345 + rank, device=dev)
        return s, mh, B * Np * K, images[0], dict(
            workload=f"C4: {B} x 8x8 M71 tiles/GPU (batched), S={S}, N={Np}, {K} MH iters per "
                     "SMC step, systematic, rho=0.5", tiles_per_gpu=B, particles=Np, tile=H,
            sources=S, mh_iters=K, kernel=args.kernel)
    from smcdet_amd.cssmc import CountStratifiedSMC
    smax, Np = 6, 8192
    prior = M71Prior(min_objects=0, max_objects=smax, counts_rate=M71_COUNTS_RATE,
                     image_height=H, image_width=H, flux_alpha=p["flux_alpha"],
                     flux_lower=p["flux_lower"], flux_upper=p["flux_upper"], pad=4)
    cs = CountStratifiedSMC(images.reshape(1, B, H, H), H, prior, model, mh, Np, 0.5,
                            "systematic", p["flux_detection_threshold"], 10 ** 9, 10 ** 9,
                            seed=12345 + rank, device=dev)
    NS = smax + 1
    # the count-0 stratum has no source to move (its MH launch does no work):
    # only the NS - 1 strata with s >= 1 make particle-steps
    return cs.sampler, cs.MutationKernel, B * (NS - 1) * Np * K, images[0], dict(
        workload=f"C5: CS-SMC over {B} x 8x8 M71 tiles/GPU, counts 0..{smax} "
                 f"({NS} strata as tiles, S={smax}; particle-steps counted over the {NS - 1} strata "
                 f"with s >= 1), N={Np} per count, {K} MH iters per SMC step, systematic, rho=0.5",
        tiles_per_gpu=B, particles=Np * NS, tile=H, sources=smax,
        mh_iters=K, kernel=args.kernel)


def bench_agg(args, dev, rank, world):
    """Aggregate.run() on one synthetic 32x32 M71 image per GPU, after
    count-stratified SMC on its 4x4 grid of 8x8 tiles (untimed).  value =
    aggregation MH particle-steps (sum over levels of joint tiles x N x K x
    SMC iterations) / the run's wall time."""
    import contextlib
    import io
    from smcdet_amd.aggregate import Aggregate
    from smcdet_amd.cssmc import CountStratifiedSMC
    from smcdet_amd.kernel import SingleComponentMH
    from smcdet_amd.prior import M71Prior
    p = M71
    H, tile, N, K = 32, 8, args.particles, args.mh_iters
    model32, _, truth = make_models(H, 10)
    model8, _, _ = make_models(tile, 10)
    kp = M71Prior(min_objects=0, max_objects=6, counts_rate=COUNTS_RATE_C2, image_height=tile,
                  image_width=tile, flux_alpha=p["flux_alpha"], flux_lower=p["flux_lower"],
                  flux_upper=p["flux_upper"], pad=2, pad_mode="partition")
    torch.manual_seed(3000 + rank)
    while True:
        c, l, f = truth.sample(num_catalogs=1, device=dev)
        if int(c.reshape(-1)[0]) <= 10:
            break
    img = model32.sample(l, f)[0, 0, :, :, 0].contiguous()

    def mh():
        return SingleComponentMH(K, 0.1, 2.5, p["flux_lower"], p["flux_upper"])

    def one(seed):
        kids = CountStratifiedSMC(img, tile, kp, model8, mh(), N, 0.5, "systematic",
                                  p["flux_detection_threshold"], 200, print_every=10 ** 9,
                                  num_catalogs=N, seed=seed, device=dev)
        with contextlib.redirect_stdout(io.StringIO()):
            kids.run()
        agg = Aggregate(kp, model8, mh(), kids.tiled_image, kids.counts, kids.locs, kids.fluxes,
                        kids.weights, kids.log_normalizing_constant,
                        p["flux_detection_threshold"], "systematic", 0.5, print_every=10 ** 9,
                        seed=seed + 1, device=dev)
        torch.cuda.synchronize()
        if world > 1:
            import torch.distributed as tdist
            tdist.barrier()
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            agg.run()
        torch.cuda.synchronize()
        if world > 1:
            tdist.barrier()
        return agg, time.perf_counter() - t0
    one(11 + 100 * rank)  # warm-up
    agg, elapsed = one(12 + 100 * rank)
    if world > 1:
        import torch.distributed as tdist
        on_dev = os.environ.get("SMCDET_DIST_BACKEND", "nccl") == "nccl"
        t = torch.tensor([elapsed], device=dev if on_dev else "cpu", dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t)
    tiles_per_level = [(H // tile) ** 2 // 2 ** (lv + 1) for lv in range(agg.num_aggregation_levels)]
    steps = sum(t * it for t, it in zip(tiles_per_level, agg.iters_per_level)) * N * K
    return {
        "metric": "aggregation MH particle-steps/sec (agg workload: 4x4 8x8 tiles -> 32x32)",
        "value": world * steps / elapsed, "unit": "particle-steps/sec", "n_gpus": world,
        "steps": 1, "warmup": 1, "ms_per_step": elapsed * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (M71 prior + image model, seed 3000+rank)",
        "config": {"workload": f"AGG: one 32x32 M71 image/GPU, CS-SMC on 4x4 8x8 tiles (counts "
                               f"0..6, pad 2 partition), Aggregate N={N}, K={K}",
                   "particles": N, "mh_iters": K, "levels": agg.num_aggregation_levels,
                   "parallelism": f"image-sharded x{world}"},
        "aggregate": {"iters_per_level": agg.iters_per_level, "joint_tiles_per_level":
                      tiles_per_level, "final_sources": int(agg.locs.shape[-2]),
                      "log_evidence": float(agg.log_evidence.reshape(-1)[0]),
                      "detected_mean": float(agg.pruned_counts.float().mean())},
    }


def bench_mcmc(args, dev, rank, world):
    """MHsampler over a batch of 8x8 M71 cutouts (one chain each): the whole
    run() is timed, as run_mcmc.py:121-125 times it per image."""
    from smcdet_amd.images import M71ImageModel
    from smcdet_amd.prior import M71Prior
    from smcdet_amd.sampler import MHsampler
    p = M71
    H, S, B = 8, 10, max(1, args.tiles_per_gpu)
    total, burnin, keep = 50000, 30000, 2
    model = M71ImageModel(image_height=H, image_width=H, background=p["background"],
                          psf_radius=p["psf_radius"], adu_per_nmgy=p["adu_per_nmgy"],
                          psf_params=p["psf_params"], noise_additive=p["noise_additive"],
                          noise_multiplicative=p["noise_multiplicative"])
    truth = M71Prior(min_objects=0, max_objects=100, counts_rate=M71_COUNTS_RATE, image_height=H,
                     image_width=H, flux_alpha=p["flux_alpha"],
                     flux_lower=p["flux_detection_threshold"], flux_upper=p["flux_upper"], pad=4)
    prior = M71Prior(min_objects=S, max_objects=S, counts_rate=M71_COUNTS_RATE, image_height=H,
                     image_width=H, flux_alpha=p["flux_alpha"], flux_lower=p["flux_lower"],
                     flux_upper=p["flux_upper"], pad=4)
    torch.manual_seed(2000 + rank)
    c, l, f = truth.sample(num_catalogs=B, device=dev)
    tiles = model.sample(l, f)[0, 0].permute(2, 0, 1).reshape(1, B, H, H).contiguous()

    def make(n_total, n_burn):
        return MHsampler.from_tiles(tiles, prior, model, 0.1, 2.5, p["flux_detection_threshold"],
                                    n_total, n_burn, keep, print_every=10 ** 9,
                                    seed=12345 + rank, device=dev)
    make(1001, 1).run()  # warm-up
    s = make(total, burnin)
    if world > 1:
        import torch.distributed as tdist
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.run()
    torch.cuda.synchronize()
    if world > 1:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        on_dev = os.environ.get("SMCDET_DIST_BACKEND", "nccl") == "nccl"
        t = torch.tensor([elapsed], device=dev if on_dev else "cpu", dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t)
    iters = B * (total - 1)
    return {
        "metric": "chain-iterations/sec (mcmc workload: MHsampler, 8x8 M71 cutouts)",
        "value": world * iters / elapsed, "unit": "chain-iterations/sec", "n_gpus": world,
        "steps": 1, "warmup": 1, "ms_per_step": elapsed * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (M71 truth prior at the real source density, seed 2000+rank)",
        "config": {"workload": f"MCMC: {B} x 8x8 M71 cutouts/GPU, one chain each, S={S}, "
                               f"{total} samples, burn-in {burnin}, every {keep}th kept",
                   "tiles_per_gpu": B, "sources": S, "samples": total,
                   "parallelism": f"image-sharded x{world}"},
        "per_image_runtime_s": elapsed / B,
        "acc_rate": float(s.accept.float().mean()),
    }


def pmc_summary(args):
    """The committed PMC summary of the C2 MH launch, or (None, reason).  A
    summary measured on other library sources than the loaded library's is
    stale: its counters do not describe this run's kernel."""
    fname = PMC_FILES.get(args.workload)
    if fname is None or args.kernel != "mh" or args.full_recompute:
        return None, "no PMC summary for this workload"
    if REHEARSAL:
        return None, "host rehearsal (no kernel)"
    if args.workload == "c2" and (args.total_tiles > 0 or args.tiles_per_gpu != 1):
        return None, "no PMC summary for this tile count"
    path = os.path.join(ROOT, "profiles", fname)
    if not os.path.exists(path):
        return None, f"profiles/{fname} missing"
    try:
        d = json.load(open(path))
    except Exception as e:  # never fail the bench line on it
        return None, repr(e)
    from smcdet_amd import _hip
    built = _hip.built_hash()
    if d.get("source_hash") != built:
        return None, (f"stale: profiles/{fname} was measured on library sources "
                      f"{d.get('source_hash')}, this library is {built}")
    return d, f"profiles/{fname}"


def roofline_valu(args, mh_rate, f_alg, launch_steps, mh_ms, tile):
    """The binding resource's roofline (FP32 VALU, the MH sweep
    is not HBM-bound): achieved = §8d's 68.04 kFLOP per particle-step of the
    reference's full re-render x the sweep's particle-steps/s over the timed
    steps' own launches, against the FP32 vector peak.  `issue`: the executed
    instruction stream (the PMC pass's VALU and transcendental
    wave-instructions per particle-step) against its calibrated issue floor
    (issue_floor, ISSUE_MODEL at the sweep's waves per SIMD), over the SIMD
    cycles the launch had per particle-step at its measured clock."""
    tf = mh_rate * f_alg / 1e12
    out = {"bound": "valu", "achieved": tf, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
           "frac": tf / FP32_PEAK_TFLOPS, "alg_flop_per_particle_step": f_alg,
           "kernel_ms": mh_ms,
           "note": "reference-equivalent FLOPs (SURVEY §8d: the full re-render the reference "
                   "executes per particle-step); the incremental sweep executes fewer"}
    d, src = pmc_summary(args)
    if d is None:
        out["issue"] = {"omitted": src}
        return out
    try:
        clk = (d.get("effective_clock") or {}).get("ghz") or 2.4
        out["issue"] = dict(issue_floor(d["per_particle_step"], tile, clk, mh_ms, launch_steps),
                            model=ISSUE_MODEL["floor"], probe=ISSUE_MODEL["probe"], source=src)
    except Exception as e:  # never fail the bench line on it
        out["issue"] = {"error": repr(e)}
    return out


def compute_block(args, mh_rate, f_alg, launch_steps, mh_ms, tile):
    """The binding resource (FP32 VALU issue).  reference_equivalent: SURVEY
    §8d's FLOPs of the reference's full re-render per particle-step, which the
    incremental kernel does not execute.  executed: from the kernel's own VALU
    instruction counts (rocprofv3 PMC pass, profiles/PMC_FILES, same
    workload): the FP32 FLOPs they execute (64 lanes; FMA 2, packed x2) and
    the stream against its calibrated issue floor (issue_floor)."""
    out = {"bound": "valu", "mh_particle_steps_per_s": mh_rate,
           "reference_equivalent": {
               "alg_flop_per_particle_step": f_alg,
               "tflops": mh_rate * f_alg / 1e12, "peak_fp32_tflops": FP32_PEAK_TFLOPS,
               "frac": mh_rate * f_alg / 1e12 / FP32_PEAK_TFLOPS}}
    d, src = pmc_summary(args)
    if d is None:
        out["executed"] = {"omitted": src}
        return out
    try:
        per_step = d["per_particle_step"]
        # SQ_INSTS_VALU_FLOPS_FP32(_TRANS) count FLOPs per wave-instruction
        # (FMA 2, packed 2x): x 64 lanes
        flops = 64 * per_step["fp32_flop"] * launch_steps
        t = mh_ms * 1e-3
        clk = d.get("effective_clock") or {}
        out["executed"] = {
            "fp32_flop_per_particle_step": 64 * per_step["fp32_flop"],
            "tflops": flops / t / 1e12, "frac": flops / t / 1e12 / FP32_PEAK_TFLOPS,
            "issue": issue_floor(per_step, tile, clk.get("ghz") or 2.4, mh_ms, launch_steps),
            "effective_clock_source": clk.get("note"),
            "source": src, "source_hash": d.get("source_hash")}
    except Exception as e:  # never fail the bench line on it
        out["executed"] = {"error": repr(e)}
    return out


def vs_reference(dev, which="c2_moderate", n_runs=128):
    """North-star parity at the headline geometry, outside the timed region:
    the reference's recorded runs (tests/golden/stats_<which>.json: one 32x32
    M71 tile, S=10, N=4096 at K=100 (8 seeds) or K=20 (20 seeds), or N=512,
    K=20 (32 seeds), systematic) against n_runs runs
    of this sampler on the same image -- one launch grid of n_runs independent
    copies of the tile (independent stopping = one single-tile run per copy,
    each with its own Philox streams).  Means and standard errors of log Z,
    final ESS and SMC iterations."""
    import numpy as np
    from smcdet_amd.images import M71ImageModel
    from smcdet_amd.kernel import SingleComponentMH
    from smcdet_amd.prior import M71Prior
    from smcdet_amd.sampler import SMCsampler
    path = os.path.join(ROOT, "tests", "golden", f"stats_{which}.json")
    if not os.path.exists(path):
        return None
    ref = json.load(open(path))
    cfg, rr = ref["config"], ref["runs"]
    p, H, S, N, K = M71, cfg["tile"], cfg["S"], cfg["N"], cfg["K"]
    model = M71ImageModel(image_height=H, image_width=H, background=p["background"],
                          psf_radius=p["psf_radius"], adu_per_nmgy=p["adu_per_nmgy"],
                          psf_params=p["psf_params"], noise_additive=p["noise_additive"],
                          noise_multiplicative=p["noise_multiplicative"])
    prior = M71Prior(min_objects=S, max_objects=S, counts_rate=COUNTS_RATE_C2, image_height=H,
                     image_width=H, flux_alpha=p["flux_alpha"], flux_lower=p["flux_lower"],
                     flux_upper=p["flux_upper"], pad=4)
    img = torch.tensor(ref["image"], dtype=torch.float32, device=dev)
    tiles = img.reshape(1, 1, H, H).expand(1, n_runs, H, H).contiguous()
    mh = SingleComponentMH(K, 0.1, 2.5, p["flux_lower"], p["flux_upper"])
    s = SMCsampler.from_tiles(tiles, prior, model, mh, N, cfg["rho"], cfg["method"],
                              p["flux_detection_threshold"], cfg.get("max_smc_iters", 1000),
                              print_every=10 ** 9, seed=4242, device=dev,
                              stopping="independent")
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        s.run()
    lz = s.log_normalizing_constant.flatten().double().cpu().numpy()
    fe = s.ess.flatten().double().cpu().numpy()
    it = s.iters_per_tile.flatten().double().cpu().numpy()

    def ms(a):
        a = np.asarray(a, dtype=np.float64)
        return {"mean": float(a.mean()), "se": float(a.std(ddof=1) / np.sqrt(a.size)),
                "median": float(np.median(a)), "n": int(a.size)}

    kind = "oracle" if cfg.get("source") == "oracle" else "reference"
    out = {"target": f"tests/golden/stats_{which}.json ({len(rr)} {kind} runs; "
                     f"{H}x{H}, S={S}, N={N}, K={K})"}
    lz_ref = np.array([r["logZ"] for r in rr], dtype=np.float64)
    cut = float(np.median(lz_ref) - 40.0)  # the lower mode sits ~70 nats below the main one
    out["lower_mode_share"] = {"cut": cut, "ours": float((lz < cut).mean()),
                               "reference": float((lz_ref < cut).mean())}
    for key, ours, theirs in (("log_Z", lz, [r["logZ"] for r in rr]),
                              ("final_ess", fe, [r["final_ess"] for r in rr]),
                              ("iterations", it, [r["iters"] for r in rr])):
        a, b = ms(ours), ms(theirs)
        pooled = float(np.hypot(a["se"], b["se"]))
        out[key] = {"ours": a, "reference": b,
                    "rel_diff": (a["mean"] - b["mean"]) / abs(b["mean"]),
                    "diff_in_pooled_se": (a["mean"] - b["mean"]) / pooled if pooled else None}
    # the count posterior (sampler.py:198-219, 262-266): each run's pruned-count
    # histogram and pruned mean total flux, compared as tests/_stats.py does
    # (tests/test_gpu_statistical.py::test_c2_count_posterior's gates)
    if all("pruned_hist" in r and "mean_total_flux_pruned" in r for r in rr):
        from tests._stats import count_posterior_compare, hist_var
        pc = s.pruned_counts.reshape(n_runs, -1)
        hists = torch.stack([torch.bincount(pc[i], minlength=S + 1)[:S + 1] for i in range(n_runs)])
        hists = (hists.double() / pc.shape[-1]).cpu().numpy()
        pflux = s.posterior_mean_total_flux(s.pruned_fluxes).reshape(-1).double().cpu().numpy()
        ours = [{"pruned_hist": h, "mean_total_flux_pruned": float(f)} for h, f in zip(hists, pflux)]
        floor = None
        if kind == "reference":
            opath = os.path.join(ROOT, "tests", "golden", f"stats_{which}_oracle.json")
            if os.path.exists(opath):
                floor = hist_var(json.load(open(opath))["runs"], S + 1)
        cp = count_posterior_compare(ours, rr, var_floor=floor, nbins=S + 1)
        cp["gates"] = ("every bin within 3 pooled SE; TV <= 0.05 against the 648-run oracle "
                       "target; pruned flux within 3 pooled SE" +
                       ("; reference per-bin variance floored at the oracle's" if floor is not None
                        else ""))
        out["count_posterior"] = cp
    return out


def _full_run(s2):
    """One complete run() on a fresh sampler: initialise, the SMC loop with its
    per-iteration stopping check, final resample, prune."""
    import contextlib
    import io
    s2.print_every = 10 ** 9
    s2.max_smc_iters = 500
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        s2.run()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def c3_leg(args, dev, rank, world, dist, backend):
    """BASELINE configs[2] (C3) riding along the default C2 run: the 64 32x32
    tiles split contiguously over the ranks (--total-tiles 64 semantics: tile
    g drawn from seed 1000 + g whatever the rank count), timed like the main
    line (warmup, barrier + synchronize on both sides, MAX over ranks).  Every
    rank runs it, so the driver's N = 1, 2, 4, 8 runs of the default command
    measure C3's strong scaling too.  The value is the whole job's
    particle-steps/s."""
    import argparse as _ap
    import torch.distributed as tdist
    a3 = _ap.Namespace(**vars(args))
    a3.total_tiles, a3.tiles_per_gpu = C3_TILES, 1
    s, _, _, _, cfg = build_sampler(a3, dev, rank)
    s.fused_step = False
    s.initialize()
    s._temper_reweight(with_resample=True)

    def step():
        idx, s._pending_idx = s._pending_idx, None
        s._step(idx)

    steps = max(3, min(args.steps, 10))
    for _ in range(2):
        step()
    _sync()
    if dist:
        tdist.barrier()
    _sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    _sync()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=dev if backend == "nccl" else "cpu",
                         dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t)
    value = C3_TILES * args.particles * args.mh_iters * steps / elapsed
    gather = catalog_gather(s, rank, world, dist, backend) if dist else None
    return {"metric": f"particle-steps/sec (C3: {C3_TILES} x 32x32 tiles, 4096 particles)",
            "value": value, "unit": "particle-steps/sec", "n_gpus": world, "steps": steps,
            "warmup": 2, "ms_per_step": elapsed / steps * 1e3, "scaling": "strong",
            "config": {"workload": cfg["workload"], "tiles_per_gpu_rank0": cfg["tiles_per_gpu"]},
            "catalog_gather": gather}


def workload_leg(args, dev, rank, world, dist, backend, name):
    """The other BASELINE configurations riding along the default C2 run,
    each a timed SMC step on resident data like the main line (warm-up,
    barrier + synchronize on both sides, MAX over ranks), plus the MH launch's
    own duration (dispatch-stamped HIP events, untimed pass) and its roofline:
      c4             configs[3]: 42 8x8 M71 cutouts per GPU (332 over 8 GPUs,
                     manuscript.tex:562), S=10, N=4096, K=100, batched;
      c5             configs[4]: CS-SMC over the same 42 cutouts, counts 0..6,
                     N=8192 per count;
      c3_rank_share  one rank's share of configs[2] on 8 GPUs: tiles 0..7 of
                     the 64 (seeds 1000..1007, distributed.shard_tiles(64, 8, 0)),
                     so 8 x its rate projects the 8-GPU C3 line (world 1 only)."""
    import argparse as _ap
    import torch.distributed as tdist
    from smcdet_amd import _hip
    a2 = _ap.Namespace(**vars(args))
    if name == "c3_rank_share":
        a2.workload, a2.total_tiles, a2.tiles_per_gpu = "c2", 8, 1
    else:
        a2.workload, a2.total_tiles, a2.tiles_per_gpu = name, 0, 42
    steps = max(3, min(args.steps, 10))
    # everything that can fail on one rank alone (the sampler's build, its
    # allocations, the warm-up steps) happens before the leg's first
    # collective, and the ranks agree on the outcome first: a failed rank
    # makes every rank skip the leg instead of leaving the others blocked in
    # its barrier
    err = None
    try:
        s, _, steps_per_step, _, cfg = build_sampler(a2, dev, rank)
        s.fused_step = False
        s.initialize()
        s._temper_reweight(with_resample=True)

        def step():
            idx, s._pending_idx = s._pending_idx, None
            s._step(idx)

        for _ in range(2):
            step()
        _sync()
    except Exception as e:  # reported, after the ranks agree
        err = repr(e)
    if dist:
        ok = torch.tensor([0 if err else 1], dtype=torch.int32,
                          device=dev if backend == "nccl" else "cpu")
        tdist.all_reduce(ok, op=tdist.ReduceOp.MIN)
        if int(ok) == 0 and err is None:
            err = "skipped: the leg failed on another rank"
    if err is not None:
        return {"error": err}
    if dist:
        tdist.barrier()
    _sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    _sync()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=dev if backend == "nccl" else "cpu",
                         dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t)
    _hip.launch_timing(steps)
    for _ in range(steps):
        step()
    _sync()
    ev = _hip.launch_timing_read(steps)
    _hip.launch_timing(0)
    mh_ms = sum(ev) / max(len(ev), 1)
    S_, HW_ = cfg["sources"], cfg["tile"] * cfg["tile"]
    b_alg = 24 * S_ + 8
    f_alg = S_ * min(289, HW_) * 20 + HW_ * 10
    mh_rate = steps_per_step / (mh_ms * 1e-3)
    out = {"value": (world if name != "c3_rank_share" else 1) * steps_per_step * steps / elapsed,
           "unit": "particle-steps/sec", "n_gpus": world if name != "c3_rank_share" else 1,
           "steps": steps, "warmup": 2, "ms_per_step": elapsed / steps * 1e3,
           "scaling": "weak", "config": cfg, "kernel_ms": mh_ms,
           "mh_particle_steps_per_launch": steps_per_step,
           "roofline": {"bound": "hbm", "achieved": b_alg * mh_rate / 1e9, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": b_alg * mh_rate / 1e9 / HBM_PEAK_GBS,
                        "alg_bytes_per_particle_step": b_alg,
                        "kernel_timing": f"HIP dispatch events, {len(ev)} launches"}}
    pmc, _ = pmc_summary(a2)
    out["roofline"]["traffic"] = pmc.get("hbm_bytes_per_launch") if pmc else None
    out["roofline_valu"] = roofline_valu(a2, mh_rate, f_alg, steps_per_step, mh_ms, cfg["tile"])
    out["compute"] = compute_block(a2, mh_rate, f_alg, steps_per_step, mh_ms, cfg["tile"])
    if name == "c3_rank_share":
        out["projected_8gpu_c3_value"] = 8 * out["value"]
        out["note"] = ("one rank's share (8 tiles) of the 64-tile C3 split at 8 GPUs, run on "
                       "this GPU alone; the 8-GPU figure is 8 x this rate (ranks share no "
                       "data path), a projection, not a measurement")
    return out


def catalog_gather(s, rank, world, dist, backend):
    """north_star's one collective: the end-of-run catalog gather of every
    rank's tiles (smcdet_amd.distributed.gather_tile_results: one gather to
    rank 0 per field, RCCL over xGMI for device tensors), timed after the C3
    leg with barrier + synchronize on both sides, MAX over ranks."""
    import torch.distributed as tdist
    from smcdet_amd.distributed import gather_tile_results
    T = s._T
    local = {"counts": s.counts.reshape(T, -1), "locs": s.locs.reshape(T, *s.locs.shape[2:]),
             "fluxes": s.fluxes.reshape(T, *s.fluxes.shape[2:]),
             "weights": s.weights.reshape(T, -1),
             "log_normalizing_constant": s.log_normalizing_constant.reshape(T),
             "ess": s.ess.reshape(T)}
    nbytes = sum(v.numel() * v.element_size() for v in local.values())
    gather_tile_results(local, C3_TILES, 8, rank, world)  # warm-up (communicator setup)
    _sync()
    tdist.barrier()
    t0 = time.perf_counter()
    out = gather_tile_results(local, C3_TILES, 8, rank, world)
    _sync()
    tdist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=s.device if backend == "nccl" else "cpu", dtype=torch.float64)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    res = {"backend": backend, "ms": float(t) * 1e3, "bytes_per_rank": nbytes,
           "fields": sorted(local)}
    if rank == 0:
        res["gathered_shape_locs"] = list(out["locs"].shape)
        res["gathered_device"] = str(out["locs"].device)
    return res


def _hip_fused(s):
    """Whether smcdet_mh_sweep_step runs this sampler's shapes as one launch."""
    from smcdet_amd import _hip
    mh = s.MutationKernel
    flags = _hip.SMCDET_MH_FULL_RECOMPUTE if getattr(mh, "full_recompute", False) else 0
    return bool(_hip.lib().smcdet_mh_sweep_step_fused(
        _hip.ref(s.ImageModel._cmodel()), int(s.counts.shape[-1]), int(s.locs.shape[-2]), flags))


def launch_ranks(n):
    """The driver's multi-GPU command (torch.distributed.run, one rank per GPU,
    rendezvous on 127.0.0.1) with this process's arguments, as a child."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    global REHEARSAL
    args = parse()
    if args.host_rehearsal:
        REHEARSAL = True
        os.environ["SMCDET_DIST_BACKEND"] = "gloo"
        args.no_kernel_timing = args.no_full_run = args.no_cpu_baseline = True
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start the driver's
        # torchrun command as a CHILD process (nothing has touched the GPU in
        # this process: no exec from a GPU-initialised process) and exit with
        # its status
        sys.exit(launch_ranks(args.gpus))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started "
                         f"WORLD_SIZE={os.environ['WORLD_SIZE']} ranks; they must agree")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("SMCDET_DIST_BACKEND", "nccl") != "nccl":
        local %= max(torch.cuda.device_count(), 1)  # rehearsal: ranks may share a GPU
    # a process group whenever torchrun launched us -- also at world size 1
    # (the driver's N = 1 SCALE run), so its barriers, MAX-over-ranks and the
    # catalog gather run through the same RCCL path as N = 2, 4, 8
    dist = world > 1 or ("MASTER_ADDR" in os.environ and "RANK" in os.environ)
    # backend "nccl" (= RCCL on ROCm) for the driver's multi-GPU runs;
    # SMCDET_DIST_BACKEND=gloo rehearses the same code path with several ranks
    # sharing one GPU (RCCL refuses two ranks on one device)
    backend = os.environ.get("SMCDET_DIST_BACKEND", "nccl")
    if dist:
        import torch.distributed as tdist
        if not REHEARSAL:
            torch.cuda.set_device(local)
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)
    if REHEARSAL:
        dev = torch.device("cpu")
    else:
        dev = torch.device("cuda", local if dist else 0)
        torch.cuda.set_device(dev)

    if args.workload not in ("c2", "agg") and args.tiles_per_gpu == 1:
        args.tiles_per_gpu = 42  # 332 M71 cutouts over 8 GPUs (manuscript.tex:562)
    if args.workload in ("mcmc", "agg"):
        out = (bench_mcmc if args.workload == "mcmc" else bench_agg)(args, dev, rank, world)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if dist:
            tdist.destroy_process_group()
        return
    s, mh, steps_per_step, cpu_tile, cfg = build_sampler(args, dev, rank)
    s.fused_step = args.fused_step
    s.ancestor_bins = not args.ancestor_indices
    # the random streams' state before the run: restart() reruns the identical
    # workload (Philox-keyed draws: same proposals, decisions, ladder)
    rng0 = dict(s.rng.state()) if hasattr(s, "rng") else None

    def restart():
        if rng0 is not None:
            s.rng.load_state(rng0)
        s.initialize()
        s._temper_reweight(with_resample=True)

    s.initialize()
    cfg = dict(cfg, ancestors="indices" if args.ancestor_indices else "bins")
    cfg = dict(cfg, step="two launches" if not args.fused_step else (
        "fused" if s._step_fusable() and _hip_fused(s) else "two launches (shape)"))
    s._temper_reweight(with_resample=True)

    from smcdet_amd import _hip

    def step():
        # one SMC iteration: the MH sweep from the ancestors, then temper /
        # reweight / next indices in the same launch (SMCsampler._step)
        idx, s._pending_idx = s._pending_idx, None
        s._step(idx)

    prewarm = None
    cold = None
    if args.prewarm_s > 0 and not REHEARSAL:
        # for the record: the same W + K steps timed from a cold chip first
        # (what the line measured before round 5), then the prewarm
        for _ in range(args.warmup):
            step()
        _sync()
        t_c = time.perf_counter()
        for _ in range(args.steps):
            step()
        _sync()
        cold_ms = (time.perf_counter() - t_c) / args.steps * 1e3
        cold = {"ms_per_step": cold_ms, "value": world * steps_per_step / (cold_ms * 1e-3),
                "note": "the same W warmup + K timed steps before the prewarm (this rank; "
                        "the chip's clock still ramping from idle)"}
        # the clock's ramp from idle, outside the measured run: untimed steps
        # until prewarm_s seconds have passed, then a fresh start of the same
        # sampler (initialise, first temper), so the timed steps are SMC
        # iterations W+1..W+K of a new run, as without the prewarm
        t_pw, n_pw = time.perf_counter(), 0
        while time.perf_counter() - t_pw < args.prewarm_s:
            for _ in range(10):
                step()
            n_pw += 10
            _sync()
        restart()
        prewarm = {"seconds": round(time.perf_counter() - t_pw, 3), "steps": n_pw,
                   "note": "untimed back-to-back steps before the warmup steps (the chip's "
                           "clock ramps up over its first ~60 busy steps after idle: C2 sweep "
                           "0.273 -> 0.246 ms, scripts/warmup_probe.py), then the sampler "
                           "restarts from initialize(); the timed steps are iterations "
                           "W+1..W+K of that fresh run", "cold": cold}
    for _ in range(args.warmup):
        step()
    _sync()
    if dist:
        tdist.barrier()
    _sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    _sync()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    end_state = [x.detach().clone() for x in (s.log_normalizing_constant, s.temperature,
                                              s.locs)] if not REHEARSAL else None
    # The roofline's kernel durations describe the TIMED steps themselves: the
    # sampler restarts from the same random-stream state and replays the
    # identical W warmup + K timed SMC iterations (same draws, decisions and
    # temperature ladder; replay_identical checks the end state bit for bit),
    # this time with every launch of the K steps timed by HIP events stamped
    # on its own dispatch packet (hipExtLaunchKernel, smcdet_launch_timing):
    # the MH sweep and the per-tile temper / reweight / resampling pass.  Not
    # inside the timed region: per-launch timing leaves a 7-10 us bubble
    # before the next launch (profiles/r02_s3_gap_bench.txt), while untimed
    # back-to-back launches run gap-free.
    starts, tile_ev, replay = [], [], None
    if args.no_kernel_timing:
        ev = [elapsed * 1e3 / args.steps]
    else:
        restart()
        for _ in range(args.warmup):
            step()
        _sync()
        _hip.launch_timing(2 * args.steps)
        _hip.launch_timing_tiles(True)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step()
        _sync()
        replay_s = time.perf_counter() - t1
        ev_all = _hip.launch_timing_read(2 * args.steps)
        st_all = _hip.launch_timing_starts(2 * args.steps)
        _hip.launch_timing(0)
        if len(ev_all) == 2 * args.steps:  # two launches per step: sweep, tile pass
            ev, tile_ev, starts = ev_all[0::2], ev_all[1::2], st_all[0::2]
        else:                              # fused step: one launch per step
            ev, starts = ev_all, st_all
        same = all(torch.equal(a_, b_) for a_, b_ in zip(
            end_state, (s.log_normalizing_constant, s.temperature, s.locs)))
        replay = {"ms_per_step": replay_s / args.steps * 1e3, "replay_identical": bool(same),
                  "launches_timed": len(ev_all)}
    # step-time spread (untimed): the same W + K steps replayed 3 more times,
    # each bracketed like the timed region
    passes = []
    for _ in range(0 if args.no_spread else 3):
        restart()
        for _ in range(args.warmup):
            step()
        _sync()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step()
        _sync()
        passes.append((time.perf_counter() - t1) / args.steps * 1e3)
    if dist:
        t = torch.tensor([elapsed], device=dev if backend == "nccl" else "cpu",
                         dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t)
    mh_ms = sum(ev) / max(len(ev), 1)
    c3 = None
    if (args.workload == "c2" and args.kernel == "mh" and args.total_tiles == 0
            and args.tiles_per_gpu == 1 and not args.no_c3 and world <= C3_TILES):
        c3 = c3_leg(args, dev, rank, world, dist, backend)

    legs = {}
    if (args.workload == "c2" and args.kernel == "mh" and args.total_tiles == 0
            and args.tiles_per_gpu == 1 and not args.no_legs and not REHEARSAL):
        for name in ("c4", "c5") + (("c3_rank_share",) if world == 1 else ()):
            try:
                legs[name] = workload_leg(args, dev, rank, world, dist, backend, name)
            except Exception as e:  # report, never fail the bench line on it
                legs[name] = {"error": repr(e)}

    if args.total_tiles > 0:  # strong scaling: every rank's tiles, uneven shares included
        value = args.total_tiles * args.particles * args.mh_iters * args.steps / elapsed
    else:
        value = world * steps_per_step * args.steps / elapsed
    launch_steps = steps_per_step  # particle-steps per MH launch
    # SURVEY §8d per-particle-step figures, for this workload's S and tile
    S_, HW_ = cfg["sources"], cfg["tile"] * cfg["tile"]
    b_alg = 24 * S_ + 8
    f_alg = S_ * min(289, HW_) * 20 + HW_ * 10
    if args.kernel == "mala":
        # a MALA step needs the log target at the proposal and the gradient at
        # the current state and at the proposal, each an adjoint sweep costing
        # about one forward render: 3 x the MH figure
        f_alg *= 3
    achieved_gbs = b_alg * launch_steps / (mh_ms * 1e-3) / 1e9
    mh_rate = launch_steps / (mh_ms * 1e-3)
    pmc, _ = pmc_summary(args)
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    out = {
        "metric": ("particle-steps/sec (4096 particles, 32x32 tile)"
                   if args.workload == "c2" and args.kernel == "mh"
                   else f"particle-steps/sec ({args.workload} workload, {args.kernel})"),
        "value": value,
        "unit": "particle-steps/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if args.total_tiles > 0 else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (M71 prior + image model, seed 1000+rank)",
        "config": dict(cfg, mode="full" if args.full_recompute else "incremental",
                       parallelism=f"tile-sharded x{world}"),
        "prewarm": prewarm,
        "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": f"smcdet {args.kernel}_sweep_kernel", "kernel_ms": mh_ms,
                     "kernel_timing": ("step time (no timing pass)" if args.no_kernel_timing
                                       else f"HIP dispatch events on the {len(ev)} sweep "
                                            "launches of the timed steps, replayed identically "
                                            "(step_attribution)"),
                     "alg_bytes_per_particle_step": b_alg},
        "roofline_valu": roofline_valu(args, mh_rate, f_alg, launch_steps, mh_ms, cfg["tile"]),
        "compute": compute_block(args, mh_rate, f_alg, launch_steps, mh_ms, cfg["tile"]),
        "smc": {"temperature_min": float(s.temperature.min()),
                "acc_rate": float(s.mutation_acc_rates.mean()),
                "ess_mean": float(s.ess.mean())},
    }
    def pct(v):
        import numpy as np
        if len(v) == 0:
            return None
        a = np.asarray(v, dtype=np.float64)
        return {"min": float(a.min()), "p50": float(np.percentile(a, 50)),
                "p90": float(np.percentile(a, 90)), "max": float(a.max()), "n": int(a.size)}

    import numpy as _np
    out["step_spread"] = {
        "timed_ms_per_step": elapsed / args.steps * 1e3,
        "repeat_passes_ms_per_step": passes,
        "launch_interval_ms": pct(_np.diff(starts)) if len(starts) > 1 else None,
        "kernel_ms": pct(ev),
        "note": "untimed: the timed steps replayed 3 more times, each bracketed like the timed "
                "region; sweep-launch start-to-start intervals and durations from the "
                "dispatch-stamped replay"}
    if replay is not None:
        # ms_per_step = sweep + tile pass + the rest (launch gaps, host enqueue
        # stalls), all over the timed steps' own workload
        sw_ms = mh_ms
        tl_ms = sum(tile_ev) / len(tile_ev) if tile_ev else 0.0
        step_ms = elapsed / args.steps * 1e3
        out["step_attribution"] = dict(
            replay, timed_ms_per_step=step_ms, sweep_ms=sw_ms, tile_pass_ms=tl_ms,
            gap_ms=step_ms - sw_ms - tl_ms, tile_pass_kernel_ms=pct(tile_ev),
            note="the timed region's W warmup + K SMC iterations replayed from the same "
                 "random-stream state with every sweep and tile-pass launch of the K steps "
                 "timed on its dispatch packet; gap = timed ms/step - sweep - tile pass")
    if c3 is not None:
        out["c3_strong"] = c3
    out.update(legs)
    # SURVEY §8d also asks for the wall time to temperature 1: one complete
    # run() (initialise, SMC loop with its per-iteration stopping check, final
    # resample, prune) on a fresh sampler, outside the timed region
    if args.no_full_run:
        s2 = None
    else:
        s2, _, _, _, _ = build_sampler(args, dev, rank)
    if s2 is not None:
        run_s = _full_run(s2)
        out["smc"]["run_to_tau1"] = {"iterations": int(s2.iter), "wall_s": run_s,
                                     "ms_per_iteration": run_s / max(int(s2.iter), 1) * 1e3,
                                     "temperature_min": float(s2.temperature.min())}
    if rank == 0 and args.workload == "c2" and args.kernel == "mh" and not args.no_vs_ref:
        # the headline configuration first (N = 4096, K = 100: tests/golden/
        # stats_c2_moderate_4096_k100.json), then N = 4096 at K = 20 (more
        # reference seeds) and the reduced-N target
        # ("vs_oracle_k100": the same configuration run to completion by the
        # CPU restatement of the reference's algorithm, 48 seeds, which
        # resolves the lower log Z mode the 8 reference runs happen to miss)
        for key, which in (("vs_reference", "c2_moderate_4096_k100"),
                           ("vs_oracle_k100", "c2_moderate_4096_k100_oracle"),
                           ("vs_reference_k20", "c2_moderate_4096"),
                           ("vs_reference_n512", "c2_moderate")):
            try:
                r = ({"rehearsal": f"vs_reference({which}) on rank {rank}"} if REHEARSAL
                     else vs_reference(dev, which))
            except Exception as e:  # report, never fail the bench line on it
                r = {"error": repr(e)}
            if r is not None:
                out["smc"][key] = r
    if REHEARSAL and rank == 0 and world == 1:
        out["cpu_baseline"] = {"rehearsal": f"cpu_baseline on rank {rank}"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "c2":
        try:
            out["cpu_baseline"] = cpu_baseline(args, cpu_tile.cpu().numpy(),
                                               args.cpu_baseline_seconds)
            out["cpu_baseline"]["reference_measured"] = REFERENCE_CPU
            cc = json.load(open(os.path.join(ROOT, CROSSCAL_FILE)))
            r = cc["port_over_reference"]
            out["cpu_baseline"]["calibration"] = {
                "port_over_reference": r,
                "reference_equivalent_value": out["cpu_baseline"]["value"] / r,
                "reference_8_threads_same_container": cc["reference"]["particle_steps_per_s"],
                "port_8_threads_same_container": cc["port"]["particle_steps_per_s"],
                "source": CROSSCAL_FILE,
                "note": "the reference's SingleComponentMH and this port on the same 8 cores "
                        "(build container; the reference does not travel to the GPU box); "
                        "reference_equivalent_value = this box's port rate / port_over_reference"}
        except Exception as e:  # report, never fail the bench line on it
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
