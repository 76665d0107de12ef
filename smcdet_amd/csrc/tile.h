// tile.h — per-tile SMC bookkeeping on device: adaptive tempering
// (sampler.py:93-125), reweighting / log-evidence / ESS (sampler.py:181-196)
// and the next resampling indices (sampler.py:127-169), as one workgroup's
// work over one tile's N particles.
//
// Two callers: tile_kernel (smc_kernels.hip, one 512-thread workgroup per
// tile) and the MH sweep's tail (mh_kernel.hip: the tile's last-finishing
// 256-thread workgroup runs it right after its own particles, so an SMC
// iteration is one launch).  Both compute on the same *virtual* layout of
// kTB = 512 threads: a physical thread of an NT-thread workgroup plays the
// virtual threads tid + h*NT (h < 512/NT), virtual wave `wave + h*NT/64`
// being physical wave `wave`'s lanes.  Every reduction, scan and Brent step
// is therefore the same sequence of float operations whichever workgroup
// runs it: the fused and the separate launch give bit-identical temperatures,
// weights and indices.
//
// ESS(delta) is monotone, but brentq stops within xtol = 1e-6 of the root,
// which early in a run is as large as delta itself: the tempering schedule
// (and so the iteration count) is brentq's, not the exact root's.  The root
// is therefore found by the same Brent iteration as scipy's brentq, each f
// evaluation being a workgroup-wide reduction.
#pragma once

#include <math.h>

#include <type_traits>

#include "device.h"

namespace smcdet {

// (profiling builds: the phase-timestamp table of the including file)
SMCDET_TRACE_TABLE

constexpr int kTB = 512;            // virtual threads of the tile layout
constexpr int kTW = kTB / kWave;    // 8 virtual waves
constexpr int kMaxPer = 32;         // log-likelihoods per virtual thread
constexpr int kMaxN = kTB * kMaxPer;

enum : uint32_t { kDoTemper = 1u, kDoWeights = 2u, kDoResample = 4u };

struct TileArgs {
  uint32_t flags;
  int T, N;
  double ess_threshold;
  const float* loglik;       // [T,N]
  float* temperature;        // [T]
  float* temperature_prev;   // [T]
  float* log_w;              // [T,N]
  float* weights;            // [T,N]
  float* ess;                // [T]
  float* logZ;               // [T]
  int method;                // SMCDET_RESAMPLE_*
  uint32_t k0, k1;
  uint64_t offset;
  const float* u;            // replay uniforms or null
  int64_t* idx;              // [T,N]
  uint32_t smc_flags;        // SMCDET_SMC_*
  int32_t* fin_iter;         // [T] SMC iteration a tile reached temperature 1 (-1: not yet) or null
  int32_t iter;              // the caller's SMC iteration number
  int32_t* live;             // [3] zeroed, 8-byte aligned: count, ticket, tiles below 1 (or null)
  const int32_t* go;         // predicate: skip the launch when *go == 0 (or null)
  int32_t* live_host;        // host-mapped copy of live[2] (pinned host memory) or null
  float* bins_out;           // [T*N + 65T] bins, offsets U, chunk ends, instead of idx (or null)
};

// one tile pass launch (smc_kernels.hip)
int launch_tile(const TileArgs& a, hipStream_t st);

// The systematic ancestor of particle n, idx[n] = #{i : bins[i] < u_n}
// clamped to N - 1, u_n = (n + U)/N in float32 (sampler.py:141-148), found by
// the 64 lanes of a wave in the monotone bins (global memory, L2-resident): a
// 64-ary search, log64(N) dependent loads (two at N = 4096).  The first level
// reads the tile's 64 chunk ends from `coarse` (kBinsCoarse contiguous floats,
// written by the tile pass: one 256-byte read instead of 64 cache lines per
// wave) when it is given.  The test is the tile pass's (bins[i] < u_n, for N a
// power of two as b*N < fl(n + U), exact), so the index is the one the tile
// pass's search would write.  Call from converged code; the result is
// wave-uniform.
constexpr int kBinsCoarse = 64;
__device__ __forceinline__ int bins_ancestor(const float* __restrict__ bins,
                                             const float* __restrict__ coarse, int N, float U,
                                             int n) {
  const int lane = threadIdx.x & 63;
  const float Nf = (float)N;
  const bool pow2 = (N & (N - 1)) == 0;
  const float nu = (float)n + U;
  const float key = pow2 ? nu : nu / Nf;
  int lo = 0, len = N;
  bool first = coarse != nullptr;
  while (true) {
    // chunk l = [l*step, min((l+1)*step, len)) of [lo, lo+len): its last bin
    // below the key means the whole chunk is (bins are monotone)
    const int step = (len + 63) >> 6;
    const bool valid = lane * step < len;
    const float b = !valid ? 0.f
                  : first ? coarse[lane]
                          : bins[lo + min((lane + 1) * step, len) - 1];
    first = false;
    const bool less = valid && (pow2 ? (b * Nf < key) : (b < key));
    const int c = __popcll(__ballot(less));
    if (step == 1) return min(lo + c, N - 1);
    if (c * step >= len) return min(lo + len, N - 1);
    lo += c * step;
    len = min(step, len - c * step);
  }
}

// the chunk-end index of coarse entry l: min((l+1)*c, N) - 1, c = ceil(N/64)
__device__ __forceinline__ int bins_coarse_end(int l, int N) {
  const int c = (N + kBinsCoarse - 1) / kBinsCoarse;
  return min((l + 1) * c, N) - 1;
}

// end-of-temper bookkeeping, thread 0 of each tile: the iteration at which the
// tile reached temperature 1, and (last tile, by ticket) the number of tiles
// still below 1 -- the reference's while condition (sampler.py:230) without
// extra launches; the counter and ticket are zero again afterwards
// The count reaches its readers across a launch boundary (the next sweep's
// `go`; the host after this launch's completion event), which orders it: no
// system-scope fence here, and no agent-scope one between the tiles' counts
// and tickets either (one 64-bit atomic carries both): such a fence is an L2
// write-back, on the tile pass's path right after the sweep filled the L2
// with rate images.
__device__ __forceinline__ void tile_status(const TileArgs& a, int t, float tnew) {
  if (a.fin_iter && tnew >= 1.0f && a.fin_iter[t] < 0) a.fin_iter[t] = a.iter;
  if (!a.live) return;
  int nlive = tnew < 1.0f ? 1 : 0;
  if (a.T > 1) {
    // count (high word) and ticket (low word) of live[0..1] in one 64-bit
    // atomic: the last tile reads every other tile's count in the value it
    // replaces, no fence between a count and a ticket (live: 8-byte aligned)
    unsigned long long* slot = reinterpret_cast<unsigned long long*>(a.live);
    const unsigned long long old = atomicAdd(slot, ((unsigned long long)nlive << 32) | 1ull);
    if ((int)(old & 0xffffffffull) != a.T - 1) return;
    nlive += (int)(old >> 32);
    atomicExch(slot, 0ull);
  }
  a.live[2] = nlive;
  // the host reads it after the launch completes: no copy launch
  if (a.live_host) *reinterpret_cast<volatile int32_t*>(a.live_host) = nlive;
}

// Per-virtual-wave partials of the workgroup reductions, double-buffered.
// `parity` lives in registers and toggles identically in every thread, so a
// buffer is not rewritten before all threads passed the next call's barrier.
struct TileRed {
  double d[2][kTW][2];
  float f[2][kTW];
  float f2[2][kTW][2];
  int i[2][kTW];
};

template <int NT>
struct VLayout {
  static_assert(NT % kWave == 0 && kTB % NT == 0, "NT must divide the 512-thread layout");
  static constexpr int VPT = kTB / NT;  // virtual threads per physical thread
  static constexpr int NW = NT / kWave;
};
template <int NT>
__device__ __forceinline__ int vthread(int h) {
  return (int)threadIdx.x + h * NT;
}
template <int NT>
__device__ __forceinline__ int vwave(int h) {
  return ((int)threadIdx.x >> 6) + h * VLayout<NT>::NW;
}

// Workgroup reductions with ONE barrier each: wave DPP reductions per virtual
// wave -> its slot -> the kTW slots combined in a fixed order (deterministic;
// every thread ends with the same value).
//
// The combine: lane i < 8 of every wave reads slot i of the first sum, lane
// 8 + i slot i of the second, one LDS read per lane, then a pairwise tree over
// the 8 lanes (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror: lane 0 ends
// with ((s0+s1)+(s2+s3))+((s4+s5)+(s6+s7)), lane 8 likewise), read back with
// v_readlane.  Every thread reading every slot instead moved 16-64 KB through
// the LDS return path per reduction at 512 threads (~130-500 cycles on the
// Brent path: scripts/probe/brent_probe.hip).
static_assert(kTW == 8, "the slot combine is an 8-lane tree");
__device__ __forceinline__ double readlane_d(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ void slot_tree2(float v, float& A, float& B) {
  v += dpp_f<0xb1>(v);
  v += dpp_f<0x4e>(v);
  v += dpp_f<0x141>(v);
  A = readlane(v, 0);
  B = readlane(v, 8);
}
__device__ __forceinline__ void slot_tree2(double v, double& A, double& B) {
  v += dpp_d<0xb1>(v);
  v += dpp_d<0x4e>(v);
  v += dpp_d<0x141>(v);
  A = readlane_d(v, 0);
  B = readlane_d(v, 8);
}
template <int NT>
__device__ __forceinline__ double vblock_sumd(const double (&a)[VLayout<NT>::VPT], TileRed* r,
                                              int& parity) {
  const int lane = threadIdx.x & 63;
  const int k = parity;
  parity ^= 1;
#pragma unroll
  for (int h = 0; h < VLayout<NT>::VPT; ++h) {
    const double s = wave_sum(a[h]);
    if (lane == 0) r->d[k][vwave<NT>(h)][0] = s;
  }
  __syncthreads();
  double sa, sb;
  slot_tree2(r->d[k][lane & 7][0], sa, sb);
  return sa;
}
template <int NT>
__device__ __forceinline__ void vblock_sum2d(const double (&a)[VLayout<NT>::VPT],
                                             const double (&b)[VLayout<NT>::VPT], double& A,
                                             double& B, TileRed* r, int& parity) {
  const int lane = threadIdx.x & 63;
  const int k = parity;
  parity ^= 1;
#pragma unroll
  for (int h = 0; h < VLayout<NT>::VPT; ++h) {
    const double x = wave_sum(a[h]);
    const double y = wave_sum(b[h]);
    if (lane == 0) {
      r->d[k][vwave<NT>(h)][0] = x;
      r->d[k][vwave<NT>(h)][1] = y;
    }
  }
  __syncthreads();
  slot_tree2(r->d[k][lane & 7][(lane >> 3) & 1], A, B);
}
template <int NT>
__device__ __forceinline__ void vblock_sum2f(const float (&a)[VLayout<NT>::VPT],
                                             const float (&b)[VLayout<NT>::VPT], float& A,
                                             float& B, TileRed* r, int& parity) {
  const int lane = threadIdx.x & 63;
  const int k = parity;
  parity ^= 1;
#pragma unroll
  for (int h = 0; h < VLayout<NT>::VPT; ++h) {
    float x = a[h], y = b[h];
    wave_sum2(x, y);
    if (lane == 0) {
      r->f2[k][vwave<NT>(h)][0] = x;
      r->f2[k][vwave<NT>(h)][1] = y;
    }
  }
  __syncthreads();
  slot_tree2(r->f2[k][lane & 7][(lane >> 3) & 1], A, B);
}
template <int NT>
__device__ __forceinline__ float vblock_max(const float (&v)[VLayout<NT>::VPT], TileRed* r,
                                            int& parity) {
  const int lane = threadIdx.x & 63;
  const int k = parity;
  parity ^= 1;
#pragma unroll
  for (int h = 0; h < VLayout<NT>::VPT; ++h) {
    const float m = wave_max(v[h]);
    if (lane == 0) r->f[k][vwave<NT>(h)] = m;
  }
  __syncthreads();
  float m = r->f[k][lane & 7];
  m = fmaxf(m, dpp_fmax<0xb1>(m));
  m = fmaxf(m, dpp_fmax<0x4e>(m));
  m = fmaxf(m, dpp_fmax<0x141>(m));
  return readlane(m, 0);
}

// the 512-thread forms (aggregation kernels)
__device__ __forceinline__ float block_max(float v, TileRed* r, int& parity) {
  const float a[1] = {v};
  return vblock_max<kTB>(a, r, parity);
}
__device__ __forceinline__ void block_sum2(double& a, double& /*unused*/, TileRed* r,
                                           int& parity) {
  const double x[1] = {a};
  a = vblock_sumd<kTB>(x, r, parity);
}

// Pairwise (depth log2 PER) sum of a register array: short dependency chains,
// which is what a one-workgroup-per-tile pass with nothing to hide latency
// behind needs.
template <class V, int PER>
__device__ __forceinline__ V tree_sum(V (&x)[PER]) {
#pragma unroll
  for (int w = 1; w < PER; w <<= 1) {
#pragma unroll
    for (int j = 0; j + w < PER; j += 2 * w) x[j] += x[j + w];
  }
  return x[0];
}

// a / b by v_rcp_f64 + two Newton steps + one residual correction: the
// quotient to the last bit or so, without the IEEE division sequence's scale /
// fixup steps on the latency-bound Brent path (b = 0 or inf gives a NaN/inf
// step, which the Brent tests reject exactly as they reject scipy's)
__device__ __forceinline__ double ddiv(double a, double b) {
  double r = __builtin_amdgcn_rcp(b);
  r = fma(fma(-b, r, 1.0), r, r);
  r = fma(fma(-b, r, 1.0), r, r);
  const double q = a * r;
  return fma(fma(-b, q, a), r, q);
}

// The log-likelihoods of virtual thread v (i = v + j*kTB) live in registers
// for the whole tempering search.
template <int NT, int PER>
struct TileLL {
  float l[VLayout<NT>::VPT][PER];
  __device__ __forceinline__ bool valid(int h, int j, int N) const {
    return vthread<NT>(h) + j * kTB < N;
  }
};

// f(delta) = ESS(delta) - threshold: ESS = (sum e)^2 / sum e^2,
// e = exp(d*l - max(d*l)), d = float32(delta) (the reference multiplies its
// float32 log-likelihoods by the python float delta and reduces in float32;
// sampler.py:93-97).  Sums are float32 pairwise trees (relative error ~1e-6,
// the reference's own float32 logsumexp level); only the ratio is double.
// This sits on the latency-bound path of every Brent iteration, so it is
// short: one exp per element, float DPP reductions, one barrier.
//
// In gfx950's packed float ops: element j is paired with element j + PER/2
// (v_pk_mul / v_pk_add: the same roundings per element), the pairs summed by
// a pairwise tree and the two halves added last -- for PER a power of two
// exactly tree_sum's order over the PER elements.  Tiles of exactly kTB * PER
// particles skip the per-element bounds masks.
template <int NT, int PER>
__device__ __forceinline__ double block_ess_objective(const TileLL<NT, PER>& ll, int N,
                                                      float lmax, double delta, double thr,
                                                      TileRed* red, int& parity) {
#pragma clang fp contract(off)
  constexpr int VPT = VLayout<NT>::VPT;
  const float df = (float)delta;
  const float m = df * lmax;
  float s1[VPT], s2[VPT];
  auto sums = [&](auto full) {
#pragma unroll
    for (int h = 0; h < VPT; ++h) {
      if constexpr (PER % 2 == 0) {
        constexpr int H = PER / 2;
        f2 E[H], Q[H];
#pragma unroll
        for (int k = 0; k < H; ++k) {
          f2 v = f2{ll.l[h][k], ll.l[h][k + H]} * df;
          v = (v - m) * kLog2e;
          f2 e = exp2_2(v);
          if constexpr (!decltype(full)::value) {
            e.x = ll.valid(h, k, N) ? e.x : 0.f;
            e.y = ll.valid(h, k + H, N) ? e.y : 0.f;
          }
          E[k] = e;
          Q[k] = e * e;
        }
        const f2 se = tree_sum(E), sq = tree_sum(Q);
        s1[h] = se.x + se.y;
        s2[h] = sq.x + sq.y;
      } else {
        float e1[PER], e2[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
          const float e = ll.valid(h, j, N) ? fast_exp2((df * ll.l[h][j] - m) * kLog2e) : 0.f;
          e1[j] = e;
          e2[j] = e * e;
        }
        s1[h] = tree_sum(e1);
        s2[h] = tree_sum(e2);
      }
    }
  };
  if (N == kTB * PER) sums(std::true_type{});
  else sums(std::false_type{});
  float S1, S2;
  vblock_sum2f<NT>(s1, s2, S1, S2, red, parity);
  const double d1 = (double)S1;
  return ddiv(d1 * d1, (double)S2) - thr;
}

// scipy.optimize.brentq (scipy/optimize/Zeros/brentq.c, the algorithm the
// reference calls at sampler.py:114-120) with xtol = rtol = 1e-6, maxiter
// 100.  Every thread runs the (deterministic) control flow on identical
// values; the workgroup evaluates f together.  (brentq.c's branches stay
// branches: a select form computing every candidate step measured 745-787
// vs 644-675 cycles of control per iteration, round 4's
// scripts/probe/brent_probe.hip, as in round 2.)
template <class F>
__device__ double block_brentq(F&& f, double xa, double xb, double fa, double fb) {
#pragma clang fp contract(off)
  const double xtol = 1e-6, rtol = 1e-6;
  double xpre = xa, xcur = xb, xblk = 0., fpre = fa, fcur = fb, fblk = 0., spre = 0., scur = 0.;
  if (fpre == 0.0) return xpre;
  if (fcur == 0.0) return xcur;
  for (int it = 0; it < 100; ++it) {
    if (fpre != 0 && fcur != 0 && (signbit(fpre) != signbit(fcur))) {
      xblk = xpre;
      fblk = fpre;
      spre = scur = xcur - xpre;
    }
    if (fabs(fblk) < fabs(fcur)) {
      xpre = xcur; xcur = xblk; xblk = xpre;
      fpre = fcur; fcur = fblk; fblk = fpre;
    }
    const double delta = (xtol + rtol * fabs(xcur)) / 2;
    const double sbis = (xblk - xcur) / 2;
    if (fcur == 0 || fabs(sbis) < delta) return xcur;
    if (fabs(spre) > delta && fabs(fcur) < fabs(fpre)) {
      double stry;
      if (xpre == xblk) {
        stry = ddiv(-fcur * (xcur - xpre), fcur - fpre);  // interpolate
      } else {                                         // extrapolate
        const double dpre = ddiv(fpre - fcur, xpre - xcur);
        const double dblk = ddiv(fblk - fcur, xblk - xcur);
        stry = ddiv(-fcur * (fblk * dblk - fpre * dpre), dblk * dpre * (fblk - fpre));
      }
      if (2 * fabs(stry) < fmin(fabs(spre), 3 * fabs(sbis) - delta)) {
        spre = scur;
        scur = stry;
      } else {
        spre = sbis;
        scur = sbis;
      }
    } else {
      spre = sbis;
      scur = sbis;
    }
    xpre = xcur;
    fpre = fcur;
    if (fabs(scur) > delta) xcur += scur;
    else xcur += (sbis > 0 ? delta : -delta);
    fcur = f(xcur);
  }
  return xcur;
}

// One tile's temper -> reweight -> resample-index pass (a.flags select the
// parts) by an NT-thread workgroup.  buf: 2N+1 words of LDS (weights /
// cumsum, then N+1 resampling slots).  trow: SMC_TRACE row (-1: none).
template <int NT, int PER>
__device__ __forceinline__ void tile_work(const TileArgs& a, int t, float* buf, TileRed& red,
                                          [[maybe_unused]] int trow) {
#pragma clang fp contract(off)
  constexpr int VPT = VLayout<NT>::VPT;
  int parity = 0;
  const int N = a.N;
  const int lane = threadIdx.x & 63;

  SMC_TRACE(trow, 0);
  // independent stopping: a finished tile stays as it is (uniform weights of
  // its final resampled population, identity ancestors, log Z unchanged)
  if ((a.smc_flags & SMCDET_SMC_FREEZE_DONE) && a.temperature[t] >= 1.0f) {
    if ((a.flags & kDoTemper) && threadIdx.x == 0) {
      a.temperature_prev[t] = a.temperature[t];
      tile_status(a, t, a.temperature[t]);
    }
    if (a.flags & kDoWeights) {
      for (int i = threadIdx.x; i < N; i += NT) {
        a.log_w[(size_t)t * N + i] = 0.0f;
        a.weights[(size_t)t * N + i] = 1.0f / (float)N;
      }
      // a.ess[t] keeps the ESS of the tile's last step, as a single-tile
      // run of the reference reports it after its final resample
    }
    if (a.flags & kDoResample) {
      if (a.bins_out && a.method == SMCDET_RESAMPLE_SYSTEMATIC) {
        // identity ancestors as bins: bins[i] = (i + 1)/N with U = 1/2 gives
        // #{i : bins[i] < (n + 1/2)/N} = n exactly (bins_ancestor's test)
        for (int i = threadIdx.x; i < N; i += NT)
          a.bins_out[(size_t)t * N + i] = (float)(i + 1) / (float)N;
        if (threadIdx.x == 0) a.bins_out[(size_t)a.T * N + t] = 0.5f;
        if (threadIdx.x < kBinsCoarse)
          a.bins_out[(size_t)a.T * (N + 1) + (size_t)t * kBinsCoarse + threadIdx.x] =
              (float)(bins_coarse_end(threadIdx.x, N) + 1) / (float)N;
      } else {
        for (int i = threadIdx.x; i < N; i += NT) a.idx[(size_t)t * N + i] = i;
      }
    }
    return;
  }
  TileLL<NT, PER> ll;
  if (a.flags & (kDoTemper | kDoWeights)) {
    const float* llg = a.loglik + (size_t)t * N;
#pragma unroll
    for (int h = 0; h < VPT; ++h)
#pragma unroll
      for (int j = 0; j < PER; ++j)
        ll.l[h][j] = ll.valid(h, j, N) ? llg[vthread<NT>(h) + j * kTB] : 0.f;
  }

  // ------------------------------------------------------------------ temper
  float d_new = 0.f;  // float32 temperature increment, when tempered here
  float lm_t = -INFINITY;  // the temper pass's max log-likelihood
  if (a.flags & kDoTemper) {
    const float tau = a.temperature[t];
    float lmv[VPT];
#pragma unroll
    for (int h = 0; h < VPT; ++h) {
      lmv[h] = -INFINITY;
#pragma unroll
      for (int j = 0; j < PER; ++j)
        if (ll.valid(h, j, N)) lmv[h] = fmaxf(lmv[h], ll.l[h][j]);
    }
    const float lm = vblock_max<NT>(lmv, &red, parity);
    lm_t = lm;
    SMC_TRACE(trow, 1);
    const double thr = a.ess_threshold;
    auto f = [&](double x) { return block_ess_objective(ll, N, lm, x, thr, &red, parity); };
    const double top = 1.0 - (double)tau;
    // sampler.py:113-122: root-find only if ESS at delta = 1 - tau is below threshold
    const double ftop = f(top);
    SMC_TRACE(trow, 2);
    double delta = top;
    // f(0) = N - thr exactly: every weight is exp(0) = 1
    if (ftop < 0.0) delta = block_brentq(f, 0.0, top, (double)N - thr, ftop);
    SMC_TRACE(trow, 3);
    const float tnew = tau + (float)delta;  // delta tensor is float32 (sampler.py:105)
    d_new = tnew - tau;
    if (threadIdx.x == 0) {
      a.temperature_prev[t] = tau;
      a.temperature[t] = tnew;
      tile_status(a, t, tnew);
    }
  }

  // ------------------------------------------------------------ update weights
  if (a.flags & kDoWeights) {
    const float d = (a.flags & kDoTemper) ? d_new : a.temperature[t] - a.temperature_prev[t];
    float* lwg = a.log_w + (size_t)t * N;
    float* wg = a.weights + (size_t)t * N;
    float e[VPT][PER];
    float mxv[VPT];
#pragma unroll
    for (int h = 0; h < VPT; ++h) {
      mxv[h] = -INFINITY;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        e[h][j] = nan_to_num(d * ll.l[h][j], -INFINITY);
        if (ll.valid(h, j, N)) {
          lwg[vthread<NT>(h) + j * kTB] = e[h][j];
          mxv[h] = fmaxf(mxv[h], e[h][j]);
        }
      }
    }
    // max of the weights' exponents: tempered here with a finite max
    // log-likelihood, it is fl(d * lmax) (d >= 0: rounding and nan_to_num
    // are monotone, the block_ess_objective argument), no reduction
    const float mt = d * lm_t;
    const float mx = ((a.flags & kDoTemper) && isfinite(mt)) ? mt
                                                            : vblock_max<NT>(mxv, &red, parity);
    double ssum[VPT], qsum[VPT];
#pragma unroll
    for (int h = 0; h < VPT; ++h) {
      double s[PER], q[PER];
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        e[h][j] = ll.valid(h, j, N) ? expf(e[h][j] - mx) : 0.f;
        s[j] = (double)e[h][j];
        q[j] = s[j] * s[j];
      }
      ssum[h] = tree_sum(s);
      qsum[h] = tree_sum(q);
    }
    // one reduction for the sum and the sum of squares: ESS = (sum e)^2 /
    // sum e^2 in double -- algebraically the reference's 1 / sum W^2
    // (sampler.py:189), which squares and sums the float32-rounded weights
    // W = softmax in float32; the two agree to float32 rounding (relative
    // ~1e-7), not bit for bit (a second reduction over W after sum e is known
    // would cost one more block barrier per tile pass)
    SMC_TRACE(trow, 7);
    double se, qe;
    vblock_sum2d<NT>(ssum, qsum, se, qe, &red, parity);
    SMC_TRACE(trow, 8);
    const float sf = (float)se;
#pragma unroll
    for (int h = 0; h < VPT; ++h) {
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const float wv = e[h][j] / sf;
        if (ll.valid(h, j, N)) {
          wg[vthread<NT>(h) + j * kTB] = wv;
          buf[vthread<NT>(h) + j * kTB] = wv;
        }
      }
    }
    SMC_TRACE(trow, 4);
    if (threadIdx.x == 0) {
      a.ess[t] = (float)(se * se / qe);
      a.logZ[t] = (a.logZ[t] + mx) + logf(sf / (float)N);
    }
  }

  // ---------------------------------------------------------- resample index
  if (a.flags & kDoResample) {
    if (!(a.flags & kDoWeights)) {
      const float* W = a.weights + (size_t)t * N;
      for (int i = threadIdx.x; i < N; i += NT) buf[i] = W[i];
    }
    __syncthreads();
    // bins = cumsum(W): float64 running sum rounded per element to float32
    // (what torch's CPU cumsum does), contiguous chunk per virtual thread, in place
    const int chunk = (N + kTB - 1) / kTB;
    // chunks of 8 (N = 4096) move as two 16-byte LDS accesses per thread
    const bool vec8 = chunk == 8 && (N & 7) == 0;
    int b0[VPT], b1[VPT];
    float cv[VPT][8];
    double part[VPT], incl[VPT];
#pragma unroll
    for (int h = 0; h < VPT; ++h) {
      b0[h] = min(vthread<NT>(h) * chunk, N);
      b1[h] = min(b0[h] + chunk, N);
      part[h] = 0.0;
      if (vec8) {
        if (b0[h] < b1[h]) {
          const float4 v0 = *reinterpret_cast<const float4*>(buf + b0[h]);
          const float4 v1 = *reinterpret_cast<const float4*>(buf + b0[h] + 4);
          cv[h][0] = v0.x; cv[h][1] = v0.y; cv[h][2] = v0.z; cv[h][3] = v0.w;
          cv[h][4] = v1.x; cv[h][5] = v1.y; cv[h][6] = v1.z; cv[h][7] = v1.w;
#pragma unroll
          for (int i = 0; i < 8; ++i) part[h] += (double)cv[h][i];
        }
      } else {
        for (int i = b0[h]; i < b1[h]; ++i) part[h] += (double)buf[i];
      }
      incl[h] = part[h];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double y = __shfl_up(incl[h], o, kWave);
        if (lane >= o) incl[h] += y;
      }
    }
    const int k = parity;
    parity ^= 1;
#pragma unroll
    for (int h = 0; h < VPT; ++h)
      if (lane == 63) red.d[k][vwave<NT>(h)][0] = incl[h];
    __syncthreads();
    SMC_TRACE(trow, 5);
    // systematic resampling handed to the next sweep (bins_ancestor): the
    // bins go straight to bins_out (coalesced: thread chunks are adjacent),
    // not through LDS
    const bool to_bins = a.bins_out && a.method == SMCDET_RESAMPLE_SYSTEMATIC;
    float* dst = to_bins ? a.bins_out + (size_t)t * N : buf;
    const bool dst_al16 = ((uintptr_t)dst & 15) == 0;  // (a C caller's bins_out may not be)
    // the first search level's chunk ends (bins_ancestor): element gi of a
    // thread's chunk is entry l's end when gi == bins_coarse_end(l)
    float* coarse = to_bins ? a.bins_out + (size_t)a.T * (N + 1) + (size_t)t * kBinsCoarse
                            : nullptr;
    const int cstep = (N + kBinsCoarse - 1) / kBinsCoarse;
#pragma unroll
    for (int h = 0; h < VPT; ++h) {
      double base = 0.0;
      for (int i = 0; i < vwave<NT>(h); ++i) base += red.d[k][i][0];
      double run = base + incl[h] - part[h];
      if (vec8) {
        if (b0[h] < b1[h]) {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            run += (double)cv[h][i];
            cv[h][i] = (float)run;
          }
          if (coarse) {
            int l = b0[h] / cstep, end = bins_coarse_end(l, N);
#pragma unroll
            for (int i = 0; i < 8; ++i)
              if (b0[h] + i == end) {
                coarse[l] = cv[h][i];
                end = bins_coarse_end(++l, N);
              }
          }
          if (dst_al16) {
            *reinterpret_cast<float4*>(dst + b0[h]) =
                make_float4(cv[h][0], cv[h][1], cv[h][2], cv[h][3]);
            *reinterpret_cast<float4*>(dst + b0[h] + 4) =
                make_float4(cv[h][4], cv[h][5], cv[h][6], cv[h][7]);
          } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) dst[b0[h] + i] = cv[h][i];
          }
        }
      } else {
        int l = b0[h] / cstep, end = bins_coarse_end(l, N);
        for (int i = b0[h]; i < b1[h]; ++i) {
          run += (double)buf[i];
          dst[i] = (float)run;
          if (coarse && i == end) {
            coarse[l] = (float)run;
            end = bins_coarse_end(++l, N);
          }
        }
      }
    }
    if (!to_bins) __syncthreads();
    float U = 0.f;
    if (a.method == SMCDET_RESAMPLE_SYSTEMATIC) {
      if (a.u) {
        U = a.u[t];
      } else {
        const U4 r = philox4x32((uint32_t)a.offset, (uint32_t)(a.offset >> 32), (uint32_t)t,
                                kTagResample, a.k0, a.k1);
        U = u01(r.x);
      }
    }
    if (to_bins) {
      // the next sweep's waves search their own ancestors (bins_ancestor):
      // the bins (written above) and U instead of the indices
      if (threadIdx.x == 0) a.bins_out[(size_t)a.T * N + t] = U;
      SMC_TRACE(trow, 6);
      return;
    }
    const float total = buf[N - 1];
    int64_t* idxg = a.idx + (size_t)t * N;
    if (a.method == SMCDET_RESAMPLE_SYSTEMATIC) {
      // bucketize(u, bins), u_n = (n + U) / N in float32 (sampler.py:144),
      // right=False: idx[n] = #{i : bins[i] < u_n}, clamped to N - 1.  bins
      // is monotone (float32 roundings of a running sum of non-negative
      // weights), so the count is a binary search: binary lifting with
      // power-of-two steps, log2(N) LDS reads per n whatever the weights'
      // degeneracy, G searches per thread interleaved.  The test
      // bins[i] < u_n is exact: u_n is formed with the reference's float
      // ops, and for N a power of two the division is an exact scaling, so
      // b < u_n  <=>  b*N < fl(n + U) (exact) without the division.
      const float Nf = (float)N;
      const bool pow2 = (N & (N - 1)) == 0;
      int top = 1;
      while (2 * top <= N) top *= 2;
      constexpr int G = 8;
      for (int base = threadIdx.x; base < N; base += NT * G) {
        float key[G];
        int lo[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const float nu = (float)(base + g * NT) + U;
          key[g] = pow2 ? nu : nu / Nf;
          lo[g] = 0;
        }
        for (int step = top; step > 0; step >>= 1) {
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const int i = lo[g] + step - 1;
            const float b = buf[min(i, N - 1)];
            const bool less = pow2 ? (b * Nf < key[g]) : (b < key[g]);
            lo[g] += (i < N && less) ? step : 0;
          }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int n = base + g * NT;
          if (n < N) idxg[n] = (int64_t)min(lo[g], N - 1);
        }
      }
      SMC_TRACE(trow, 6);
    } else {
      // multinomial (sampler.py:127-140): target = u * total, first bin > target
      for (int n = threadIdx.x; n < N; n += NT) {
        float un;
        if (a.u) {
          un = a.u[(size_t)t * N + n];
        } else {
          const uint64_t c = a.offset + (uint64_t)n;
          const U4 r = philox4x32((uint32_t)c, (uint32_t)(c >> 32), (uint32_t)t,
                                  kTagResample + 1, a.k0, a.k1);
          un = u01(r.x);
        }
        const float target = un * total;
        int lo = 0, hi = N;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (buf[mid] > target) hi = mid; else lo = mid + 1;
        }
        idxg[n] = (int64_t)min(lo, N - 1);
      }
    }
  }
}

// LDS words tile_work needs in `buf`
__host__ __device__ inline size_t tile_lds_bytes(int N) { return (size_t)(2 * N + 1) * sizeof(float); }

}  // namespace smcdet
