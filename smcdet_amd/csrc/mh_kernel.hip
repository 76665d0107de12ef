// mh_kernel.hip — the fused single-component Metropolis-Hastings sweep
// (restates smcdet/kernel.py:26-130, SingleComponentMH.run, with the
// log_target of smcdet/sampler.py:87-91 evaluated in-kernel).
//
// One particle per 64-lane wavefront, 4 particles (of one tile) per 256-thread
// workgroup sharing the tile image staged in LDS.  All K iterations run in one
// launch; the particle's state lives in registers (lane s holds source s) and
// its rate image lambda[H*W] lives in the wave's LDS slice.
//
// Per iteration (wave-uniform control):
//   * draws: Philox4x32-10, 64 iterations at a time (lane i generates the 5
//     uniforms of iteration k0+i, then they are broadcast by v_readlane), or
//     replayed from recorded reference draws;
//   * proposal: lanes 0,1,2 sample the truncated normals of (h, w, flux) of the
//     chosen source in parallel (distributions.py:40-48) and evaluate the
//     truncated-proposal Hastings terms; the Normal log-density terms cancel
//     exactly between numerator and denominator, so only the log-mass-in-box
//     terms remain (log Z(current) - log Z(proposed)), which are cached per
//     source and dimension;
//   * likelihood: only the moved source changes, so the delta log-likelihood
//     is evaluated over the union of its old and new PSF windows (clipped to
//     the tile, <= 18x18 positions for a step < 1 px): the rate changes by
//     dl = g f' psf_new - g f psf_old there, and the per-pixel log-likelihood
//     change is evaluated in a cancellation-free form (pix_delta, device.h)
//     whose error scales with the change, not with the absolute terms.  (Mode SMCDET_MH_FULL_RECOMPUTE instead
//     re-renders every source each step, as the reference does.)
//   * accept iff U <= min(1, exp(log alpha)) (kernel.py:114-116), evaluated
//     as log alpha >= log U with log U precomputed per proposal batch.
// The rate image comes from the ancestor's persisted image (rate_in) or a
// fresh render; the returned loglik_out is summed over the final rate image
// (fresh full render in FULL_RECOMPUTE mode).  The union-window positions run
// two per lane in packed f32 arithmetic (position_delta2), and everything
// wave-uniform about an iteration (anchors, amplitudes, prior and Hastings
// terms) is computed once per proposal batch in the batch's lanes.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <type_traits>
#include <vector>

#include "render.h"
#include "tile.h"

namespace smcdet {

SMCDET_WAVE_TABLE

// The diagnostic build (make diag -> libsmcdet_hip_diag.so, -DSMCDET_DIAG)
// adds the A/B and timing-only variants: the radial PSF table
// (SMCDET_MH_PSF_TABLE), scalar union-window slots (SMCDET_MH_SCALAR_SLOTS),
// the ablations (SMCDET_MH_ABLATE_*), the sweep without the 1/v cache
// (SMCDET_MH_NO_RCP_CACHE) and the SMCDET_MH_BLOCK_SLOTS override.  The product
// library compiles only the instantiations its API paths dispatch and refuses
// those flags (instantiation table).
#ifdef SMCDET_DIAG
constexpr bool kDiag = true;
#else
constexpr bool kDiag = false;
#endif

constexpr int kMhWaves = 4;
constexpr int kMhBlock = kMhWaves * kWave;
constexpr int kSlots = 6;  // register-resident window passes (6*64 = 384 positions)
// proposals computed together (3 lanes each): 21 entries = 63 lanes.  A batch
// is recomputed at its end and when an accepted move dirties a later entry's
// source, so longer batches mean fewer recomputes (a simulation of the rule:
// 0.145 -> 0.084 per iteration at acceptance 0.1, 0.183 -> 0.157 at 0.37) at
// the same cost per recompute (SIMD lanes); results do not depend on it.
// Same box (scripts/r05_batch_pass.sh): C4 MH launch 4.36 -> 4.26 ms, C2
// microbench -1..-4% against 8 entries
constexpr int kBatch = 21;

struct MhArgs {
  DevModel m;
  DevPrior pr;
  int K, T, N, S;
  float sl, isl, sf, isf;            // proposal sd and 1/sd (loc, flux)
  float lb_h, lb_w, ub_h, ub_w;      // loc box
  float lb_f, ub_f;                  // flux box
  uint32_t k0, k1;                   // Philox key (seed)
  uint64_t offset;                   // Philox counter base (iterations)
  uint32_t ablate;                   // SMCDET_MH_ABLATE_* (diagnostics)
  int by_count;                      // SMCDET_MH_COMPONENT_BY_COUNT
  int scalar_slots;                  // SMCDET_MH_SCALAR_SLOTS (diagnostic)
  int skip_done;                     // SMCDET_MH_SKIP_DONE
  int no_psf_cache;                  // SMCDET_MH_NO_PSF_CACHE (diagnostic)
  int no_rcp_cache;                  // SMCDET_MH_NO_RCP_CACHE (diagnostic)
  int blk_slots;                     // block form (M71, same anchor) from this many slots; 0: off
  const float4* psf_tab;             // M71 radial PSF table [kTabNodes] (or null: exp2/log2)
  float tab_inv_h;                   // 1 / its node spacing in r^2
  const float* img;                  // [T,H,W]
  const float* temperature;          // [T]
  const int64_t* ancestors;          // [T,N] or null
  const float* anc_bins;             // [T*N + T] systematic bins + offsets (bins_ancestor) or null
  const float* counts_in;
  const float* locs_in;
  const float* fluxes_in;
  float* counts_out;
  float* locs_out;
  float* fluxes_out;
  float* loglik_out;                 // [T,N] or null
  const float* rate_in;              // [T,N,H*W] persisted rate images or null
  float* rate_out;                   // [T,N,H*W] or null
  const int32_t* go;                 // predicate: skip the launch when *go == 0 (or null)
  const float* boxes;                // [T,4] per-tile location boxes (or null: lb_*/ub_*)
  int32_t* acc_count;                // [2T] zeroed workspace: [T] uint64 (count << 32 | ticket)
  float* acc_rate;                   // [T]
  const int32_t* r_comp;             // replay (or null)
  const float* r_uloc;
  const float* r_uflux;
  const float* r_uacc;
  float* r_loga;                     // replay decision trace [K,T,N] (or null)
  uint8_t* r_accept;
  // fused SMC iteration: the tile's last workgroup runs temper -> reweight ->
  // next resampling indices (tile.h) on loglik_out right after the sweep
  int has_tail;
  TileArgs tail;
};

// The fused tail: tile_work by the 256 threads of the tile's last workgroup
// on the 512-thread virtual layout, so the results equal
// smcdet_temper_reweight's bit for bit.  One instantiation (8 log-likelihoods
// per virtual thread, N <= 4096, host-checked): smaller N only masks slots,
// and a masked slot adds an exact 0 to every sum.  Inlined -- as a call, the
// callee-saved register convention pushed the sweep to 128 VGPRs and
// scratch.
constexpr int kTailMaxN = 8 * kTB;

// truncated-normal cache at mean mu: Phi(lb) and log Z, Z = Phi(ub) - Phi(lb)
// (distributions.py:33-35)
__device__ __forceinline__ void tn_cache(float mu, float isig, float lb, float ub, float& phl,
                                         float& lZ) {
  phl = normal_cdf(lb, mu, isig);
  lZ = nan_to_num(fast_log(normal_cdf(ub, mu, isig) - phl), 0.0f);
}

// the summed Hastings + prior term of an edge hit (-inf), tested on the
// wave-uniform bits (a scalar compare, not a VALU float compare)
__device__ __forceinline__ bool edge_hit(float hast) { return __float_as_uint(hast) == 0xff800000u; }

// A proposal for one MH iteration: the chosen source j moves (h, w, f) ->
// (hn, wn, fn).  Wave-uniform (SGPR) values.
struct Proposal {
  int j;
  float h, w;         // current location of source j
  float hn, wn, fn;   // proposed location and flux
  float hast;         // log q(z|z') - log q(z'|z)
};

struct Dim {  // per-lane constants of the dimension this lane proposes
  float sig, isig, lb, ub;
};

// One dimension of one truncated-normal proposal (distributions.py:40-48),
// evaluated by one lane: mu = current value, (c_ph, c_lZ) its cached Phi(lb)
// and log-mass-in-box; returns the proposed value, the caches at it, the
// dimension's Hastings term and log(value).  The Normal log-densities of
// q(z|z') and q(z'|z) cancel (kernel.py:71-111); the log-mass terms remain.
template <bool ABLATE>
__device__ __forceinline__ void propose_lane(float mu, float c_ph, float c_lZ, float u,
                                             const Dim& dm, float& xn, float& n_ph, float& n_lZ,
                                             float& hast_d, float& n_lf) {
  if (ABLATE) {  // timing-only stand-in: a small deterministic move
    xn = fminf(fmaxf(mu + (u - 0.5f) * dm.sig, dm.lb), dm.ub);
    n_ph = c_ph;
    n_lZ = c_lZ;
    hast_d = 0.f;
    n_lf = xn;
  } else {
    const float pc = fminf(fmaxf(u, 1e-6f), 0.999999f);
    float pt = c_ph + pc * fast_exp(c_lZ);
    pt = fminf(fmaxf(pt, 1e-6f), 0.999999f);
    xn = mu + dm.sig * erfinv_fast(2.0f * pt - 1.0f) * kSqrt2;
    xn = fminf(fmaxf(xn, dm.lb), dm.ub);
    tn_cache(xn, dm.isig, dm.lb, dm.ub, n_ph, n_lZ);
    hast_d = c_lZ - n_lZ;
    n_lf = fast_log(xn);
  }
}

// One position of the union window: rate change dl and log-likelihood change.
// WINDOWS = false when old and new windows coincide (same floor anchors): every
// position of the (clipped) box is in both.
// GL: the tile image lives in global memory (tiles above the LDS budget): a
// masked lane's dummy position HW + lane reads the last pixel instead
// TB: the PSF values from the radial table in LDS (psf_tab, device.h)
template <int MODEL, bool WINDOWS, bool GL = false, bool RV = false, bool TB = false>
__device__ __forceinline__ float position_delta(const DevModel& m, const float* xs,
                                                const float* lg, const float* lam,
                                                const float* rv, const float4* tab, float tinv,
                                                int p, int aa, int bb, int ph, int pw,
                                                const Proposal& P, float amp_o, float amp_n,
                                                int ao_h, int ao_w, int an_h, int an_w,
                                                float& lnew, float& rnew) {
  const float fph = (float)ph + 0.5f, fpw = (float)pw + 0.5f;
  const float dho = fph - P.h, dwo = fpw - P.w;
  const float dhn = fph - P.hn, dwn = fpw - P.wn;
  float psi_o, psi_n;
  if constexpr (TB) {
    psi_o = psf_tab(tab, tinv, fmaf(dho, dho, dwo * dwo));
    psi_n = psf_tab(tab, tinv, fmaf(dhn, dhn, dwn * dwn));
  } else {
    psi_o = psf_raw<MODEL>(m, fmaf(dho, dho, dwo * dwo));
    psi_n = psf_raw<MODEL>(m, fmaf(dhn, dhn, dwn * dwn));
  }
  if (WINDOWS) {
    const unsigned span = 2u * (unsigned)m.R;
    psi_o = ((unsigned)(aa - ao_h) <= span && (unsigned)(bb - ao_w) <= span) ? psi_o : 0.f;
    psi_n = ((unsigned)(aa - an_h) <= span && (unsigned)(bb - an_w) <= span) ? psi_n : 0.f;
  }
  const float dl = fmaf(amp_n, psi_n, -amp_o * psi_o);
  const float lo = lam[p];
  lnew = lo + dl;
  const float lgx = (MODEL == SMCDET_MODEL_POISSON) ? lg[p] : 0.0f;
  const float x = GL ? xs[min(p, m.H * m.W - 1)] : xs[p];
  if constexpr (RV) {
    // M71 with the 1/v cache: pix_delta's operations, r0 read, v0 not formed
    const float r0 = rv[p];
    const float v1 = fmaf(m.eta, lnew, m.s0sq);
    const float r1 = fast_rcp(v1);
    rnew = r1;
    const float d0 = x - lo, d1 = x - lnew;
    const float t = fmaf(d0 * d0, r0, -(d1 * d1) * r1);
    return fmaf(0.5f, t, (-0.5f * kLn2) * fast_log2(v1 * r0));
  }
  return pix_delta<MODEL>(m, x, lgx, lo, dl);
}

// Two positions per lane at once (union-window slots 2i and 2i+1): the float
// arithmetic runs as packed v_pk_{fma,mul,add}_f32 (one issue for both
// halves), the transcendentals per half.  Same per-element operation order as
// position_delta.
template <int MODEL, bool WINDOWS, bool GL = false, bool RV = false, bool TB = false>
__device__ __forceinline__ f2 position_delta2(const DevModel& m, const float* xs, const float* lg,
                                             const float* lam, const float* rv,
                                             const float4* tab, float tinv, const int (&p)[2],
                                             const int (&aa)[2], const int (&bb)[2], f2 fph,
                                             f2 fpw, const Proposal& P, float amp_o, float amp_n,
                                             int ao_h, int ao_w, int an_h, int an_w, f2& lnew,
                                             f2& rnew) {
  const f2 dho = fph - P.h, dwo = fpw - P.w;
  const f2 dhn = fph - P.hn, dwn = fpw - P.wn;
  f2 psi_o, psi_n;
  if constexpr (TB) {
    psi_o = psf_tab2(tab, tinv, fma2(dho, dho, dwo * dwo));
    psi_n = psf_tab2(tab, tinv, fma2(dhn, dhn, dwn * dwn));
  } else {
    psi_o = psf_raw2<MODEL>(m, fma2(dho, dho, dwo * dwo));
    psi_n = psf_raw2<MODEL>(m, fma2(dhn, dhn, dwn * dwn));
  }
  if (WINDOWS) {
    const unsigned span = 2u * (unsigned)m.R;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      psi_o[h] = ((unsigned)(aa[h] - ao_h) <= span && (unsigned)(bb[h] - ao_w) <= span) ? psi_o[h]
                                                                                       : 0.f;
      psi_n[h] = ((unsigned)(aa[h] - an_h) <= span && (unsigned)(bb[h] - an_w) <= span) ? psi_n[h]
                                                                                       : 0.f;
    }
  }
  const f2 dl = fma2(psi_n, amp_n, -amp_o * psi_o);
  const f2 lo = {lam[p[0]], lam[p[1]]};
  f2 x;
  if constexpr (GL) {
    const int hw1 = m.H * m.W - 1;
    x = f2{xs[min(p[0], hw1)], xs[min(p[1], hw1)]};
  } else {
    x = f2{xs[p[0]], xs[p[1]]};
  }
  lnew = lo + dl;
  if constexpr (RV) {
    // M71 with the 1/v cache: pix_delta2's operations, r0 read, v0 not formed
    const f2 r0 = {rv[p[0]], rv[p[1]]};
    const f2 v1 = fma2(lnew, m.eta, m.s0sq);
    const f2 r1 = rcp2(v1);
    rnew = r1;
    const f2 d0 = x - lo, d1 = x - lnew;
    const f2 t = fma2(d0 * d0, r0, -(d1 * d1) * r1);
    return fma2(t, 0.5f, (-0.5f * kLn2) * log2_2(v1 * r0));
  }
  f2 lgx = {0.f, 0.f};
  if constexpr (MODEL == SMCDET_MODEL_POISSON) lgx = f2{lg[p[0]], lg[p[1]]};
  return pix_delta2<MODEL>(m, x, lgx, lo, dl);
}

// ---- the 16x16 block form of a same-anchor M71 step (mh_sweep_kernel `block`)
// The moved source's old and new PSF windows share their anchor, so the
// union is one (clipped) box of at most 17x17 pixels.  Its first 16 rows and
// columns are evaluated as a 16x16 block of the tile in the layout of
// v_mfma_f32_16x16x4_f32's result (lane l holds rows 4(l>>4) + r, r < 4, of
// column l & 15), the 17th row / column (<= 33 pixels) as one union-window
// slot.  In the block, the profile's two Gaussian terms are separable,
//   g exp2(k r^2) = g exp2(k dy^2) exp2(k dx^2),
// so the rate change's Gaussian part,
//   sum_k A[i][k] B[k][j],  k = (new, k1), (new, k2), (old, k1), (old, k2),
//   A = +-amp (x b) exp2(k dy_i^2),  B = exp2(k dx_j^2),
// is ONE rank-4 MFMA (exact f32 fused multiply-adds), built from 2 exp2 per
// lane instead of 4 per pixel; the pixels keep only the power-law term
// (exp2 of log2, old and new) and the likelihood change.  Same quantity as
// position_delta's, rounded differently (a few ulp of the profile).
typedef float f4 __attribute__((ext_vector_type(4)));

// the per-pixel log-likelihood change of position_delta2 from the rate change
// dl (M71; RV: the old pixel's 1/v read from the cache, the new one returned)
template <int MODEL, bool RV>
__device__ __forceinline__ f2 delta_from_dl2(const DevModel& m, f2 x, f2 lo, f2 dl,
                                             const float* rv, const int (&p)[2], f2& lnew,
                                             f2& rnew) {
  lnew = lo + dl;
  if constexpr (RV) {
    const f2 r0 = {rv[p[0]], rv[p[1]]};
    const f2 v1 = fma2(lnew, m.eta, m.s0sq);
    const f2 r1 = rcp2(v1);
    rnew = r1;
    const f2 d0 = x - lo, d1 = x - lnew;
    const f2 t = fma2(d0 * d0, r0, -(d1 * d1) * r1);
    return fma2(t, 0.5f, (-0.5f * kLn2) * log2_2(v1 * r0));
  }
  return pix_delta2<MODEL>(m, x, f2{0.f, 0.f}, lo, dl);
}

// Small tiles with the PSF cache (PC): the moved source's old PSF values come
// from the wave's cache row of that source (its raw PSF at every tile pixel,
// 0 outside its window) instead of being re-evaluated; the new window's
// values are returned for the cache update on accept.  Both are the values
// position_delta computes, by the same operations on the same inputs (the
// cached row was evaluated at the source's current position), so decisions
// and rates are bit-identical to the uncached sweep.
template <int MODEL, bool WINDOWS, bool TB = false>
__device__ __forceinline__ float position_delta_pc(const DevModel& m, const float* xs,
                                                   const float* lg, const float* lam,
                                                   const float* pcj, const float4* tab,
                                                   float tinv, int p, bool valid, int aa,
                                                   int bb, int ph, int pw, const Proposal& P,
                                                   float amp_o, float amp_n, int an_h, int an_w,
                                                   float& lnew, float& psi_new) {
  const float fph = (float)ph + 0.5f, fpw = (float)pw + 0.5f;
  const float dhn = fph - P.hn, dwn = fpw - P.wn;
  const float psi_o = pcj[valid ? p : 0];  // (a masked lane's value is discarded)
  float psi_n;
  if constexpr (TB) psi_n = psf_tab(tab, tinv, fmaf(dhn, dhn, dwn * dwn));
  else psi_n = psf_raw<MODEL>(m, fmaf(dhn, dhn, dwn * dwn));
  if (WINDOWS) {
    const unsigned span = 2u * (unsigned)m.R;
    psi_n = ((unsigned)(aa - an_h) <= span && (unsigned)(bb - an_w) <= span) ? psi_n : 0.f;
  }
  psi_new = psi_n;
  const float dl = fmaf(amp_n, psi_n, -amp_o * psi_o);
  const float lo = lam[p];
  lnew = lo + dl;
  const float lgx = (MODEL == SMCDET_MODEL_POISSON) ? lg[p] : 0.0f;
  return pix_delta<MODEL>(m, xs[p], lgx, lo, dl);
}

// Persisted rate image in / out for tiles of <= 64*PPL pixels: each lane's
// (at most ceil(PPL/4)) float4 pieces all issued before any is used.
template <int PPL>
__device__ __forceinline__ void copy_in_regs(const float* __restrict__ rin, float* lam, int HW,
                                             int lane) {
  constexpr int NV = (PPL + 3) / 4;
  if ((HW & 3) == 0) {
    float4 v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int p = 4 * (k * kWave + lane);
      if (p < HW) v[k] = *reinterpret_cast<const float4*>(rin + p);
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int p = 4 * (k * kWave + lane);
      if (p < HW) {
        lam[p] = v[k].x;
        lam[p + 1] = v[k].y;
        lam[p + 2] = v[k].z;
        lam[p + 3] = v[k].w;
      }
    }
  } else {
    float v[PPL];
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
      const int p = k * kWave + lane;
      if (p < HW) v[k] = rin[p];
    }
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
      const int p = k * kWave + lane;
      if (p < HW) lam[p] = v[k];
    }
  }
  wave_sync();
}
template <int PPL>
__device__ __forceinline__ void copy_out_regs(const float* lam, float* __restrict__ rout, int HW,
                                              int lane) {
  constexpr int NV = (PPL + 3) / 4;
  if ((HW & 3) == 0) {
    float4 v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int p = 4 * (k * kWave + lane);
      if (p < HW) v[k] = make_float4(lam[p], lam[p + 1], lam[p + 2], lam[p + 3]);
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int p = 4 * (k * kWave + lane);
      if (p < HW) *reinterpret_cast<float4*>(rout + p) = v[k];
    }
  } else {
    for (int p = lane; p < HW; p += kWave) rout[p] = lam[p];
  }
}

// PPL > 0: tiles of <= 64*PPL pixels rendered in registers (render_regs);
// PPL = 0: LDS render (larger tiles)
// PAIRED: union-window positions two per lane in packed arithmetic (default);
// false: one per lane (SMCDET_MH_SCALAR_SLOTS, for A/B timing).
// Small tiles (PPL == 1: H*W <= 64, e.g. the 8x8 M71 cutouts) never need more
// than one union-window slot (npos <= H*W): only that path is compiled, which
// fits the kernel in 72 VGPRs (3 spilled) and so runs 7 waves per SIMD instead
// of 4 -- the per-iteration control of these short iterations is
// latency-bound.  Same-box A/B (C4, MH launch): 4 waves + all slot paths
// 5.93 ms; 1-slot path at 4 waves 5.33; 6 waves (80 VGPRs, no spill) 5.17;
// 7 waves 5.11; 8 waves (64 VGPRs, 15 spilled) 5.62.
#ifndef SMCDET_SMALL_TILE_WAVES
#define SMCDET_SMALL_TILE_WAVES 7
#endif
// (the replay instantiation of small tiles, tests only, holds the replayed
// draws too: 6 waves per SIMD, 80 VGPRs, instead of spilling at 72; FULL
// mode's register re-render of 65..1024-pixel tiles -- the reference's
// arithmetic, a parity control, bit-identical to the loglik kernel's render --
// runs at 2 waves per SIMD instead of spilling at 128 VGPRs)
template <int PPL, bool REPLAY = false, bool FULL = false>
constexpr int mh_waves_per_eu() {
  return PPL == 1 ? (REPLAY ? SMCDET_SMALL_TILE_WAVES - 1 : SMCDET_SMALL_TILE_WAVES)
                  : (FULL && PPL == 16 ? 2 : 4);
}
template <int PPL>
constexpr int mh_slots() { return PPL == 1 ? 1 : kSlots; }

// TAIL: the fused SMC step's instantiation (a.has_tail); the sweep alone
// compiles without the tail pass, which would otherwise raise its SGPR
// pressure (spills reloaded by v_readlane in the loop).
// GL: tiles above the LDS budget (M71, PPL = 0): the tile image is read from
// global memory (L2-resident) and the particle's rate image lives in rate_out
// (row stride H*W + 64: the 64 dummy cells of masked lanes), which the sweep
// updates in place; LDS holds only the workgroup counters.
// PC: small tiles (PPL == 1, incremental) with the per-wave PSF cache in LDS
// (S rows of H*W floats after the rate images; position_delta_pc).
// RV: M71 tiles rendered in registers (PPL > 1, incremental, no fused tail):
// a per-wave image of 1/v = 1/(s0^2 + eta*lambda) in LDS after the rate
// images, so pix_delta reads the old pixel's reciprocal instead of forming it
// (kept current on accept with the same operations: bit-identical).
// TB: M71 incremental sweeps with the radial PSF table (psf_tab, device.h)
// staged into LDS after the images / caches: every union-window PSF value
// (and the PSF cache's rows) comes from the table.
template <int MODEL, bool REPLAY, bool FULL, int PPL, bool PAIRED, bool TAIL, bool GL = false,
          bool PC = false, bool RV = false, bool TB = false>
__global__ __launch_bounds__(kMhBlock, (mh_waves_per_eu<PPL, REPLAY, FULL>())) void mh_sweep_kernel(
    MhArgs a) {
  static_assert(!PC || (PPL == 1 && !FULL && !GL && !TAIL), "PSF cache: small incremental tiles");
  static_assert(!RV || (MODEL == SMCDET_MODEL_M71 && PPL > 1 && !FULL && !GL && !TAIL && PAIRED),
                "1/v cache: M71 register-render tiles, incremental, paired");
  static_assert(!TB || (MODEL == SMCDET_MODEL_M71 && PPL > 0 && !FULL && !GL && !TAIL && PAIRED),
                "PSF table: M71 register-render tiles, incremental, paired");
  constexpr int NSL = mh_slots<PPL>();
  // 16-byte aligned: the PSF table (TB) is read as float4 at smem + offset
  extern __shared__ __align__(16) float smem[];
  __shared__ int wg_acc, wg_done;  // last-iteration accepts / finished waves of this workgroup
  __shared__ int wg_last;          // this workgroup finished its tile last (fused tail)
  if (a.go && *a.go == 0) return;  // speculatively enqueued sweep that must not run
  const DevModel& m = a.m;
  [[maybe_unused]] const int trow = (int)(blockIdx.x * kMhWaves + (threadIdx.x >> 6));
  SMC_TRACE(trow, 0);
  SMC_WAVE_MARK(trow, 0);
  const int HW = m.H * m.W;
  const int HWp = HW + kWave;  // + one dummy cell per lane (HW + lane) for masked lanes
  const int t = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int kImg = (MODEL == SMCDET_MODEL_POISSON) ? 2 : 1;
  float* xs = smem;
  float* lg = smem + HWp;
  float* lam = smem + kImg * HWp + wave * HWp;
  if constexpr (GL) {
    xs = const_cast<float*>(a.img) + (size_t)t * HW;
    lg = nullptr;
  } else {
    stage_image<MODEL>(a.img + (size_t)t * HW, xs, lg, HW, threadIdx.x, kMhBlock);
  }
  if (threadIdx.x == 0) {
    wg_acc = 0;
    wg_done = 0;
    wg_last = 0;
  }
  if (!GL && threadIdx.x < kWave) {
    xs[HW + threadIdx.x] = m.bg;
    if (MODEL == SMCDET_MODEL_POISSON) lg[HW + threadIdx.x] = 0.f;
  }
  // the radial PSF table, 16-B aligned after the images and caches
  [[maybe_unused]] const float4* tab = nullptr;
  [[maybe_unused]] const float tinv = a.tab_inv_h;
  if constexpr (TB) {
    const int off = ((kImg + kMhWaves) * HWp + (RV ? kMhWaves * HWp : 0) +
                     (PC ? kMhWaves * a.S * HW : 0) + 3) & ~3;
    float4* t4 = reinterpret_cast<float4*>(smem + off);
    for (int i = threadIdx.x; i < kTabNodes; i += kMhBlock) t4[i] = a.psf_tab[i];
    tab = t4;
  }
  __syncthreads();
  SMC_TRACE(trow, 1);
  const int n = blockIdx.x * kMhWaves + wave;
  if (n >= a.N) return;  // (never with the fused tail: N % 4 == 0, host-checked)

  const int N = a.N, S = a.S;
  const size_t pid = (size_t)t * N + n;
  size_t src = a.ancestors ? (size_t)t * N + (size_t)a.ancestors[pid] : pid;
  if (a.anc_bins)  // the wave finds its ancestor in the previous tile pass's bins
    src = (size_t)t * N +
          (size_t)bins_ancestor(a.anc_bins + (size_t)t * N,
                                a.anc_bins + (size_t)a.T * (N + 1) + (size_t)t * kBinsCoarse, N,
                                a.anc_bins[(size_t)a.T * N + t], n);
  if constexpr (GL) lam = a.rate_out + pid * (size_t)HWp;
  const float count = a.counts_in[src];
  if (a.counts_out && lane == 0) a.counts_out[pid] = count;
  // range of the moved component: 0..S-1 (kernel.py:35-37), or 0..count-1
  // for count-stratified populations padded to S sources (count 0: no moves)
  const int Sj = a.by_count ? min(max((int)count, 0), S) : S;
  const float tau = a.temperature[t];
  // independent stopping: a tile already at temperature 1 keeps its
  // (resampled) particles unchanged (SMCDET_MH_SKIP_DONE)
  const int K = (Sj > 0 && !(a.skip_done && tau >= 1.0f)) ? a.K : 0;

  // ---- particle state: lane s holds source s --------------------------------
  float sh = 0.f, sw = 0.f, sfx = 0.f;
  if (lane < S) {
    sh = a.locs_in[(src * S + lane) * 2 + 0];
    sw = a.locs_in[(src * S + lane) * 2 + 1];
    sfx = a.fluxes_in[src * S + lane];
  }
  SMC_TRACE(trow, 2);

  double cur_ll = 0.0;  // tracked only in FULL mode (incremental mode works on deltas)
  if constexpr (GL && !FULL) {
    // the working image is rate_out's row: copy the ancestor's row in, or render
    if (a.rate_in && !(a.rate_in == a.rate_out && src == pid)) {
      const float* rin = a.rate_in + src * (size_t)HWp;
      for (int p = lane; p < HW; p += kWave) lam[p] = rin[p];
      wave_sync();
    } else if (!a.rate_in) {
      render_chunks<MODEL>(m, lam, sh, sw, sfx, S, lane);
    }
  } else if constexpr (GL) {
    render_sources<MODEL>(m, lam, sh, sw, sfx, S, lane);
    cur_ll = pixel_sum<MODEL>(m, xs, lg, lam, nullptr, lane);
  } else if constexpr (!FULL) {
    if (a.rate_in) {
      // the ancestor's rate image, persisted by the previous sweep: no render
      const float* rin = a.rate_in + src * (size_t)HW;
      if constexpr (PPL > 0) {
        // HW <= 64*PPL (register-render tiles): every lane's float4 loads in
        // flight before the LDS stores (the generic loop below kept at most
        // two in flight: one HBM round trip per pair on the sweep's start)
        copy_in_regs<PPL>(rin, lam, HW, lane);
      } else if ((HW & 3) == 0) {
        for (int p = 4 * lane; p < HW; p += 4 * kWave) {
          const float4 v = *reinterpret_cast<const float4*>(rin + p);
          lam[p] = v.x;
          lam[p + 1] = v.y;
          lam[p + 2] = v.z;
          lam[p + 3] = v.w;
        }
      } else {
        for (int p = lane; p < HW; p += kWave) lam[p] = rin[p];
      }
      wave_sync();
    } else if constexpr (PPL > 0) {
      float lamk[PPL > 0 ? PPL : 1];
      render_regs<MODEL, PPL>(m, lamk, sh, sw, sfx, S, lane);
      store_regs<MODEL, PPL>(m, lam, lamk, lane);
    } else {
      render_sources<MODEL>(m, lam, sh, sw, sfx, S, lane);
    }
  } else if constexpr (PPL > 0) {
    float lamk[PPL > 0 ? PPL : 1];
    render_regs<MODEL, PPL>(m, lamk, sh, sw, sfx, S, lane);
    cur_ll = pixel_sum_regs<MODEL, PPL>(m, xs, lg, lamk, lane);
  } else {
    render_sources<MODEL>(m, lam, sh, sw, sfx, S, lane);
    cur_ll = pixel_sum<MODEL>(m, xs, lg, lam, nullptr, lane);
  }
  lam[HW + lane] = m.bg;
  [[maybe_unused]] float* rv = nullptr;
  if constexpr (RV) {
    rv = lam + kMhWaves * HWp;
    wave_sync();
    if constexpr (PPL > 0) {
      // (PPL + 1) cells per lane: the LDS reads first, then the reciprocals
      constexpr int NR = PPL + 1;
      float v[NR];
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        const int p = k * kWave + lane;
        v[k] = p < HWp ? lam[p] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        const int p = k * kWave + lane;
        if (p < HWp) rv[p] = fast_rcp(fmaf(m.eta, v[k], m.s0sq));
      }
    } else {
      for (int p = lane; p < HWp; p += kWave) rv[p] = fast_rcp(fmaf(m.eta, lam[p], m.s0sq));
    }
    wave_sync();
  }
  // the PSF cache: row s = source s's raw PSF at every pixel, 0 outside its
  // (2R+1)^2 window anchored at floor(loc) -- position_delta's old-window value
  [[maybe_unused]] float* pcw = nullptr;
  if constexpr (PC) {
    pcw = smem + (kImg + kMhWaves) * HWp + wave * S * HW;
    const int ph = lane / m.W, pw = lane - ph * m.W;
    const float fph = (float)ph + 0.5f, fpw = (float)pw + 0.5f;
    for (int s = 0; s < S; ++s) {
      const float hs = readlane(sh, s), ws = readlane(sw, s);
      const int fh = ifloor16(hs), fw = ifloor16(ws);
      const float dh = fph - hs, dw = fpw - ws;
      float v;
      if constexpr (TB) v = psf_tab(tab, tinv, fmaf(dh, dh, dw * dw));
      else v = psf_raw<MODEL>(m, fmaf(dh, dh, dw * dw));
      if (lane < HW) pcw[s * HW + lane] = (abs(ph - fh) <= m.R && abs(pw - fw) <= m.R) ? v : 0.f;
    }
    wave_sync();
  }
  SMC_TRACE(trow, 3);

  // ---- proposals, batched: lane 3b+d proposes dimension d (h, w, flux) of
  // iteration batch_k0 + b (b < kBatch), from the state at batch time.  An
  // entry goes stale only if an earlier accepted iteration of the batch moved
  // the same source (tracked in `dirty`); the batch is then recomputed.
  const int lb3 = lane / 3;
  const int d = lane - 3 * lb3;
  Dim dm;
  dm.isig = d < 2 ? a.isl : a.isf;
  dm.sig = d < 2 ? a.sl : a.sf;
  {
    float lb_h = a.lb_h, lb_w = a.lb_w, ub_h = a.ub_h, ub_w = a.ub_w;
    if (a.boxes) {  // the tile's own box (a partition of the padded image)
      const float* bx_ = a.boxes + 4 * t;
      lb_h = bx_[0];
      lb_w = bx_[1];
      ub_h = bx_[2];
      ub_w = bx_[3];
    }
    dm.lb = d == 0 ? lb_h : (d == 1 ? lb_w : a.lb_f);
    dm.ub = d == 0 ? ub_h : (d == 1 ? ub_w : a.ub_f);
  }
  const bool ablate_prop = kDiag && (a.ablate & SMCDET_MH_ABLATE_PROPOSAL) != 0;
  const bool ablate_lik = kDiag && (a.ablate & SMCDET_MH_ABLATE_LIKELIHOOD) != 0;

  // ---- draws: lane i of the cache holds iteration (block*64 + i) ------------
  float ru0 = 0.f, ru1 = 0.f, ru2 = 0.f, ru3 = 0.f, ru4 = 0.f;
  int rcomp = 0;
  auto refill = [&](int k0) {
    const int kk = k0 + lane;
    if constexpr (REPLAY) {
      if (kk < a.K) {
        const size_t r = ((size_t)kk * a.T + t) * N + n;
        rcomp = a.r_comp[r];
        ru1 = a.r_uloc[r * 2 + 0];
        ru2 = a.r_uloc[r * 2 + 1];
        ru3 = a.r_uflux[r];
        ru4 = a.r_uacc[r];
      }
    } else {
      const uint64_t ctr = a.offset + (uint64_t)kk;
      const uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32);
      const U4 r0 = philox4x32(c0, c1, (uint32_t)pid, kTagMH0, a.k0, a.k1);
      const U4 r1 = philox4x32(c0, c1, (uint32_t)pid, kTagMH1, a.k0, a.k1);
      ru0 = u01(r0.x);
      ru1 = u01(r0.y);
      ru2 = u01(r0.z);
      ru3 = u01(r0.w);
      ru4 = u01(r1.x);
    }
  };

  float bx = 0.f, bhd = 0.f;
  // per batch element b, precomputed in its lanes (amortised over the batch
  // instead of wave-uniform VALU work every iteration): bmu = current value
  // (lanes 3b+d); bfl = floor(current) | floor(proposed) << 16 (lanes 3b, 3b+1);
  // lane 3b+2: bampo/bampn = rate amplitudes g f psf_scale of the current /
  // proposed flux, bdp = prior term, bhs = summed Hastings term
  float bmu = 0.f, bampo = 0.f, bampn = 0.f, bdp = 0.f, bhs = 0.f, blu = 0.f;
  int bfl = 0;
  unsigned bmg = 1u;  // lane 3b+1: ceil(65536 / union-window width), for q / bw
  int bj = 0, batch_k0 = 0, batch_n = 0;
  uint64_t dirty = 0;
  auto compute_batch = [&](int k0) {
    const int n_ = min(min(kBatch, kWave - (k0 & 63)), K - k0);
    const int b = min(lb3, n_ - 1);
    const int kl = (k0 & 63) + b;
    int j;
    if constexpr (REPLAY) j = __shfl(rcomp, kl, kWave);
    else j = min((int)(__shfl(ru0, kl, kWave) * (float)Sj), Sj - 1);
    const float u1 = __shfl(ru1, kl, kWave), u2 = __shfl(ru2, kl, kWave);
    const float u3 = __shfl(ru3, kl, kWave);
    const float u = d == 0 ? u1 : (d == 1 ? u2 : u3);
    const float m0 = __shfl(sh, j, kWave), m1 = __shfl(sw, j, kWave), m2 = __shfl(sfx, j, kWave);
    const float mu = d == 0 ? m0 : (d == 1 ? m1 : m2);
    // the truncated normal's Phi(lb) and log-mass at the current value, in the
    // lane that proposes the dimension (recomputed per batch rather than
    // cached per source: no cache update on accept, fewer registers)
    float c_ph, c_lZ;
    tn_cache(mu, dm.isig, dm.lb, dm.ub, c_ph, c_lZ);
    float n_ph, n_lZ, blf;
    if (ablate_prop)
      propose_lane<true>(mu, c_ph, c_lZ, u, dm, bx, n_ph, n_lZ, bhd, blf);
    else
      propose_lane<false>(mu, c_ph, c_lZ, u, dm, bx, n_ph, n_lZ, bhd, blf);
    bmu = mu;
    bfl = (int)(((unsigned)ifloor16(mu) & 0xffffu) | ((unsigned)ifloor16(bx) << 16));
    {  // union-window width of the column anchors (meaningful in lane 3b+1)
      const int f0 = ifloor16(mu), f1 = ifloor16(bx);
      const int c0_ = max(min(f0, f1) - m.R, 0), c1_ = min(max(f0, f1) + m.R, m.W - 1);
      const unsigned bw_ = (unsigned)max(c1_ - c0_ + 1, 1);
      bmg = (65536u + bw_ - 1u) / bw_;
    }
    // lane 3b+2 (flux): amplitudes, prior term (kernel.py:64-112 via
    // prior.py:220-226: the uniform location terms are constant in the box)
    // and the Hastings sum of the triple, in the per-iteration order
    const float lf_cur = fast_log(mu);  // (lane 3b+2: mu = the current flux)
    bampo = m.g * mu * psf_scale<MODEL>(m);
    bampn = m.g * bx * psf_scale<MODEL>(m);
    bdp = ((float)j < count) ? -a.pr.ap1 * (blf - lf_cur) : 0.0f;
    // a location proposal clamped onto the box's upper edge (distributions.py:48)
    // has log prior -inf (Uniform.log_prob(high), prior.py:73): its lane's
    // term carries it into the summed Hastings + prior term of lane 3b+2
    if (d < 2 && bx >= dm.ub) bhd = -INFINITY;
    const float hd0 = __shfl(bhd, max(lane - 2, 0), kWave);
    const float hd1 = __shfl(bhd, max(lane - 1, 0), kWave);
    // log alpha = (Hastings + prior term) + tau * dll, accepted iff it is >= log U
    // (U <= min(1, exp(log alpha)) for U in [0, 1); nan rejects).
    bhs = (hd0 + hd1 + bhd) + bdp;  // -inf in lane 3b+2 iff entry b hits the edge
    blu = fast_log(__shfl(ru4, kl, kWave));
    bj = j;
    batch_k0 = k0;
    batch_n = n_;
    dirty = 0;
  };

  int accept = 0;
#ifdef SMCDET_TRACE
  unsigned tr_pos = 0, tr_acc = 0;
#endif
  // Progress-based issue priority: the SIMD's arbiter otherwise favours the
  // oldest of its 4 resident waves, which then finish one after another and
  // leave the SIMD with a single (latency-bound) wave for the last quarter of
  // the sweep.  Waves ahead of the others drop to a lower priority so the four
  // progress together and keep the SIMD saturated to the end.
  int prio_lvl = 0;
  __builtin_amdgcn_s_setprio(3);
  for (int k = 0; k < K; ++k) {
    const int lvl = (k * 4) / K;
    if (lvl != prio_lvl) {
      prio_lvl = lvl;
      if (lvl == 1) __builtin_amdgcn_s_setprio(2);
      else if (lvl == 2) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
    const int kl = k & 63;
    if (kl == 0) refill(k);
    if (k >= batch_k0 + batch_n) compute_batch(k);
    int b = k - batch_k0;
    int j = readlane(bj, 3 * b);
    if ((dirty >> j) & 1ull) {
      compute_batch(k);
      b = 0;
      j = readlane(bj, 0);
    }
    // the batch entry is current (its source was not moved since the batch);
    // its lane base as one SGPR (b's phi may sit in a VGPR)
    const int b3 = __builtin_amdgcn_readfirstlane(3 * b);
    Proposal P;
    P.j = j;
    P.h = readlane(bmu, b3);
    P.w = readlane(bmu, b3 + 1);
    P.hn = readlane(bx, b3);
    P.wn = readlane(bx, b3 + 1);
    P.fn = readlane(bx, b3 + 2);
    P.hast = readlane(bhs, b3 + 2);  // Hastings + prior terms
    const float log_u = readlane(blu, b3 + 2);
    // rate contributions g*f*psf, the psf normalisation folded into the amplitude
    const float amp_o = readlane(bampo, b3 + 2), amp_n = readlane(bampn, b3 + 2);

    // ---- likelihood difference -----------------------------------------------
    float dll;
    double new_ll = 0.0;
    float s_lam[NSL];
    int s_pix[NSL];
    [[maybe_unused]] float s_rv[RV ? NSL : 1];  // RV: the new 1/v of each slot
    [[maybe_unused]] float s_psi = 0.f;  // PC: the new window's PSF values (one slot)
    int npos = 0, bw = 1, r0 = 0, c0 = 0, nslots = 0;
    if constexpr (FULL) {
      const float ch = lane == P.j ? P.hn : sh, cw = lane == P.j ? P.wn : sw;
      const float cf = lane == P.j ? P.fn : sfx;
      if constexpr (PPL > 0) {
        float lamk[PPL > 0 ? PPL : 1];
        render_regs<MODEL, PPL>(m, lamk, ch, cw, cf, S, lane);
        new_ll = pixel_sum_regs<MODEL, PPL>(m, xs, lg, lamk, lane);
      } else {
        render_sources<MODEL>(m, lam, ch, cw, cf, S, lane);
        new_ll = pixel_sum<MODEL>(m, xs, lg, lam, nullptr, lane);
      }
      dll = (float)(new_ll - cur_ll);
    } else {
      const int flh = readlane(bfl, b3), flw = readlane(bfl, b3 + 1);
      const int fh0 = (int)(int16_t)(flh & 0xffff), fh1 = flh >> 16;
      const int fw0 = (int)(int16_t)(flw & 0xffff), fw1 = flw >> 16;
      r0 = max(min(fh0, fh1) - m.R, 0);
      const int r1 = min(max(fh0, fh1) + m.R, m.H - 1);
      c0 = max(min(fw0, fw1) - m.R, 0);
      const int c1 = min(max(fw0, fw1) + m.R, m.W - 1);
      bw = c1 - c0 + 1;
      npos = (r1 >= r0 && c1 >= c0 && !ablate_lik) ? (r1 - r0 + 1) * bw : 0;
      nslots = (npos + kWave - 1) / kWave;
#ifdef SMCDET_TRACE
      tr_pos += npos;
#endif
      const unsigned magic = (unsigned)readlane((int)bmg, b3 + 1);  // q/bw, q < 1024
      const bool same = (fh0 == fh1) && (fw0 == fw1);
      const int ao_h = fh0 - m.R - r0, ao_w = fw0 - m.R - c0;
      const int an_h = fh1 - m.R - r0, an_w = fw1 - m.R - c0;
      // NS predicated slots in one basic block, with the (independent) next
      // proposal in the same block so the scheduler can interleave the two
      auto slots = [&](auto NS, auto WIN) -> float {
        constexpr int ns = decltype(NS)::value;
        constexpr bool win = decltype(WIN)::value;
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < ns; ++i) {
          const int q = i * kWave + lane;
          const bool valid = q < npos;
          const int aa = (int)(__umul24((unsigned)q, magic) >> 16);
          const int bb = q - (int)__umul24((unsigned)aa, (unsigned)bw);
          const int ph = r0 + aa, pw = c0 + bb;
          const int p = valid ? (int)__umul24((unsigned)ph, (unsigned)m.W) + pw : HW + lane;
          float lnew, rnew, e;
          if constexpr (PC)
            e = position_delta_pc<MODEL, win, TB>(m, xs, lg, lam, pcw + P.j * HW, tab, tinv, p,
                                                  valid, aa, bb, ph, pw, P, amp_o, amp_n, an_h,
                                                  an_w, lnew, s_psi);
          else
            e = position_delta<MODEL, win, GL, RV, TB>(m, xs, lg, lam, rv, tab, tinv, p, aa, bb,
                                                       ph, pw, P, amp_o, amp_n, ao_h, ao_w, an_h,
                                                       an_w, lnew, rnew);
          acc += valid ? e : 0.f;
          s_lam[i] = lnew;
          if constexpr (RV) s_rv[i] = rnew;
          s_pix[i] = p;
        }
        return acc;
      };
      // the same, two slots (2i, 2i+1) per lane at once in packed arithmetic
      // (ODD: one more slot 2*np, one position per lane, as `slots` does)
      auto pairs = [&](auto NP, auto ODD, auto WIN) -> float {
        constexpr int np = decltype(NP)::value;
        constexpr bool odd = decltype(ODD)::value;
        constexpr bool win = decltype(WIN)::value;
        f2 acc = {0.f, 0.f};
#pragma unroll
        for (int i = 0; i < np; ++i) {
          int aa[2], bb[2], p[2];
          bool valid[2];
          f2 fph, fpw;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int q = (2 * i + h) * kWave + lane;
            valid[h] = q < npos;
            aa[h] = (int)(__umul24((unsigned)q, magic) >> 16);
            bb[h] = q - (int)__umul24((unsigned)aa[h], (unsigned)bw);
            const int ph = r0 + aa[h], pw = c0 + bb[h];
            p[h] = valid[h] ? (int)__umul24((unsigned)ph, (unsigned)m.W) + pw : HW + lane;
            fph[h] = (float)ph + 0.5f;
            fpw[h] = (float)pw + 0.5f;
          }
          f2 lnew, rnew;
          f2 e = position_delta2<MODEL, win, GL, RV, TB>(m, xs, lg, lam, rv, tab, tinv, p, aa, bb,
                                                         fph, fpw, P, amp_o, amp_n, ao_h, ao_w,
                                                         an_h, an_w, lnew, rnew);
          e.x = valid[0] ? e.x : 0.f;
          e.y = valid[1] ? e.y : 0.f;
          acc += e;
          s_lam[2 * i] = lnew.x;
          s_lam[2 * i + 1] = lnew.y;
          if constexpr (RV) {
            s_rv[2 * i] = rnew.x;
            s_rv[2 * i + 1] = rnew.y;
          }
          s_pix[2 * i] = p[0];
          s_pix[2 * i + 1] = p[1];
        }
        float acc1 = 0.f;
        if constexpr (odd) {
          const int q = 2 * np * kWave + lane;
          const bool valid = q < npos;
          const int aa = (int)(__umul24((unsigned)q, magic) >> 16);
          const int bb = q - (int)__umul24((unsigned)aa, (unsigned)bw);
          const int ph = r0 + aa, pw = c0 + bb;
          const int p = valid ? (int)__umul24((unsigned)ph, (unsigned)m.W) + pw : HW + lane;
          float lnew, rnew;
          const float e = position_delta<MODEL, win, GL, RV, TB>(m, xs, lg, lam, rv, tab, tinv, p,
                                                             aa, bb, ph, pw, P, amp_o, amp_n,
                                                             ao_h, ao_w, an_h, an_w, lnew, rnew);
          acc1 = valid ? e : 0.f;
          s_lam[2 * np] = lnew;
          if constexpr (RV) s_rv[2 * np] = rnew;
          s_pix[2 * np] = p;
        }
        return (acc.x + acc.y) + acc1;
      };
      using I0 = std::integral_constant<int, 0>;
      using I1 = std::integral_constant<int, 1>;
      using One = std::true_type;
      using Zero = std::false_type;
      using I2 = std::integral_constant<int, 2>;
      using I3 = std::integral_constant<int, 3>;
      using I4 = std::integral_constant<int, 4>;
      using I5 = std::integral_constant<int, 5>;
      using I8 = std::integral_constant<int, kSlots>;
      using Win = std::true_type;
      using Same = std::false_type;
      // The union-window positions beyond the register slots (a jump of
      // several px; rare): their delta (WRITE = false) or their rate-image
      // update after an accept (WRITE = true).
      auto far_positions = [&](auto WRITE) -> float {
        float acc = 0.f;
        const float inv_bw = 1.0f / (float)bw;
        for (int q = kSlots * kWave + lane; q < npos; q += kWave) {
          const int aa = (int)(((float)q + 0.5f) * inv_bw);
          const int bb = q - (int)__umul24((unsigned)aa, (unsigned)bw);
          const int ph = r0 + aa, pw = c0 + bb;
          const int p = (int)__umul24((unsigned)ph, (unsigned)m.W) + pw;
          float lnew, rnew;
          acc += position_delta<MODEL, true, GL, RV, TB>(m, xs, lg, lam, rv, tab, tinv, p, aa, bb,
                                                         ph, pw, P, amp_o, amp_n, ao_h, ao_w, an_h,
                                                         an_w, lnew, rnew);
          if constexpr (decltype(WRITE)::value) {
            lam[p] = lnew;
            if constexpr (RV) rv[p] = rnew;
          }
        }
        return acc;
      };
      // Reduction, accept decision (kernel.py:114-116) and rate-image update,
      // inlined into each slot variant's own block: the NS slots' new rates
      // and pixel indices (s_lam / s_pix) die inside it instead of flowing
      // into a merge point (their phi copies cost ~16 VALU moves per
      // iteration).  log alpha = (Hastings + prior term) + tau * dll,
      // accepted iff it is >= log U (U <= min(1, exp(log alpha)) for U in
      // [0, 1); nan rejects).  An edge hit (hast = -inf) never updates the
      // state (the sweep ends below).
      auto finish = [&](float dsum, auto NS) {
        constexpr int ns = decltype(NS)::value;
        constexpr bool kFar = NSL > 1 && ns >= kSlots;
        if (kFar && npos > kSlots * kWave) dsum += far_positions(std::false_type{});
        dll = wave_sum(dsum);
        accept = __builtin_amdgcn_ballot_w64(fmaf(tau, dll, P.hast) >= log_u) != 0;
        if (accept && !edge_hit(P.hast)) {
#pragma unroll
          for (int i = 0; i < ns; ++i)
            if (i < nslots) {
              lam[s_pix[i]] = s_lam[i];
              // the moved pixels' 1/v: the delta's own reciprocal of the new rate
              if constexpr (RV) rv[s_pix[i]] = s_rv[i];
            }
          if (kFar && npos > kSlots * kWave) (void)far_positions(std::true_type{});
          wave_sync();
        }
      };
      // The 16x16 block form of a same-anchor step (M71; delta_from_dl2): the
      // block of the tile at (r0, c0) holds the union box's first 16 rows and
      // columns, the strip (one slot, s_*[4]) its 17th row and / or column.
      // Taken where the box has 16 or 17 rows and columns and the per-pixel
      // form would need a.blk_slots (default 5) slots: a same-box microbench
      // at the C2 state measured the MH launch 4.7-5.2% faster with it there;
      // a first version that also took 4-slot boxes (16x16, and masked blocks
      // of clipped boxes) gained only 1.2%.
      constexpr bool kBlk = MODEL == SMCDET_MODEL_M71 && PPL > 1 && !GL && !TB && PAIRED;
      bool blk = false;
      if constexpr (kBlk)
        blk = same && a.blk_slots > 0 && m.R <= 8 && nslots >= a.blk_slots && r1 - r0 >= 15 &&
              c1 - c0 >= 15 && r1 - r0 <= 16 && c1 - c0 <= 16;  // (the strip holds one row and one
                                                                 // column: R <= 8, clipped or not)
      auto block = [&]() -> float {
        const int li = lane & 15, lk = lane >> 4;
        // MFMA operands: lane l is A[l & 15][l >> 4] and B[l >> 4][l & 15]
        const bool knew = lk < 2;
        const float kk = (lk & 1) ? m.k2 : m.k1;
        const float ak = (knew ? amp_n : -amp_o) * ((lk & 1) ? m.b : 1.0f);
        const float dy = ((float)(r0 + li) + 0.5f) - (knew ? P.hn : P.h);
        const float dx = ((float)(c0 + li) + 0.5f) - (knew ? P.wn : P.w);
        const float av = ak * fast_exp2(kk * (dy * dy));
        const float bv = fast_exp2(kk * (dx * dx));
        const f4 g = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        // this lane's block pixels: rows prow0 + r (r < 4) of column pcol
        const int prow0 = r0 + 4 * lk, pcol = c0 + li;
        const float fpw = (float)pcol + 0.5f;
        const float dwo = fpw - P.w, dwn = fpw - P.wn;
        const f2 dwo2 = {dwo * dwo, dwo * dwo}, dwn2 = {dwn * dwn, dwn * dwn};
        const float po = amp_o * m.p0, pn = amp_n * m.p0;
        const int pb = prow0 * m.W + pcol;
        const float fph0 = (float)prow0 + 0.5f;
        f2 acc = {0.f, 0.f};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f2 fph = {fph0 + (float)(2 * h), fph0 + (float)(2 * h + 1)};
          const f2 dho = fph - P.h, dhn = fph - P.hn;
          const f2 e3o = exp2_2(m.kb * log2_2(fma2(fma2(dho, dho, dwo2), m.k3, 1.0f)));
          const f2 e3n = exp2_2(m.kb * log2_2(fma2(fma2(dhn, dhn, dwn2), m.k3, 1.0f)));
          const f2 dl = f2{g[2 * h], g[2 * h + 1]} + fma2(e3n, pn, -po * e3o);
          const int p[2] = {pb + 2 * h * m.W, pb + (2 * h + 1) * m.W};
          const f2 lo = {lam[p[0]], lam[p[1]]};
          const f2 x = {xs[p[0]], xs[p[1]]};
          f2 lnew, rnew;
          acc += delta_from_dl2<MODEL, RV>(m, x, lo, dl, rv, p, lnew, rnew);
          s_lam[2 * h] = lnew.x;
          s_lam[2 * h + 1] = lnew.y;
          s_pix[2 * h] = p[0];
          s_pix[2 * h + 1] = p[1];
          if constexpr (RV) {
            s_rv[2 * h] = rnew.x;
            s_rv[2 * h + 1] = rnew.y;
          }
        }
        // the strip: the box's 17th row, then its 17th column over the
        // block's rows, one pixel per lane (<= 33)
        const int nb = r1 > r0 + 15 ? c1 - c0 + 1 : 0;
        const int nr = c1 > c0 + 15 ? 16 : 0;
        const bool valid = lane < nb + nr, bot = lane < nb;
        const int ph = bot ? r0 + 16 : r0 + (lane - nb);
        const int pw = bot ? c0 + lane : c0 + 16;
        const int p = valid ? ph * m.W + pw : HW + lane;
        float lnew, rnew;
        const float e = position_delta<MODEL, false, false, RV, false>(
            m, xs, lg, lam, rv, tab, tinv, p, 0, 0, ph, pw, P, amp_o, amp_n, 0, 0, 0, 0, lnew, rnew);
        s_lam[4] = lnew;
        s_pix[4] = p;
        if constexpr (RV) s_rv[4] = rnew;
        return (acc.x + acc.y) + (valid ? e : 0.f);
      };
      if constexpr (NSL == 1) {
        // small tiles (latency-bound at 7 waves per SIMD): one reduction and
        // accept after the merge measured faster (C4 4.95 vs 5.12 ms)
        float dsum = 0.f;
        if (nslots == 1) dsum = same ? slots(I1{}, Same{}) : slots(I1{}, Win{});
        dll = wave_sum(dsum);
        accept = __builtin_amdgcn_ballot_w64(fmaf(tau, dll, P.hast) >= log_u) != 0;
      } else if (blk) {
        if constexpr (kBlk) {
          nslots = 5;  // (finish: the writes of s_*[0..5): 4 block pixels + the strip)
          finish(block(), I5{});
        }
      } else if (nslots == 0) {
        finish(0.f, I0{});
      } else if (PAIRED && nslots == 1) {
        if (same) finish(pairs(I0{}, One{}, Same{}), I1{});
        else finish(pairs(I0{}, One{}, Win{}), I1{});
      } else if (PAIRED && nslots == 2) {
        if (same) finish(pairs(I1{}, Zero{}, Same{}), I2{});
        else finish(pairs(I1{}, Zero{}, Win{}), I2{});
      } else if (PAIRED && nslots <= 3) {
        if (same) finish(pairs(I1{}, One{}, Same{}), I3{});
        else finish(pairs(I1{}, One{}, Win{}), I3{});
      } else if (PAIRED && nslots <= 4) {
        if (same) finish(pairs(I2{}, Zero{}, Same{}), I4{});
        else finish(pairs(I2{}, Zero{}, Win{}), I4{});
      } else if (PAIRED && nslots <= 5) {
        if (same) finish(pairs(I2{}, One{}, Same{}), I5{});
        else finish(pairs(I2{}, One{}, Win{}), I5{});
      } else if (PAIRED) {
        // 6 slots (both anchors moved): rare; the scalar form needs fewer
        // registers than three packed pairs
        finish(slots(I8{}, Win{}), I8{});
      } else if (nslots <= 3) {
        if (same) finish(slots(I3{}, Same{}), I3{});
        else finish(slots(I3{}, Win{}), I3{});
      } else if (nslots <= 5) {
        if (same) finish(slots(I5{}, Same{}), I5{});
        else finish(slots(I5{}, Win{}), I5{});
      } else {
        finish(slots(I8{}, Win{}), I8{});
      }
    }
    if constexpr (FULL) {
      // ---- accept / reject (kernel.py:114-128) --------------------------------
      const float loga = fmaf(tau, dll, P.hast);
      accept = __builtin_amdgcn_readfirstlane((loga >= log_u) ? 1 : 0);
    }
#ifdef SMCDET_TRACE
    tr_acc += accept;
#endif
    if constexpr (REPLAY) {  // decision trace (tests only; not in the Philox build)
      if (lane == 0) {
        const size_t r = ((size_t)k * a.T + t) * N + n;
        if (a.r_loga) a.r_loga[r] = fmaf(tau, dll, P.hast);
        if (a.r_accept) a.r_accept[r] = (uint8_t)(accept && P.hast != -INFINITY);
      }
    }
    // An edge hit (log prior -inf) is rejected, and the reference caches the
    // rejected -inf log target as -inf * 0 = NaN (kernel.py:125), so every
    // later proposal of this particle in the sweep is rejected too: the state
    // is final, the sweep ends.  (Measured: this per-iteration scalar test
    // costs ~1% of the launch; once-per-batch forms that change loop-carried
    // state cost 3-13% through register allocation)  Not
    // reproduced: U = 0 exactly with an edge hit (probability 2^-24 per hit),
    // where the reference accepts and its cached target becomes -inf, so it
    // accepts every later proposal of the sweep; here the sweep ends.
    if (edge_hit(P.hast)) break;
    if (accept) {
      if constexpr (FULL) {
        cur_ll = new_ll;
      } else {
        if constexpr (NSL == 1) {
          if (nslots == 1) {
            lam[s_pix[0]] = s_lam[0];
            if constexpr (PC)  // (masked lanes: s_pix = HW + lane, outside the row)
              if (s_pix[0] < HW) pcw[P.j * HW + s_pix[0]] = s_psi;
          }
          wave_sync();
        }
        cur_ll += (double)dll;
      }
      // source j takes the proposal (v_writelane)
      sh = writelane(P.hn, P.j, sh);
      sw = writelane(P.wn, P.j, sw);
      sfx = writelane(P.fn, P.j, sfx);
      dirty |= 1ull << P.j;
    }
  }

  __builtin_amdgcn_s_setprio(0);
  SMC_TRACE(trow, 4);
#ifdef SMCDET_TRACE
  SMC_WAVE_STAT(trow, 5, tr_pos);
  SMC_WAVE_STAT(trow, 6, tr_acc);
#endif
  // ---- write back --------------------------------------------------------------
  if (lane < S) {
    a.locs_out[(pid * S + lane) * 2 + 0] = sh;
    a.locs_out[(pid * S + lane) * 2 + 1] = sw;
    a.fluxes_out[pid * S + lane] = sfx;
  }
  if (a.loglik_out) {
    double ll;
    if constexpr (!FULL) {
      // the LDS rate image is current (every accepted move was applied to it):
      // sum the per-pixel terms over it instead of re-rendering all sources
      ll = pixel_sum<MODEL>(m, xs, lg, lam, nullptr, lane);
    } else if constexpr (PPL > 0) {
      float lamk[PPL > 0 ? PPL : 1];
      render_regs<MODEL, PPL>(m, lamk, sh, sw, sfx, S, lane);
      ll = pixel_sum_regs<MODEL, PPL>(m, xs, lg, lamk, lane);
    } else {
      render_sources<MODEL>(m, lam, sh, sw, sfx, S, lane);
      ll = pixel_sum<MODEL>(m, xs, lg, lam, nullptr, lane);
    }
    if (lane == 0) a.loglik_out[pid] = (float)ll;
  }
  if constexpr (!FULL && !GL) {  // (GL: the sweep worked in rate_out's row)
    if (a.rate_out) {
      float* rout = a.rate_out + pid * (size_t)HW;
      if constexpr (PPL > 0) {
        copy_out_regs<PPL>(lam, rout, HW, lane);
      } else if ((HW & 3) == 0) {
        for (int p = 4 * lane; p < HW; p += 4 * kWave)
          *reinterpret_cast<float4*>(rout + p) = make_float4(lam[p], lam[p + 1], lam[p + 2],
                                                             lam[p + 3]);
      } else {
        for (int p = lane; p < HW; p += kWave) rout[p] = lam[p];
      }
    }
  }
  SMC_TRACE(trow, 5);
  SMC_WAVE_MARK(trow, 1);
  // ---- acceptance rate of the last iteration (kernel.py:130), no extra launch:
  // waves add into LDS; the workgroup's last wave adds the total to the tile's
  // counter and takes a ticket; the tile's last workgroup writes the rate and
  // re-zeroes counter and ticket (the workspace is zero on entry and exit).
  // With the fused tail, the tail workgroup (another CU) reads every wave's
  // loglik_out / rate_out: each wave releases its own stores at agent scope
  // before it counts itself done, rather than relying on the last wave's
  // fence being cumulative over the workgroup-scope ones.
  if constexpr (TAIL) __threadfence();
  if (lane == 0) {
    const int nw = min(kMhWaves, N - (int)blockIdx.x * kMhWaves);
    if (accept && a.K > 0) atomicAdd(&wg_acc, 1);
    // orders this wave's wg_acc add before its wg_done ticket (both builds;
    // the TAIL build's agent-scope fence above precedes both atomics)
    __threadfence_block();
    if (atomicAdd(&wg_done, 1) == nw - 1) {
      // the tile's count (high word) and ticket (low word) in ONE 64-bit
      // atomic: the tile's last workgroup reads every other workgroup's count
      // in the value it replaces, with no fence between a count and a ticket
      // (an agent-scope fence is an L2 write-back, right after this
      // workgroup's rate-image stores).  acc_count [2T] int32 = [T] uint64,
      // 8-byte aligned (host-checked).
      unsigned long long* slot = reinterpret_cast<unsigned long long*>(a.acc_count) + t;
      const unsigned long long mine = (unsigned long long)(unsigned)atomicAdd(&wg_acc, 0);
      const unsigned long long old = atomicAdd(slot, (mine << 32) | 1ull);
      if ((unsigned)(old & 0xffffffffull) == gridDim.x - 1) {
        const unsigned long long total = (old >> 32) + mine;
        atomicExch(slot, 0ull);
        a.acc_rate[t] = (float)total / (float)N;
        wg_last = 1;
      }
    }
  }
  // ---- fused SMC iteration: the tile's last workgroup tempers, reweights and
  // draws the next resampling indices once every particle's log-likelihood is
  // in (the ticket above); its LDS (rate images written back) becomes the
  // tile pass's buffer.  Not for 8x8 tiles: their 7 workgroups per CU cannot
  // hold the 2N+1-word buffer (the host launches the tile kernel instead).
  if constexpr (TAIL && PPL != 1 && !FULL && PAIRED) {
    {
      __shared__ TileRed tail_red;
      __syncthreads();
      if (wg_last) {
        // acquire: the other workgroups' loglik_out stores (released by their
        // device-scope fence before the ticket)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        // the tail's arguments are read only here: the opaque pointer keeps
        // the compiler from hoisting their kernarg loads above the sweep,
        // where they would stay live in SGPRs across the MH loop (spills)
        // (MhArgs is the kernel's only argument: offset 0 of the kernarg
        // segment; taking &a.tail instead would copy all of `a` to scratch)
        const TileArgs* tp = reinterpret_cast<const TileArgs*>(
            (const char*)__builtin_amdgcn_kernarg_segment_ptr() +
            offsetof(MhArgs, tail));
        __asm__ volatile("" : "+s"(tp));
        tile_work<kMhBlock, 8>(*tp, t, smem, tail_red, -1);
      }
    }
  }
}

template <int MODEL, bool REPLAY, bool FULL, int PPL>
static int launch_mh1(const MhArgs& a, dim3 grid, size_t lds, hipStream_t st) {
  // FULL mode never evaluates union-window slots: one instantiation
  constexpr bool kPair = !FULL;
  // (scalar slots: diagnostic build only, host-checked)
  const bool paired = kPair && !(kDiag && a.scalar_slots);
  // the fused tail exists only where tail_fusable() allows it
  constexpr bool kTail = !FULL && PPL != 1;
  const bool tail = kTail && paired && a.has_tail;
  if (a.has_tail && !tail) return set_error(SMCDET_EINVAL, "fused step: unsupported shape");
  // The LDS-cached variants, richest first, where their workgroups per CU
  // (the occupancy the instantiation is built for) still fit the 160 KiB:
  // PC (small tiles) = the per-wave PSF cache, RV (M71, 65..1024 px) = the
  // per-wave 1/v image, TB = the radial PSF table (diagnostic build: a.psf_tab
  // set by the host for M71 models whose table passes its accuracy check).
  auto fits = [&](size_t bytes, int wg_per_cu) {
    return (size_t)wg_per_cu * (bytes + 1024) <= 160 * 1024;
  };
  [[maybe_unused]] auto with_tab = [&](size_t bytes) {
    return ((bytes + 15) & ~(size_t)15) + (size_t)kTabNodes * sizeof(float4);
  };
  auto go_variant = [&](auto kern, size_t bytes) -> int {
    int rc = ensure_lds((const void*)kern, bytes);
    if (rc) return rc;
    launch_sweep(kern, grid, dim3(kMhBlock), bytes, st, a);
    return SMCDET_OK;
  };
  [[maybe_unused]] const bool tb = kDiag && a.psf_tab != nullptr && paired && !tail;
  if constexpr (PPL == 1 && !FULL) {
    // small tiles: the PSF cache (S rows of H*W floats per wave)
    const size_t lds_pc = lds + (size_t)kMhWaves * a.S * a.m.H * a.m.W * sizeof(float);
    constexpr int wg = SMCDET_SMALL_TILE_WAVES;
    if constexpr (MODEL == SMCDET_MODEL_M71 && kDiag) {
      if (tb && !a.no_psf_cache && fits(with_tab(lds_pc), wg))
        return go_variant(mh_sweep_kernel<MODEL, REPLAY, FULL, PPL, true, false, false, true,
                                          false, true>, with_tab(lds_pc));
    }
    if (paired && !a.no_psf_cache && fits(lds_pc, wg))
      return go_variant(mh_sweep_kernel<MODEL, REPLAY, FULL, PPL, true, false, false, true>,
                        lds_pc);
    if constexpr (MODEL == SMCDET_MODEL_M71 && kDiag) {
      if (tb && fits(with_tab(lds), wg))
        return go_variant(mh_sweep_kernel<MODEL, REPLAY, FULL, PPL, true, false, false, false,
                                          false, true>, with_tab(lds));
    }
  }
  if constexpr (MODEL == SMCDET_MODEL_M71 && PPL > 1 && !FULL) {
    // M71 register-render tiles: the 1/v image (HWp floats per wave) and / or
    // the PSF table, at 4 workgroups per CU (4 waves per SIMD).  The 1/v image
    // always fits at these sizes (9 (H*W + 64) floats per workgroup), so
    // the product's only other M71 variant here is the fused tail's.
    const size_t lds_rv = lds + (size_t)kMhWaves * (a.m.H * a.m.W + kWave) * sizeof(float);
    const bool rv = paired && !tail && !(kDiag && a.no_rcp_cache);
    if constexpr (kDiag) {
      if (tb && rv && fits(with_tab(lds_rv), 4))
        return go_variant(mh_sweep_kernel<MODEL, REPLAY, FULL, PPL, true, false, false, false,
                                          true, true>, with_tab(lds_rv));
      if (tb && fits(with_tab(lds), 4))
        return go_variant(mh_sweep_kernel<MODEL, REPLAY, FULL, PPL, true, false, false, false,
                                          false, true>, with_tab(lds));
    }
    if (rv && fits(lds_rv, 4))
      return go_variant(mh_sweep_kernel<MODEL, REPLAY, FULL, PPL, true, false, false, false, true>,
                        lds_rv);
    if constexpr (!kDiag) {
      if (!tail) return set_error(SMCDET_EUNSUPPORTED, "M71 sweep: the 1/v image does not fit");
    }
  }
  // M71 register-render tiles without the fused tail take the 1/v variant
  // above: the plain paired instantiation is the diagnostic build's
  // (SMCDET_MH_NO_RCP_CACHE) there; scalar slots likewise
  constexpr bool kPlainPaired = kPair && (kDiag || !(MODEL == SMCDET_MODEL_M71 && PPL > 1));
  constexpr bool kUnpaired = FULL || kDiag;
  const void* fn = nullptr;
  if (tail) {
    if constexpr (kTail) fn = (const void*)mh_sweep_kernel<MODEL, REPLAY, FULL, PPL, kPair, kTail>;
  } else if (paired) {
    if constexpr (kPlainPaired) fn = (const void*)mh_sweep_kernel<MODEL, REPLAY, FULL, PPL, kPair, false>;
  } else {
    if constexpr (kUnpaired) fn = (const void*)mh_sweep_kernel<MODEL, REPLAY, FULL, PPL, false, false>;
  }
  if (!fn) return set_error(SMCDET_EUNSUPPORTED, "MH sweep variant not in this build");
  int rc = ensure_lds(fn, lds);
  if (rc) return rc;
  if (tail) {
    if constexpr (kTail)
      launch_sweep(mh_sweep_kernel<MODEL, REPLAY, FULL, PPL, kPair, kTail>, grid, dim3(kMhBlock),
                   lds, st, a);
  } else if (paired) {
    if constexpr (kPlainPaired)
      launch_sweep(mh_sweep_kernel<MODEL, REPLAY, FULL, PPL, kPair, false>, grid, dim3(kMhBlock),
                   lds, st, a);
  } else {
    if constexpr (kUnpaired)
      launch_sweep(mh_sweep_kernel<MODEL, REPLAY, FULL, PPL, false, false>, grid, dim3(kMhBlock),
                   lds, st, a);
  }
  return SMCDET_OK;
}

// tiles above the LDS budget (M71 only; host-checked): paired slots, no
// fused tail, no dynamic LDS
template <int MODEL, bool REPLAY, bool FULL>
static int launch_mh_gl(const MhArgs& a, dim3 grid, hipStream_t st) {
  if (a.has_tail || (kDiag && a.scalar_slots))
    return set_error(SMCDET_EUNSUPPORTED, "tiles above %d pixels: no fused step / scalar slots",
                     kMaxLdsPixels);
  constexpr bool kPair = !FULL;
  launch_sweep(mh_sweep_kernel<MODEL, REPLAY, FULL, 0, kPair, false, true>, grid, dim3(kMhBlock),
               0, st, a);
  return SMCDET_OK;
}

template <int MODEL, bool REPLAY, bool FULL>
static int launch_mh_ppl(const MhArgs& a, dim3 grid, size_t lds, hipStream_t st) {
  const int HW = a.m.H * a.m.W;
  if constexpr (MODEL == SMCDET_MODEL_M71) {
    if (HW > kMaxLdsPixels) return launch_mh_gl<MODEL, REPLAY, FULL>(a, grid, st);
  }
  if (a.S <= kWave) {
    if (HW <= 64) return launch_mh1<MODEL, REPLAY, FULL, 1>(a, grid, lds, st);
    if (HW <= 256) return launch_mh1<MODEL, REPLAY, FULL, 4>(a, grid, lds, st);
    if (HW <= 1024) return launch_mh1<MODEL, REPLAY, FULL, 16>(a, grid, lds, st);
  }
  return launch_mh1<MODEL, REPLAY, FULL, 0>(a, grid, lds, st);
}

template <int MODEL>
static int launch_mh(const MhArgs& a, bool replay, bool full, dim3 grid, size_t lds,
                     hipStream_t st) {
  if (replay)
    return full ? launch_mh_ppl<MODEL, true, true>(a, grid, lds, st)
                : launch_mh_ppl<MODEL, true, false>(a, grid, lds, st);
  return full ? launch_mh_ppl<MODEL, false, true>(a, grid, lds, st)
              : launch_mh_ppl<MODEL, false, false>(a, grid, lds, st);
}

}  // namespace smcdet

using namespace smcdet;

SMCDET_TRACE_READER(smcdet_trace_read_mh)
SMCDET_WAVE_READER(smcdet_trace_read_waves)

// the fused step's shape test; lds: the launch's dynamic LDS bytes
static bool tail_fusable(const smcdet_image_model_t& m, int N, int S, uint32_t flags,
                         size_t* lds) {
  const size_t HWp = (size_t)m.H * m.W + kWave;
  const size_t mh_lds =
      ((m.model == SMCDET_MODEL_POISSON ? 2 : 1) * HWp + (size_t)kMhWaves * HWp) * sizeof(float);
  const size_t need = mh_lds > tile_lds_bytes(N) ? mh_lds : tile_lds_bytes(N);
  if (lds) *lds = need;
  if (flags & (SMCDET_MH_FULL_RECOMPUTE | SMCDET_MH_SCALAR_SLOTS)) return false;
  if (m.H * m.W > kMaxLdsPixels) return false;  // global-memory tiles: two launches
  if (N % kMhWaves != 0 || N > kTailMaxN) return false;
  if (S <= kWave && m.H * m.W <= 64) return false;  // small-tile instantiation (PPL = 1)
  // 4 waves per SIMD = 4 workgroups per CU must still fit the 160 KiB LDS
  return 4 * (need + 2048) <= 160 * 1024;
}

#ifdef SMCDET_DIAG  // the radial PSF table: diagnostic build only
// ---- the radial PSF table (psf_tab, device.h) --------------------------------
// Device copies live in a module-scope table of slots, one per (device, PSF
// parameters); a slot is filled once (upload + stream synchronisation, so any
// later launch on any stream sees it), reused by every later sweep of those
// parameters and never recycled (parameter sets past kTabSlots fall back to
// the exp2/log2 form).
namespace smcdet {
constexpr int kTabSlots = 8;
__device__ float4 g_psf_tab[kTabSlots][kTabNodes];

struct TabEntry {
  int dev, slot;
  float key[8];
  float inv_h;
};
static std::mutex g_tab_mu;
static std::vector<TabEntry> g_tab_entries;

// psi(r^2) of psf_raw (device.h) for the float32 model constants, in double
static double psf_raw_d(const DevModel& m, double x) {
  return exp2((double)m.k1 * x) + (double)m.b * exp2((double)m.k2 * x) +
         (double)m.p0 * exp2((double)m.kb * log2(1.0 + (double)m.k3 * x));
}

// The cubic per node (least squares at 16 Chebyshev points of t in [-1/2,
// 1/2]; node 0 only [0, 1/2]) over r^2 in [0, 2(R + 3/2)^2]: every position of
// a window (|dh|, |dw| <= R + 1/2) and of a union window of anchors one pixel
// apart.  Returns false when the fit's relative error exceeds 2e-7 anywhere
// (an unusually sharp profile or a large radius): the sweep then keeps the
// exp2/log2 form, whose float32 evaluation errs by up to 7.5e-7.  (M71 at
// R = 8: fit error 1.1e-7 at r^2 = 0.53, about half an ulp of the core value;
// 3.0e-7 with the float32 coefficients and Horner steps.)
static bool psf_table_build(const DevModel& m, float4* tab, float* inv_h_out) {
  const double xmax = 2.0 * (m.R + 1.5) * (m.R + 1.5);
  const float inv_h = (float)(kTabIntervals / xmax);
  const double h = 1.0 / (double)inv_h;  // the spacing the device's index implies
  constexpr int kPts = 16;
  double worst = 0.0;
  for (int i = 0; i < kTabNodes; ++i) {
    double ata[4][5] = {};
    for (int k = 0; k < kPts; ++k) {
      const double c = 0.5 * cos((2.0 * k + 1.0) / (2.0 * kPts) * M_PI);
      const double t = i == 0 ? 0.5 * (c + 0.5) : c;
      const double y = psf_raw_d(m, (i + t) * h);
      const double v[4] = {1.0, t, t * t, t * t * t};
      for (int r = 0; r < 4; ++r) {
        for (int q = 0; q < 4; ++q) ata[r][q] += v[r] * v[q];
        ata[r][4] += v[r] * y;
      }
    }
    for (int c = 0; c < 4; ++c) {  // Gauss-Jordan on the 4x4 normal equations
      int piv = c;
      for (int r = c + 1; r < 4; ++r)
        if (fabs(ata[r][c]) > fabs(ata[piv][c])) piv = r;
      for (int q = 0; q < 5; ++q) std::swap(ata[c][q], ata[piv][q]);
      for (int r = 0; r < 4; ++r) {
        if (r == c) continue;
        const double f = ata[r][c] / ata[c][c];
        for (int q = c; q < 5; ++q) ata[r][q] -= f * ata[c][q];
      }
    }
    double co[4];
    for (int r = 0; r < 4; ++r) co[r] = ata[r][4] / ata[r][r];
    if (!(std::isfinite(co[0]) && std::isfinite(co[1]) && std::isfinite(co[2]) &&
          std::isfinite(co[3])))
      return false;
    for (int k = 0; k <= 8; ++k) {  // the fit's own error (double), node interval
      const double t = i == 0 ? 0.0625 * k : -0.5 + 0.125 * k;
      const double y = psf_raw_d(m, (i + t) * h);
      const double pv = co[0] + t * (co[1] + t * (co[2] + t * co[3]));
      if (y > 0) worst = fmax(worst, fabs(pv - y) / y);
    }
    tab[i] = make_float4((float)co[0], (float)co[1], (float)co[2], (float)co[3]);
  }
  *inv_h_out = inv_h;
  return worst <= 2e-7;
}

// the device table for this model (null: not applicable -> exp2/log2 form)
static int psf_table_device(const smcdet_image_model_t& mdl, const DevModel& m, hipStream_t st,
                            const float4** out, float* inv_h) {
  *out = nullptr;
  if (mdl.model != SMCDET_MODEL_M71) return SMCDET_OK;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return set_error(SMCDET_EHIP, "hipGetDevice failed");
  const float key[8] = {m.k1, m.k2, m.k3, m.kb, m.b, m.p0, (float)m.R, 0.f};
  std::lock_guard<std::mutex> lock(g_tab_mu);
  void* base = nullptr;
  if (hipGetSymbolAddress(&base, HIP_SYMBOL(g_psf_tab)) != hipSuccess)
    return set_error(SMCDET_EHIP, "hipGetSymbolAddress(g_psf_tab) failed");
  for (const TabEntry& e : g_tab_entries) {
    if (e.dev != dev) continue;
    if (memcmp(e.key, key, sizeof(key)) == 0) {
      if (e.slot < 0) return SMCDET_OK;  // known not to meet the accuracy bound
      *out = reinterpret_cast<const float4*>(base) + (size_t)e.slot * kTabNodes;
      *inv_h = e.inv_h;
      return SMCDET_OK;
    }
  }
  std::vector<float4> host(kTabNodes);
  TabEntry e{};
  e.dev = dev;
  memcpy(e.key, key, sizeof(key));
  if (!psf_table_build(m, host.data(), &e.inv_h)) {
    e.slot = -1;
    g_tab_entries.push_back(e);
    return SMCDET_OK;
  }
  int slots = 0;
  for (const TabEntry& x : g_tab_entries) slots += (x.dev == dev && x.slot >= 0);
  if (slots >= kTabSlots) {
    // every slot taken (more than kTabSlots PSF parameter sets on this
    // device): this model keeps the exp2/log2 form.  A slot is never reused,
    // so a pointer handed out earlier stays valid for any later launch.
    e.slot = -1;
    g_tab_entries.push_back(e);
    return SMCDET_OK;
  }
  e.slot = slots;
  // the one synchronisation: the first sweep of a PSF parameter set uploads
  // its table and waits for it (so the table's first use cannot sit inside a
  // stream capture; later launches only read the slot)
  if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_psf_tab), host.data(), kTabNodes * sizeof(float4),
                             (size_t)e.slot * kTabNodes * sizeof(float4), hipMemcpyHostToDevice,
                             st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return set_error(SMCDET_EHIP, "PSF table upload failed");
  g_tab_entries.push_back(e);
  *out = reinterpret_cast<const float4*>(base) + (size_t)e.slot * kTabNodes;
  *inv_h = e.inv_h;
  return SMCDET_OK;
}
}  // namespace smcdet
#endif  // SMCDET_DIAG

static int mh_sweep_impl(const smcdet_image_model_t* model, const smcdet_prior_t* prior,
                         const smcdet_mh_t* mh, const float* tiled_image,
                         const float* temperature, int32_t T, int32_t N, int32_t S,
                         const int64_t* ancestors, const float* counts_in,
                         const float* locs_in, const float* fluxes_in, float* counts_out,
                         float* locs_out, float* fluxes_out, const float* rate_in,
                         float* rate_out, uint64_t seed,
                         uint64_t offset, const smcdet_mh_replay_t* replay, uint32_t flags,
                         float* loglik_out, float* acc_rate, int32_t* acc_count,
                         const int32_t* go, const float* tile_boxes,
                         const smcdet_smc_tail_t* tail, void* stream) {

  int rc = validate_model(model, kMaxGlobalPixels);
  if (rc) return rc;
  rc = validate_prior(prior);
  if (rc) return rc;
  if (!mh) return set_error(SMCDET_EINVAL, "mh params are null");
  const bool global_tile = model->H * model->W > kMaxLdsPixels;
  if (global_tile && !rate_out)
    return set_error(SMCDET_EINVAL,
                     "tiles above %d pixels need rate_out [T,N,H*W+64] (the sweep's working "
                     "rate images)", kMaxLdsPixels);
  if (!tiled_image || !temperature || !counts_in || !locs_in || !fluxes_in || !locs_out ||
      !fluxes_out || !acc_rate || !acc_count)
    return set_error(SMCDET_EINVAL, "null buffer");
  if ((uintptr_t)acc_count & 7)
    return set_error(SMCDET_EINVAL, "acc_count must be 8-byte aligned (one uint64 per tile)");
  if (T <= 0 || N <= 0 || T > 65535) return set_error(SMCDET_EUNSUPPORTED, "T=%d N=%d", T, N);
  if (S < 1 || S > 64) return set_error(SMCDET_EUNSUPPORTED, "S=%d outside 1..64", S);
  if (mh->num_iters < 0) return set_error(SMCDET_EINVAL, "num_iters < 0");
  if (ancestors && (locs_in == locs_out || fluxes_in == fluxes_out ||
                    (counts_out && counts_in == counts_out)))
    return set_error(SMCDET_EINVAL, "ancestor gather needs distinct in/out buffers");
  if (ancestors && rate_in && rate_in == rate_out)
    return set_error(SMCDET_EINVAL, "ancestor gather needs distinct rate_in/rate_out buffers");
  if (replay && (!replay->comp || !replay->uloc || !replay->uflux || !replay->uacc))
    return set_error(SMCDET_EINVAL, "incomplete replay buffers");
  if (!(mh->locs_stdev > 0.f) || !(mh->fluxes_stdev > 0.f))
    return set_error(SMCDET_EINVAL, "proposal standard deviations must be > 0");

  MhArgs a{};
  a.m = make_dev_model(*model);
  a.pr = make_dev_prior(*prior);
  a.K = mh->num_iters;
  a.T = T;
  a.N = N;
  a.S = S;
  a.sl = mh->locs_stdev;
  a.isl = 1.0f / mh->locs_stdev;
  a.sf = mh->fluxes_stdev;
  a.isf = 1.0f / mh->fluxes_stdev;
  a.lb_h = mh->locs_min_h;
  a.lb_w = mh->locs_min_w;
  a.ub_h = mh->locs_max_h;
  a.ub_w = mh->locs_max_w;
  a.lb_f = mh->fluxes_min;
  a.ub_f = mh->fluxes_max;
  a.k0 = (uint32_t)seed;
  a.k1 = (uint32_t)(seed >> 32);
  a.offset = offset;
  a.img = tiled_image;
  a.temperature = temperature;
  a.ancestors = ancestors;
  a.counts_in = counts_in;
  a.locs_in = locs_in;
  a.fluxes_in = fluxes_in;
  a.counts_out = counts_out;
  a.locs_out = locs_out;
  a.fluxes_out = fluxes_out;
  a.loglik_out = loglik_out;
  a.rate_in = rate_in;
  a.rate_out = rate_out;
  a.acc_count = acc_count;
  a.acc_rate = acc_rate;
  a.go = go;
  a.boxes = tile_boxes;
  if (replay) {
    a.r_comp = replay->comp;
    a.r_uloc = replay->uloc;
    a.r_uflux = replay->uflux;
    a.r_uacc = replay->uacc;
    a.r_loga = replay->trace_loga;
    a.r_accept = replay->trace_accept;
  }
  hipStream_t st = (hipStream_t)stream;
  const size_t HWp = (size_t)model->H * model->W + kWave;
  size_t lds = global_tile ? 0 :
      ((model->model == SMCDET_MODEL_POISSON ? 2 : 1) * HWp + (size_t)kMhWaves * HWp) *
      sizeof(float);
  const dim3 grid((N + kMhWaves - 1) / kMhWaves, T);
  bool split_tail = false;  // the tile pass as its own launch after the sweep
  TileArgs ta{};
  if (tail) {
    if (!loglik_out) return set_error(SMCDET_EINVAL, "the fused step needs loglik_out");
    if (!tail->temperature_prev || !tail->log_weights_unnorm || !tail->weights || !tail->ess ||
        !tail->log_norm_const)
      return set_error(SMCDET_EINVAL, "null tail buffer");
    if ((tail->idx || tail->bins_out) && tail->resample_method != SMCDET_RESAMPLE_MULTINOMIAL &&
        tail->resample_method != SMCDET_RESAMPLE_SYSTEMATIC)
      return set_error(SMCDET_EINVAL, "unknown resample method %d", tail->resample_method);
    if (tail->resample_u && tail->resample_method != SMCDET_RESAMPLE_SYSTEMATIC)
      return set_error(SMCDET_EINVAL, "resample_u replays systematic resampling only");
    if (tail->bins_out && tail->resample_method != SMCDET_RESAMPLE_SYSTEMATIC)
      return set_error(SMCDET_EINVAL, "bins_out hands over systematic resampling only");
    if (tail->bins_out && tail->idx)
      return set_error(SMCDET_EINVAL, "tail: idx or bins_out, not both");
    if (tail->anc_bins && ancestors)
      return set_error(SMCDET_EINVAL, "ancestors or tail->anc_bins, not both");
    if (tail->anc_bins && (locs_in == locs_out || fluxes_in == fluxes_out ||
                           (counts_out && counts_in == counts_out) ||
                           (rate_in && rate_in == rate_out)))
      return set_error(SMCDET_EINVAL, "ancestor gather needs distinct in/out buffers");
    a.anc_bins = tail->anc_bins;
    ta.flags = kDoTemper | kDoWeights | ((tail->idx || tail->bins_out) ? kDoResample : 0u);
    ta.T = T;
    ta.N = N;
    ta.ess_threshold = tail->ess_threshold;
    ta.loglik = loglik_out;
    ta.temperature = const_cast<float*>(temperature);
    ta.temperature_prev = tail->temperature_prev;
    ta.log_w = tail->log_weights_unnorm;
    ta.weights = tail->weights;
    ta.ess = tail->ess;
    ta.logZ = tail->log_norm_const;
    ta.method = tail->resample_method;
    ta.k0 = (uint32_t)tail->seed;
    ta.k1 = (uint32_t)(tail->seed >> 32);
    ta.offset = tail->offset;
    ta.u = tail->resample_u;
    ta.idx = tail->idx;
    ta.bins_out = tail->bins_out;
    ta.smc_flags = tail->flags & ~SMCDET_SMC_TWO_LAUNCH;
    ta.fin_iter = tail->finished_iter;
    ta.iter = tail->iter;
    if ((uintptr_t)tail->live & 7)
      return set_error(SMCDET_EINVAL, "tail->live must be 8-byte aligned");
    ta.live = tail->live;
    ta.live_host = tail->live ? tail->live_host : nullptr;
    size_t lds_f = 0;
    if (!(tail->flags & SMCDET_SMC_TWO_LAUNCH) && tail_fusable(*model, N, S, flags, &lds_f)) {
      a.tail = ta;
      a.tail.go = nullptr;  // the sweep already returned when *go == 0
      a.has_tail = 1;
      lds = lds_f;
    } else {
      ta.go = go;
      split_tail = true;
    }
  }
  const bool full = (flags & SMCDET_MH_FULL_RECOMPUTE) != 0;
  if (!kDiag && (flags & (SMCDET_MH_ABLATE_LIKELIHOOD | SMCDET_MH_ABLATE_PROPOSAL |
                          SMCDET_MH_SCALAR_SLOTS | SMCDET_MH_PSF_TABLE | SMCDET_MH_NO_RCP_CACHE)))
    return set_error(SMCDET_EUNSUPPORTED,
                     "MH flags 0x%x: diagnostic variants (ablations, scalar slots, PSF table, no "
                     "1/v cache) are in the diagnostic build only (make diag -> "
                     "libsmcdet_hip_diag.so)", flags);
  a.ablate = flags & (SMCDET_MH_ABLATE_LIKELIHOOD | SMCDET_MH_ABLATE_PROPOSAL);
  a.by_count = (flags & SMCDET_MH_COMPONENT_BY_COUNT) != 0;
  a.scalar_slots = (flags & SMCDET_MH_SCALAR_SLOTS) != 0;
  a.skip_done = (flags & SMCDET_MH_SKIP_DONE) != 0;
  a.no_psf_cache = (flags & SMCDET_MH_NO_PSF_CACHE) != 0;
  a.no_rcp_cache = (flags & SMCDET_MH_NO_RCP_CACHE) != 0;
  // the block form for same-anchor M71 steps whose union window takes at least
  // this many 64-pixel slots (SMCDET_MH_BLOCK_SLOTS overrides, for A/Bs)
  a.blk_slots = (flags & SMCDET_MH_NO_BLOCK) ? 0 : 5;
#ifdef SMCDET_DIAG
  // (diagnostic build only: A/B thresholds of scripts/mh_microbench.py; the
  // product never reads the environment on the launch path)
  if (const char* e = getenv("SMCDET_MH_BLOCK_SLOTS")) a.blk_slots = atoi(e);
#endif
  if (kDiag && a.m.model == SMCDET_MODEL_M71 && !full && !global_tile && !a.scalar_slots &&
      (flags & SMCDET_MH_PSF_TABLE)) {
#ifdef SMCDET_DIAG
    rc = psf_table_device(*model, a.m, st, &a.psf_tab, &a.tab_inv_h);
    if (rc) return rc;
#endif
  }
  rc = a.m.model == SMCDET_MODEL_M71
           ? launch_mh<SMCDET_MODEL_M71>(a, replay != nullptr, full, grid, lds, st)
           : launch_mh<SMCDET_MODEL_POISSON>(a, replay != nullptr, full, grid, lds, st);
  if (rc) return rc;
  rc = check_launch("smcdet_mh_sweep");
  if (rc || !split_tail) return rc;
  // the tile pass on the sweep's log-likelihoods (tile.h tile_work: the same
  // work as smcdet_temper_reweight, replayed offsets and bins included)
  return launch_tile(ta, st);
}

extern "C" int smcdet_mh_sweep(const smcdet_image_model_t* model, const smcdet_prior_t* prior,
                               const smcdet_mh_t* mh, const float* tiled_image,
                               const float* temperature, int32_t T, int32_t N, int32_t S,
                               const int64_t* ancestors, const float* counts_in,
                               const float* locs_in, const float* fluxes_in, float* counts_out,
                               float* locs_out, float* fluxes_out, const float* rate_in,
                               float* rate_out, uint64_t seed,
                               uint64_t offset, const smcdet_mh_replay_t* replay, uint32_t flags,
                               float* loglik_out, float* acc_rate, int32_t* acc_count,
                               const int32_t* go, const float* tile_boxes, void* stream) {
  return mh_sweep_impl(model, prior, mh, tiled_image, temperature, T, N, S, ancestors, counts_in,
                       locs_in, fluxes_in, counts_out, locs_out, fluxes_out, rate_in, rate_out,
                       seed, offset, replay, flags, loglik_out, acc_rate, acc_count, go,
                       tile_boxes, nullptr, stream);
}

extern "C" int smcdet_mh_sweep_step(const smcdet_image_model_t* model,
                                    const smcdet_prior_t* prior, const smcdet_mh_t* mh,
                                    const float* tiled_image, float* temperature, int32_t T,
                                    int32_t N, int32_t S, const int64_t* ancestors,
                                    const float* counts_in, const float* locs_in,
                                    const float* fluxes_in, float* counts_out, float* locs_out,
                                    float* fluxes_out, const float* rate_in, float* rate_out,
                                    uint64_t seed, uint64_t offset,
                                    const smcdet_mh_replay_t* replay, uint32_t flags,
                                    float* loglik_out, float* acc_rate, int32_t* acc_count,
                                    const int32_t* go, const float* tile_boxes,
                                    const smcdet_smc_tail_t* tail, void* stream) {
  if (!tail) return set_error(SMCDET_EINVAL, "tail is null");
  return mh_sweep_impl(model, prior, mh, tiled_image, temperature, T, N, S, ancestors, counts_in,
                       locs_in, fluxes_in, counts_out, locs_out, fluxes_out, rate_in, rate_out,
                       seed, offset, replay, flags, loglik_out, acc_rate, acc_count, go,
                       tile_boxes, tail, stream);
}

extern "C" int smcdet_mh_sweep_step_fused(const smcdet_image_model_t* model, int32_t N, int32_t S,
                                          uint32_t flags) {
  if (!model) return 0;
  return tail_fusable(*model, N, S, flags, nullptr) ? 1 : 0;
}
