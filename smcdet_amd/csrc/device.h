// device.h — shared device-side helpers for the smcdet MI355X (gfx950) kernels:
// Philox4x32-10 counter-based RNG, 64-lane wave reductions, the two PSF
// profiles and the two per-pixel log-likelihoods of the reference's image
// models (timwhite0/smcdet smcdet/images.py).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

#include "../../include/smcdet_hip.h"

namespace smcdet {

constexpr int kWave = 64;

// Phase timestamps for profiling builds only (make trace -> -DSMCDET_TRACE):
// lane 0 of a traced wave stores s_memtime into a per-file device table that
// smcdet_trace_read_<file>() copies out.  Compiled out of the product library.
constexpr int kTraceRows = 256, kTraceCols = 16;
#ifdef SMCDET_TRACE
#define SMCDET_TRACE_TABLE static __device__ unsigned long long g_trace[kTraceRows * kTraceCols];
#define SMC_TRACE(row, col)                                                           \
  do {                                                                                \
    const int r_ = (row);                                                             \
    if (r_ >= 0 && r_ < kTraceRows && (threadIdx.x & 63) == 0)                        \
      g_trace[r_ * kTraceCols + (col)] = __builtin_amdgcn_s_memtime();                \
  } while (0)
// per-wave lifetime record: realtime start/end (100 MHz), memtime start/end, HW_ID
constexpr int kTraceWaves = 8192;
#define SMCDET_WAVE_TABLE static __device__ unsigned long long g_wave[kTraceWaves * 8];
#define SMC_WAVE_MARK(idx, col)                                                       \
  do {                                                                                \
    const int i_ = (idx);                                                             \
    if (i_ >= 0 && i_ < kTraceWaves && (threadIdx.x & 63) == 0) {                     \
      g_wave[i_ * 8 + (col)] = __builtin_amdgcn_s_memrealtime();                      \
      g_wave[i_ * 8 + 2 + (col)] = __builtin_amdgcn_s_memtime();                      \
      if ((col) == 0) {                                                               \
        g_wave[i_ * 8 + 4] = __builtin_amdgcn_s_getreg(0xF804);                      \
        g_wave[i_ * 8 + 7] = __builtin_amdgcn_s_getreg(0x7814);                      \
      }                                                                               \
    }                                                                                 \
  } while (0)
#define SMC_WAVE_STAT(idx, col, v)                                                    \
  do {                                                                                \
    const int i_ = (idx);                                                             \
    if (i_ >= 0 && i_ < kTraceWaves && (threadIdx.x & 63) == 0)                       \
      g_wave[i_ * 8 + (col)] = (unsigned long long)(v);                               \
  } while (0)
#define SMCDET_WAVE_READER(name)                                                      \
  extern "C" int name(unsigned long long* host, int n) {                             \
    if (n > kTraceWaves * 8) n = kTraceWaves * 8;                                     \
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wave), n * sizeof(unsigned long long)) \
                   == hipSuccess ? 0 : -3;                                            \
  }
#define SMCDET_TRACE_READER(name)                                                     \
  extern "C" int name(unsigned long long* host, int n) {                             \
    if (n > kTraceRows * kTraceCols) n = kTraceRows * kTraceCols;                     \
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_trace), n * sizeof(unsigned long long)) \
                   == hipSuccess ? 0 : -3;                                            \
  }
#else
#define SMCDET_TRACE_TABLE
#define SMCDET_WAVE_TABLE
#define SMC_WAVE_MARK(idx, col) \
  do {                          \
  } while (0)
#define SMC_WAVE_STAT(idx, col, v) \
  do {                             \
  } while (0)
#define SMCDET_WAVE_READER(name)
#define SMC_TRACE(row, col) \
  do {                      \
  } while (0)
#define SMCDET_TRACE_READER(name)
#endif
constexpr float kHalfLog2Pi = 0.91893853320467274178f;  // 0.5*log(2*pi)
constexpr float kLn2 = 0.69314718055994530942f;
constexpr float kLog2e = 1.44269504088896340736f;
constexpr float kSqrt2 = 1.41421356237309504880f;
constexpr float kSqrt1_2 = 0.70710678118654752440f;

// ---------------------------------------------------------------------------
// host-side error reporting (defined in common.hip)
// ---------------------------------------------------------------------------
int set_error(int code, const char* fmt, ...);
int check_launch(const char* what);
// raises the kernel's dynamic-LDS limit when bytes > 64 KiB (<= 160 KiB)
int ensure_lds(const void* kernel, size_t bytes);
// launch timing (smcdet_launch_timing): the next start / stop event pair of
// the pool, or false (nulls) when timing is off or the pool is used up
bool timing_next(hipEvent_t* start, hipEvent_t* stop);
// the per-tile passes are timed too (smcdet_launch_timing_tiles) and the pool
// has room
bool timing_tiles();
// A sweep launch whose timing events (if any) ride on its own dispatch packet
// (hipExtLaunchKernel): no marker packet between kernels, so timing does not
// open a launch bubble in the step it measures.
template <typename... Args, typename F = void (*)(Args...)>
inline void launch_sweep(F kernel, dim3 grid, dim3 block, size_t lds, hipStream_t st,
                         Args... args) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  timing_next(&e0, &e1);
  hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)lds, st, e0, e1, 0u, args...);
}

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. 2011) — counter (c0..c3), key (k0,k1)
// ---------------------------------------------------------------------------
struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox4x32(uint32_t c0, uint32_t c1, uint32_t c2,
                                          uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c0;
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2);
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return U4{c0, c1, c2, c3};
}

// [0,1) with 24 random mantissa bits, like torch.rand for float32
__device__ __forceinline__ float u01(uint32_t x) {
  return (float)(x >> 8) * 5.9604644775390625e-08f;
}

// stream tags keep the counter spaces of different draws disjoint
enum RngTag : uint32_t {
  kTagMH0 = 0x4d480000u,
  kTagMH1 = 0x4d480001u,
  kTagPriorLoc = 0x50520000u,
  kTagPriorFlux = 0x50520001u,
  kTagResample = 0x52530000u,
  kTagNoise = 0x4e530000u,
  kTagStrata = 0x43530000u,
  kTagMALA0 = 0x4d4c0000u,
  kTagMALA1 = 0x4d4c0001u,
  kTagChain0 = 0x43480000u,
  kTagChain1 = 0x43480001u,
  kTagAgg0 = 0x41470000u,
  kTagAgg1 = 0x41470001u,
  kTagAggResample = 0x41520000u,
};

// ---------------------------------------------------------------------------
// wave helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float readlane(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ int readlane(int v, int lane) {
  return __builtin_amdgcn_readlane(v, lane);
}
// v with lane `lane` replaced by the wave-uniform x
__device__ __forceinline__ float writelane(float x, int lane, float v) {
  return (int)(threadIdx.x & 63) == lane ? x : v;
}

// 64-lane reductions on DPP (no LDS crossbar round trips): quad_perm
// [1,0,3,2], [2,3,0,1], row_shr:4, row_shr:8 leave each row's sum in its lane
// 15; row_bcast:15 and row_bcast:31 fold the rows into lane 63, which is
// broadcast with v_readlane.  Call from converged code.  The two broadcast
// steps write every row (bound_ctrl: rows without a source add 0): lane 63
// gets the same (R3 + R2) + (R1 + R0) as with the rows 1,3 / 2,3 masks, and
// the compiler fuses each step into one v_add_f32_dpp (the masked form needs
// a zeroed `old` register and a separate v_mov_b32_dpp).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int dpp_move(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xf, false);
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(dpp_move<CTRL, ROW_MASK>(__float_as_int(v)));
}
template <int CTRL>
__device__ __forceinline__ float dpp_f_bc(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, true));
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = dpp_move<CTRL, ROW_MASK>((int)(b & 0xffffffffll));
  const int hi = dpp_move<CTRL, ROW_MASK>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xb1>(v);
  v += dpp_f<0x4e>(v);
  v += dpp_f<0x114>(v);
  v += dpp_f<0x118>(v);
  v += dpp_f_bc<0x142>(v);
  v += dpp_f_bc<0x143>(v);
  return readlane(v, 63);
}
// two independent wave sums, step by step interleaved (each value gets
// wave_sum's exact operation sequence; the two DPP chains hide each other's
// latency on the tile pass's latency-bound path)
__device__ __forceinline__ void wave_sum2(float& a, float& b) {
  a += dpp_f<0xb1>(a);
  b += dpp_f<0xb1>(b);
  a += dpp_f<0x4e>(a);
  b += dpp_f<0x4e>(b);
  a += dpp_f<0x114>(a);
  b += dpp_f<0x114>(b);
  a += dpp_f<0x118>(a);
  b += dpp_f<0x118>(b);
  a += dpp_f_bc<0x142>(a);
  b += dpp_f_bc<0x142>(b);
  a += dpp_f_bc<0x143>(a);
  b += dpp_f_bc<0x143>(b);
  a = readlane(a, 63);
  b = readlane(b, 63);
}
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_d<0xb1>(v);
  v += dpp_d<0x4e>(v);
  v += dpp_d<0x114>(v);
  v += dpp_d<0x118>(v);
  v += dpp_d<0x142, 0xa>(v);
  v += dpp_d<0x143, 0xc>(v);
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), 63);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// max: out-of-row sources read the identity, so use -inf as `old`
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_fmax(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(-INFINITY), __float_as_int(v),
                                                    CTRL, ROW_MASK, 0xf, false));
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_fmax<0xb1>(v));
  v = fmaxf(v, dpp_fmax<0x4e>(v));
  v = fmaxf(v, dpp_fmax<0x114>(v));
  v = fmaxf(v, dpp_fmax<0x118>(v));
  v = fmaxf(v, dpp_fmax<0x142, 0xa>(v));
  v = fmaxf(v, dpp_fmax<0x143, 0xc>(v));
  return readlane(v, 63);
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fast_log2(float x) { return __builtin_amdgcn_logf(x); }
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// torch.nan_to_num(x) defaults: nan -> 0, +inf -> FLT_MAX, -inf -> -FLT_MAX
__device__ __forceinline__ float nan_to_num(float x, float nan_val) {
  if (x != x) return nan_val;
  if (isinf(x)) return x > 0.f ? 3.402823466e+38f : -3.402823466e+38f;
  return x;
}

// ---------------------------------------------------------------------------
// image model, pre-digested for the device
// ---------------------------------------------------------------------------
struct DevModel {
  int model, H, W, R;
  float bg;     // background
  float g;      // flux -> ADU scale (adu_per_nmgy; 1 for Poisson)
  // M71: psf(r2) = (exp2(k1 r2) + b exp2(k2 r2) + p0 exp2(kb log2(1 + k3 r2))) * inv_norm
  float k1, k2, b, k3, kb, p0, inv_norm;
  float lb2, lp02;  // log2(b), log2(p0): b and p0 folded into the exponents (mcmc.h)
  // Poisson (basic) model: psf(r2) = amp * exp2(kg r2)
  float kg, amp;
  // M71 noise: var = s0sq + eta * rate
  float s0sq, eta;
};

DevModel make_dev_model(const smcdet_image_model_t& m);  // common.hip
// tiles whose image and per-wave rate images fit LDS; larger tiles (up to
// kMaxGlobalPixels) run the global-memory paths (M71 model: smcdet_loglik,
// smcdet_render, smcdet_mh_sweep)
constexpr int kMaxLdsPixels = 4096;
constexpr int kMaxGlobalPixels = 65536;
int validate_model(const smcdet_image_model_t* m, int max_pixels = kMaxLdsPixels);  // common.hip

// M71ImageModel._compute_normalized_psf (images.py:137-145) / the basic
// model's Normal(0, sigma).log_prob(r).exp() (images.py:17, 25-26)
// psf_raw * psf_scale = the normalised profile
template <int MODEL>
__device__ __forceinline__ float psf_raw(const DevModel& m, float r2) {
  if constexpr (MODEL == SMCDET_MODEL_M71) {
    const float t1 = fast_exp2(m.k1 * r2);
    const float e2 = fast_exp2(m.k2 * r2);
    const float e3 = fast_exp2(m.kb * fast_log2(fmaf(m.k3, r2, 1.0f)));
    return fmaf(m.p0, e3, fmaf(m.b, e2, t1));
  } else {
    return fast_exp2(m.kg * r2);
  }
}
template <int MODEL>
__device__ __forceinline__ float psf_scale(const DevModel& m) {
  return MODEL == SMCDET_MODEL_M71 ? m.inv_norm : m.amp;
}
template <int MODEL>
__device__ __forceinline__ float psf_eval(const DevModel& m, float r2) {
  return psf_raw<MODEL>(m, r2) * psf_scale<MODEL>(m);
}

// per-pixel log-likelihood: M71 Normal(rate, sqrt(s0^2 + eta*rate)).log_prob(x)
// (images.py:169-175); basic Poisson(rate).log_prob(x), Normal(rate, sqrt(rate))
// where rate > 5e4 (images.py:91-102).  lgx = lgamma(x + 1).
template <int MODEL>
__device__ __forceinline__ float pix_loglik(const DevModel& m, float x, float lgx, float rate) {
  const float d = x - rate;
  if constexpr (MODEL == SMCDET_MODEL_M71) {
    const float v = fmaf(m.eta, rate, m.s0sq);
    return fmaf(-0.5f * d * d, fast_rcp(v), -0.5f * kLn2 * fast_log2(v) - kHalfLog2Pi);
  } else {
    const float lr = kLn2 * fast_log2(rate);
    if (rate > 50000.0f) return fmaf(-0.5f * d * d, fast_rcp(rate), -0.5f * lr - kHalfLog2Pi);
    return fmaf(x, lr, -rate) - lgx;
  }
}

// log(1 + a), accurate for small |a|: log(u) - ((u - 1) - a)/u, u = fl(1 + a)
__device__ __forceinline__ float log1p_fast(float a) {
  const float u = 1.0f + a;
  return fmaf(-((u - 1.0f) - a), fast_rcp(u), kLn2 * fast_log2(u));
}

// per-pixel log-likelihood CHANGE when the rate moves lam -> lam + dl.
// M71: 0.5 (d0^2/v0 - d1^2/v1) - 0.5 log(v1/v0), d = x - lam, v = s0^2 + eta*lam
// (images.py:169-175 differenced): the log of the ratio, not a difference of
// logs, and both quadratic terms are O(1) for pixels near the data, so the
// absolute error per pixel is a few float32 ulps of O(1) (~1e-7), summing to
// ~1e-6 nats over a window, orders below the MH decision margins and the
// reference's own float32 rounding of full 1,024-pixel sums.
// Poisson: x*log1p(dl/lam) - dl.
template <int MODEL>
__device__ __forceinline__ float pix_delta(const DevModel& m, float x, float lgx, float lam,
                                           float dl) {
  if constexpr (MODEL == SMCDET_MODEL_M71) {
    const float l1 = lam + dl;
    const float v0 = fmaf(m.eta, lam, m.s0sq), v1 = fmaf(m.eta, l1, m.s0sq);
    const float r0 = fast_rcp(v0), r1 = fast_rcp(v1);
    const float d0 = x - lam, d1 = x - l1;
    const float t = fmaf(d0 * d0, r0, -(d1 * d1) * r1);
    return fmaf(0.5f, t, (-0.5f * kLn2) * fast_log2(v1 * r0));
  } else {
    const float lnew = lam + dl;
    if (lam > 50000.0f || lnew > 50000.0f)
      return pix_loglik<MODEL>(m, x, lgx, lnew) - pix_loglik<MODEL>(m, x, lgx, lam);
    const float a = dl * fast_rcp(lam);
    const float u = 1.0f + a;
    const float l1p = fmaf(-((u - 1.0f) - a), fast_rcp(u), kLn2 * fast_log2(u));
    return fmaf(x, l1p, -dl);
  }
}

// ---------------------------------------------------------------------------
// two-wide float vectors: elementwise arithmetic compiles to gfx950's packed
// v_pk_{fma,mul,add}_f32 (one 6-cycle issue for two lanes' worth of work vs
// two 4-cycle scalar issues, measured in scripts/probe/isa_probe.hip)
// ---------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 fma2(f2 a, float b, f2 c) { return fma2(a, f2{b, b}, c); }
__device__ __forceinline__ f2 fma2(f2 a, float b, float c) { return fma2(a, f2{b, b}, f2{c, c}); }
__device__ __forceinline__ f2 exp2_2(f2 x) { return f2{fast_exp2(x.x), fast_exp2(x.y)}; }
__device__ __forceinline__ f2 log2_2(f2 x) { return f2{fast_log2(x.x), fast_log2(x.y)}; }
__device__ __forceinline__ f2 rcp2(f2 x) { return f2{fast_rcp(x.x), fast_rcp(x.y)}; }

template <int MODEL>
__device__ __forceinline__ f2 psf_raw2(const DevModel& m, f2 r2) {
  if constexpr (MODEL == SMCDET_MODEL_M71) {
    // b and p0 as multipliers (b e2 + t1, then p0 e3 + that): every packed
    // op then has one scalar operand (VOP3P reads one SGPR; a second one
    // would be copied into a VGPR pair each iteration)
    const f2 t1 = exp2_2(m.k1 * r2);
    const f2 e2 = exp2_2(m.k2 * r2);
    const f2 e3 = exp2_2(m.kb * log2_2(fma2(r2, m.k3, 1.0f)));
    return fma2(e3, m.p0, fma2(e2, m.b, t1));
  } else {
    return exp2_2(m.kg * r2);
  }
}

// ---------------------------------------------------------------------------
// M71 PSF as a radial table in LDS (the MH sweep's union-window deltas): the
// raw profile psi(r^2) of psf_raw (images.py:137-141) as one cubic per node
// of a uniform grid in r^2, node i centred at r^2 = i*h, t = r^2/h - i in
// [-1/2, 1/2] (round to nearest).  The coefficients are fitted on the host in
// double precision (psf_table_build, mh_kernel.hip) and stored as float4
// (c0, c1, c2, c3); psi = c0 + t(c1 + t(c2 + t c3)).  One ds_read_b128 and
// four VALU replace 3 exp2 + 1 log2 per evaluation; the fit error is below
// float32 rounding (max relative error 3.0e-7, mean 9e-8, against 7.5e-7 /
// 1.6e-7 for the float32 exp2/log2 form).  Opt-in (SMCDET_MH_PSF_TABLE): the
// lanes' scattered b128 reads made the 32x32 sweep 50% slower.
// The index comes from the float32 round-to-nearest trick: y = u + 1.5*2^23
// holds round(u) in its low mantissa bits (u < 2^22), y - 1.5*2^23 is that
// integer exactly, so t is exact too.  The index is clamped to the last node
// in every use: positions outside the source's window (union windows of moved
// anchors, masked lanes' dummy positions) have their value discarded, but the
// LDS address must stay inside the table.
// ---------------------------------------------------------------------------
constexpr int kTabIntervals = 512;
constexpr int kTabNodes = kTabIntervals + 1;
constexpr float kRoundMagic = 12582912.0f;  // 1.5 * 2^23
constexpr int kRoundMagicBits = 0x4B400000;

__device__ __forceinline__ float psf_tab(const float4* tab, float inv_h, float r2) {
  const float u = r2 * inv_h;
  const float y = u + kRoundMagic;
  const float t = u - (y - kRoundMagic);
  const int i = min(__float_as_int(y) - kRoundMagicBits, kTabIntervals);
  const float4 c = tab[i];
  return fmaf(fmaf(fmaf(c.w, t, c.z), t, c.y), t, c.x);
}
__device__ __forceinline__ f2 psf_tab2(const float4* tab, float inv_h, f2 r2) {
  const f2 u = r2 * inv_h;
  const f2 y = u + kRoundMagic;
  const f2 t = u - (y - kRoundMagic);
  const int i0 = min(__float_as_int(y.x) - kRoundMagicBits, kTabIntervals);
  const int i1 = min(__float_as_int(y.y) - kRoundMagicBits, kTabIntervals);
  const float4 c0 = tab[i0], c1 = tab[i1];
  return f2{fmaf(fmaf(fmaf(c0.w, t.x, c0.z), t.x, c0.y), t.x, c0.x),
            fmaf(fmaf(fmaf(c1.w, t.y, c1.z), t.y, c1.y), t.y, c1.x)};
}

template <int MODEL>
__device__ __forceinline__ f2 pix_delta2(const DevModel& m, f2 x, f2 lgx, f2 lam, f2 dl) {
  if constexpr (MODEL == SMCDET_MODEL_M71) {
    const f2 l1 = lam + dl;
    const f2 v0 = fma2(lam, m.eta, m.s0sq), v1 = fma2(l1, m.eta, m.s0sq);
    const f2 r0 = rcp2(v0), r1 = rcp2(v1);
    const f2 d0 = x - lam, d1 = x - l1;
    const f2 t = fma2(d0 * d0, r0, -(d1 * d1) * r1);
    return fma2(t, 0.5f, (-0.5f * kLn2) * log2_2(v1 * r0));
  } else {
    return f2{pix_delta<MODEL>(m, x.x, lgx.x, lam.x, dl.x),
              pix_delta<MODEL>(m, x.y, lgx.y, lam.y, dl.y)};
  }
}

__device__ __forceinline__ float fast_exp(float x) { return fast_exp2(x * kLog2e); }
__device__ __forceinline__ float fast_log(float x) { return kLn2 * fast_log2(x); }

// erfc(|x|) with fractional error < 1.2e-7 everywhere (Numerical Recipes'
// Chebyshev fit), branch-free
__device__ __forceinline__ float erfc_abs(float x) {
  const float z = fabsf(x);
  const float t = fast_rcp(fmaf(0.5f, z, 1.0f));
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  return t * fast_exp(fmaf(-z, z, p));
}

// Normal(mu, sigma).cdf(v) = 0.5 erfc(-(v-mu)/(sigma sqrt2)); accurate in both
// tails (the reference's 0.5(1+erf) form has only absolute accuracy there)
__device__ __forceinline__ float normal_cdf(float v, float mu, float inv_sigma) {
  const float u = (v - mu) * inv_sigma * kSqrt1_2;
  const float e = 0.5f * erfc_abs(u);
  return u < 0.f ? e : 1.0f - e;
}

// inverse error function (Giles 2010, single precision, |rel err| < 4e-7),
// both branches evaluated (branch-free across the lanes that call it)
__device__ __forceinline__ float erfinv_fast(float x) {
  float w = -fast_log((1.0f - x) * (1.0f + x));
  const float wa = w - 2.5f;
  float pa = 2.81022636e-08f;
  pa = fmaf(pa, wa, 3.43273939e-07f);
  pa = fmaf(pa, wa, -3.5233877e-06f);
  pa = fmaf(pa, wa, -4.39150654e-06f);
  pa = fmaf(pa, wa, 0.00021858087f);
  pa = fmaf(pa, wa, -0.00125372503f);
  pa = fmaf(pa, wa, -0.00417768164f);
  pa = fmaf(pa, wa, 0.246640727f);
  pa = fmaf(pa, wa, 1.50140941f);
  const float wb = __builtin_amdgcn_sqrtf(w) - 3.0f;
  float pb = -0.000200214257f;
  pb = fmaf(pb, wb, 0.000100950558f);
  pb = fmaf(pb, wb, 0.00134934322f);
  pb = fmaf(pb, wb, -0.00367342844f);
  pb = fmaf(pb, wb, 0.00573950773f);
  pb = fmaf(pb, wb, -0.0076224613f);
  pb = fmaf(pb, wb, 0.00943887047f);
  pb = fmaf(pb, wb, 1.00167406f);
  pb = fmaf(pb, wb, 2.83297682f);
  return (w < 5.0f ? pa : pb) * x;
}

struct DevPrior {
  int kind;
  float lo, hi_h, hi_w;      // location box: [lo, hi_h) x [lo_w, hi_w)
  float lo_w;
  float count_c0, count_c1;  // M71: log(mu), mu ; PARETO: log(1/k), unused
  int min_objects, max_objects;
  float flux_c;              // log-normaliser of the flux density
  float ap1;                 // alpha + 1
  float alpha, lower, upper;
  float loc_lp_h, loc_lp_w;  // -log(high - low) per coordinate
};

DevPrior make_dev_prior(const smcdet_prior_t& p);  // common.hip
int validate_prior(const smcdet_prior_t* p);        // common.hip

// A tile's own location box (lo_h, lo_w, hi_h, hi_w) in place of the
// prior's [-pad, H+pad) x [-pad, W+pad): the uniform densities follow the
// box, and a Poisson count mean scales with its area (M71: the mean is
// counts_rate times the padded tile area, prior.py:91-97)
__device__ __forceinline__ void tile_box_prior(DevPrior& pr, const float* b) {
  const float area0 = (pr.hi_h - pr.lo) * (pr.hi_w - pr.lo_w);
  pr.lo = b[0];
  pr.lo_w = b[1];
  pr.hi_h = b[2];
  pr.hi_w = b[3];
  pr.loc_lp_h = -logf(pr.hi_h - pr.lo);
  pr.loc_lp_w = -logf(pr.hi_w - pr.lo_w);
  if (pr.kind == SMCDET_PRIOR_M71) {
    pr.count_c1 = pr.count_c1 * ((pr.hi_h - pr.lo) * (pr.hi_w - pr.lo_w) / area0);
    pr.count_c0 = logf(pr.count_c1);
  }
}

// ---------------------------------------------------------------------------
// LDS image staging: x and (Poisson) lgamma(x+1) for one tile
// ---------------------------------------------------------------------------
template <int MODEL>
__device__ __forceinline__ void stage_image(const float* __restrict__ img, float* xs, float* lg,
                                            int HW, int tid, int nthreads) {
  for (int p = tid; p < HW; p += nthreads) {
    const float x = img[p];
    xs[p] = x;
    if constexpr (MODEL == SMCDET_MODEL_POISSON) lg[p] = lgammaf(x + 1.0f);
  }
}

}  // namespace smcdet
