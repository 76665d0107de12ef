// mcmc.h — helpers shared by the MALA sweep (mala_kernel.hip) and the MH
// chain sampler (chain_kernel.hip): one source's clipped PSF window, the PSF
// derivative, d loglik / d rate, and the truncated normal of
// smcdet/distributions.py:22-52 in torch's float32 operation order.
#pragma once

#include <math.h>

#include "render.h"

namespace smcdet {

// psf_raw and its derivative with respect to r^2 (psf_raw * psf_scale is the
// normalised profile, device.h)
template <int MODEL>
__device__ __forceinline__ float psf_raw_d(const DevModel& m, float r2, float& dpsi) {
  if constexpr (MODEL == SMCDET_MODEL_M71) {
    const float t1 = fast_exp2(m.k1 * r2);
    const float t2 = fast_exp2(fmaf(m.k2, r2, m.lb2));
    const float u = fmaf(m.k3, r2, 1.0f);
    const float t3 = fast_exp2(fmaf(m.kb, fast_log2(u), m.lp02));
    dpsi = fmaf(kLn2, fmaf(m.k1, t1, m.k2 * t2), (m.kb * m.k3) * t3 * fast_rcp(u));
    return t1 + t2 + t3;
  } else {
    const float p = fast_exp2(m.kg * r2);
    dpsi = (kLn2 * m.kg) * p;
    return p;
  }
}

// d (per-pixel log-likelihood) / d rate (images.py:169-175 / :91-102)
template <int MODEL>
__device__ __forceinline__ float dll_drate(const DevModel& m, float x, float lam) {
  const float d = x - lam;
  if constexpr (MODEL == SMCDET_MODEL_M71) {
    const float r = fast_rcp(fmaf(m.eta, lam, m.s0sq));
    return r * fmaf(0.5f * m.eta, fmaf(d * d, r, -1.0f), d);
  } else {
    const float r = fast_rcp(lam);
    if (lam > 50000.0f) return r * fmaf(0.5f, fmaf(d * d, r, -1.0f), d);
    return fmaf(x, r, -1.0f);
  }
}

// ---- truncated normal in torch's float32 operation order -------------------
// Normal(mu, sigma).cdf(v) = 0.5 * (1 + erf((v - mu) * (1/sigma) / sqrt2))
__device__ __forceinline__ float t_cdf(float v, float mu, float rsig) {
#pragma clang fp contract(off)
  return 0.5f * (1.0f + erff(__fdiv_rn((v - mu) * rsig, 1.41421356237309504880f)));
}
// log_prob_in_box = nan_to_num(log(cdf(ub) - cdf(lb))) (distributions.py:33-35)
__device__ __forceinline__ float t_logZ(float mu, float rsig, float lb, float ub) {
#pragma clang fp contract(off)
  return nan_to_num(logf(t_cdf(ub, mu, rsig) - t_cdf(lb, mu, rsig)), 0.0f);
}
// TruncatedDiagonalMVN.sample (distributions.py:40-48)
__device__ __forceinline__ float t_sample(float mu, float sig, float rsig, float lb, float ub,
                                          float u) {
#pragma clang fp contract(off)
  const float lo = 1e-6f, hi = (float)(1.0 - 1e-6);
  const float p = fminf(fmaxf(u, lo), hi);
  float pt = t_cdf(lb, mu, rsig) + p * expf(t_logZ(mu, rsig, lb, ub));
  pt = fminf(fmaxf(pt, lo), hi);
  const float x = mu + sig * erfinv_fast(2.0f * pt - 1.0f) * kSqrt2;
  return fminf(fmaxf(x, lb), ub);
}
// TruncatedDiagonalMVN.log_prob (distributions.py:50-52): Normal.log_prob - log Z
__device__ __forceinline__ float t_logprob(float v, float mu, float sig, float rsig, float lb,
                                           float ub) {
#pragma clang fp contract(off)
  const float d = v - mu;
  const float lp = -(d * d) / (2.0f * (sig * sig)) - logf(sig) - kHalfLog2Pi;
  return lp - t_logZ(mu, rsig, lb, ub);
}

// The three proposal dimensions run in lanes d = lane % 3 (lanes 3..5 and up
// replicate 0..2).  A dimension's two Normal.cdf evaluations (box bounds lb and
// ub) run in two lanes at once -- lane d takes lb, lane d+3 takes ub -- and are
// exchanged with a lane permute: one erf per wave instruction stream instead
// of two, with the same values as t_logZ.
struct TnBox {
  float cdf_lb, logZ;  // Normal(mu, sigma).cdf(lb) and log_prob_in_box
};
__device__ __forceinline__ TnBox t_box_lanes(float mu, float rsig, float lb, float ub, int lane) {
#pragma clang fp contract(off)
  const float v = (lane >= 3 && lane < 6) ? ub : lb;
  const float c = t_cdf(v, mu, rsig);
  const int d = lane % 3;
  TnBox b;
  b.cdf_lb = __shfl(c, d, kWave);
  b.logZ = nan_to_num(logf(__shfl(c, d + 3, kWave) - b.cdf_lb), 0.0f);
  return b;
}
// The same for proposal groups of 6 lanes (lane r of a group: r < 3 -> lb,
// r >= 3 -> ub of dimension r % 3): src = the group's lane of dimension d with
// r < 3.  Same arithmetic as t_box_lanes.
__device__ __forceinline__ TnBox t_box_group(float mu, float rsig, float lb, float ub, int r,
                                             int src) {
#pragma clang fp contract(off)
  const float v = r >= 3 ? ub : lb;
  const float c = t_cdf(v, mu, rsig);
  TnBox b;
  b.cdf_lb = __shfl(c, src, kWave);
  b.logZ = nan_to_num(logf(__shfl(c, src + 3, kWave) - b.cdf_lb), 0.0f);
  return b;
}
// t_sample / t_logprob with the box quantities of t_box_lanes
__device__ __forceinline__ float t_sample_box(float mu, float sig, float lb, float ub, float u,
                                              const TnBox& b) {
#pragma clang fp contract(off)
  const float lo = 1e-6f, hi = (float)(1.0 - 1e-6);
  const float p = fminf(fmaxf(u, lo), hi);
  float pt = b.cdf_lb + p * expf(b.logZ);
  pt = fminf(fmaxf(pt, lo), hi);
  const float x = mu + sig * erfinv_fast(2.0f * pt - 1.0f) * kSqrt2;
  return fminf(fmaxf(x, lb), ub);
}
__device__ __forceinline__ float t_logprob_box(float v, float mu, float sig, const TnBox& b) {
#pragma clang fp contract(off)
  const float d = v - mu;
  const float lp = -(d * d) / (2.0f * (sig * sig)) - logf(sig) - kHalfLog2Pi;
  return lp - b.logZ;
}

// clipped (2R+1)^2 window anchored at floor(h, w)
struct Window {
  int fh, fw;       // anchors
  int r0, c0, bw;   // first row / column, width
  int npos;         // positions (0 when the window misses the tile)
  float inv_bw;
};
__device__ __forceinline__ Window window_of(const DevModel& m, float h, float w) {
  Window q;
  q.fh = ifloor_clamped(h);
  q.fw = ifloor_clamped(w);
  q.r0 = max(q.fh - m.R, 0);
  q.c0 = max(q.fw - m.R, 0);
  const int r1 = min(q.fh + m.R, m.H - 1), c1 = min(q.fw + m.R, m.W - 1);
  q.bw = max(c1 - q.c0 + 1, 1);
  q.npos = (r1 >= q.r0 && c1 >= q.c0) ? (r1 - q.r0 + 1) * (c1 - q.c0 + 1) : 0;
  // v_rcp_f32 (1 ulp) instead of an IEEE division on the chain's critical path:
  // window_pos's floor((i + 0.5) / bw) stays exact, since (i + 0.5) / bw is at
  // least 0.5 / bw from an integer and the rcp error is ~1e-7 relative
  q.inv_bw = __builtin_amdgcn_rcpf((float)q.bw);
  return q;
}
__device__ __forceinline__ void window_pos(const Window& q, int i, int& ph, int& pw) {
  const int aa = (int)(((float)i + 0.5f) * q.inv_bw);
  ph = q.r0 + aa;
  pw = q.c0 + (i - aa * q.bw);
}
__device__ __forceinline__ bool in_window(const DevModel& m, int fh, int fw, int ph, int pw) {
  const unsigned span = 2u * (unsigned)m.R;
  return (unsigned)(ph - fh + m.R) <= span && (unsigned)(pw - fw + m.R) <= span;
}
// true if window qo has positions outside window qn: false when qo's clipped
// box lies inside qn's (unclipped) window -- same anchors, or both windows
// covering a small tile -- so the old-only walks can be skipped
__device__ __forceinline__ bool has_old_only(const DevModel& m, const Window& qo,
                                             const Window& qn) {
  return qo.npos > 0 &&
         !(qo.r0 >= qn.fh - m.R && min(qo.fh + m.R, m.H - 1) <= qn.fh + m.R &&
           qo.c0 >= qn.fw - m.R && min(qo.fw + m.R, m.W - 1) <= qn.fw + m.R);
}

}  // namespace smcdet
