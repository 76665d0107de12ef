// render.h — one-particle-per-wavefront rendering of a catalog into a per-wave
// LDS rate image, and the wave-reduced per-pixel log-likelihood.
//
// Restates smcdet/images.py:28-76 (psf scatter) + :159-175 / :85-102
// (likelihood) without materialising the dense [T,H,W,N,S] PSF tensor: each
// source's (2R+1)^2 window (anchored at floor(loc), clipped to the tile) is
// flattened and dealt over the 64 lanes (289 positions -> 5 passes), and its
// contribution is added straight into the particle's rate image in LDS.
#pragma once

#include "device.h"

namespace smcdet {

__device__ __forceinline__ int ifloor_clamped(float v) {
  return (int)fmaxf(fminf(floorf(v), 1.0e6f), -1.0e6f);
}

// lam[p] += amp * psf(|p + 0.5 - (h, w)|) over the source's clipped window.
// ds_add_f32 (LDS atomic, no return): the adds of one wave to one address are
// applied in program order, so the sum order is the source order (the result
// is deterministic) while no add waits for the previous one's read.
template <int MODEL>
__device__ __forceinline__ void add_source(const DevModel& m, float* lam, float h, float w,
                                           float amp, int lane) {
  const int fh = ifloor_clamped(h), fw = ifloor_clamped(w);
  const int r0 = max(fh - m.R, 0), r1 = min(fh + m.R, m.H - 1);
  const int c0 = max(fw - m.R, 0), c1 = min(fw + m.R, m.W - 1);
  if (r0 > r1 || c0 > c1) return;
  const int bw = c1 - c0 + 1;
  const int npos = (r1 - r0 + 1) * bw;
  const float inv_bw = 1.0f / (float)bw;
  const float ampn = amp * psf_scale<MODEL>(m);
  for (int q0 = 0; q0 < npos; q0 += kWave) {
    const int q = q0 + lane;
    const int aa = (int)(((float)q + 0.5f) * inv_bw);
    const int bb = q - aa * bw;
    const int ph = r0 + aa, pw = c0 + bb;
    const float dh = ((float)ph + 0.5f) - h;
    const float dw = ((float)pw + 0.5f) - w;
    const float v = ampn * psf_raw<MODEL>(m, fmaf(dh, dh, dw * dw));
    if (q < npos) atomicAdd(&lam[ph * m.W + pw], v);
  }
}

// full render: lam = B + sum_s g*f_s*psf_s ; lane s (< S) holds source s
template <int MODEL>
__device__ __forceinline__ void render_sources(const DevModel& m, float* lam, float sh, float sw,
                                               float sf, int S, int lane) {
  const int HW = m.H * m.W;
  for (int p = lane; p < HW; p += kWave) lam[p] = m.bg;
  wave_sync();
  for (int s = 0; s < S; ++s) {
    const float h = readlane(sh, s), w = readlane(sw, s), f = readlane(sf, s);
    add_source<MODEL>(m, lam, h, w, m.g * f, lane);
  }
  wave_sync();
}

// full render with the catalog read from memory (any S; the per-source loads
// are wave-uniform and become scalar loads)
template <int MODEL>
__device__ __forceinline__ void render_sources_mem(const DevModel& m, float* lam,
                                                   const float* __restrict__ locs,
                                                   const float* __restrict__ fluxes, int S,
                                                   int lane) {
  const int HW = m.H * m.W;
  for (int p = lane; p < HW; p += kWave) lam[p] = m.bg;
  wave_sync();
  for (int s = 0; s < S; ++s)
    add_source<MODEL>(m, lam, locs[2 * s], locs[2 * s + 1], m.g * fluxes[s], lane);
  wave_sync();
}

// sum over pixels of the per-pixel log-likelihood (wave-uniform result);
// optionally caches the per-pixel terms in lp
template <int MODEL>
__device__ __forceinline__ double pixel_sum(const DevModel& m, const float* xs, const float* lg,
                                            const float* lam, float* lp, int lane) {
  const int HW = m.H * m.W;
  float acc = 0.0f;
  for (int p = lane; p < HW; p += kWave) {
    const float lgx = (MODEL == SMCDET_MODEL_POISSON) ? lg[p] : 0.0f;
    const float e = pix_loglik<MODEL>(m, xs[p], lgx, lam[p]);
    if (lp) lp[p] = e;
    acc += e;
  }
  wave_sync();
  return wave_sum((double)acc);
}

}  // namespace smcdet
