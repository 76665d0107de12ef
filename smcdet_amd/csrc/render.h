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
// floor clamped to 16 bits (two anchors packed per int; locations lie within
// a few pixels of the tile, and anchors this far out give empty windows either way)
__device__ __forceinline__ int ifloor16(float v) {
  return (int)fmaxf(fminf(floorf(v), 16383.0f), -16384.0f);
}

// lam[p] += amp * psf(|p + 0.5 - (h, w)|) over the source's clipped window
// (LDS read-modify-write; used for tiles above 1024 pixels or S > 64).
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
  for (int q = lane; q < npos; q += kWave) {
    const int aa = (int)(((float)q + 0.5f) * inv_bw);
    const int bb = q - (int)__umul24((unsigned)aa, (unsigned)bw);
    const int ph = r0 + aa, pw = c0 + bb;
    const float dh = ((float)ph + 0.5f) - h;
    const float dw = ((float)pw + 0.5f) - w;
    const int p = (int)__umul24((unsigned)ph, (unsigned)m.W) + pw;
    lam[p] += ampn * psf_raw<MODEL>(m, fmaf(dh, dh, dw * dw));
  }
  wave_sync();
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
}

// ---------------------------------------------------------------------------
// Pixel-centric render into registers (tiles of <= 64*PPL pixels): lane owns
// pixels p = 64k + lane, k < PPL.  Per source only the k-rows its window
// touches are visited (a wave-uniform range), and the window test is a select,
// so there is no LDS traffic and no cross-source serialisation.  The sum
// order per pixel is background, then sources 0..S-1.
// ---------------------------------------------------------------------------
template <int MODEL, int PPL>
__device__ __forceinline__ void render_regs(const DevModel& m, float (&lamk)[PPL], float sh,
                                            float sw, float sf, int S, int lane) {
  const int HW = m.H * m.W;
  const unsigned magic = (65536u + (unsigned)m.W - 1u) / (unsigned)m.W;  // p / W, p < 1024
#pragma unroll
  for (int k = 0; k < PPL; ++k) lamk[k] = m.bg;
  const float scale = m.g * psf_scale<MODEL>(m);
  for (int s = 0; s < S; ++s) {
    const float h = readlane(sh, s), w = readlane(sw, s);
    const float amp = scale * readlane(sf, s);
    const int fh = ifloor_clamped(h), fw = ifloor_clamped(w);
    const int r0 = max(fh - m.R, 0), r1 = min(fh + m.R, m.H - 1);
    if (r0 > r1 || fw + m.R < 0 || fw - m.R > m.W - 1) continue;
    const int klo = (r0 * m.W) >> 6, khi = ((r1 + 1) * m.W - 1) >> 6;
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
      if (k >= klo && k <= khi) {
        const int p = k * kWave + lane;
        const int ph = (int)(__umul24((unsigned)p, magic) >> 16);
        const int pw = p - (int)__umul24((unsigned)ph, (unsigned)m.W);
        const float dh = ((float)ph + 0.5f) - h;
        const float dw = ((float)pw + 0.5f) - w;
        const float v = amp * psf_raw<MODEL>(m, fmaf(dh, dh, dw * dw));
        const bool in = (unsigned)(ph - fh + m.R) <= 2u * (unsigned)m.R &&
                        (unsigned)(pw - fw + m.R) <= 2u * (unsigned)m.R && p < HW;
        lamk[k] += in ? v : 0.0f;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Tiles of any size (above the LDS budget): pixel-centric chunks of 64
// pixels, p = 64k + lane.  Lane s precomputes source s's amplitude and the
// chunk range [klo, khi] its clipped window's rows cover (wave-uniform
// skips); per pixel the sum order is background, then sources 0..S-1, with
// render_regs's arithmetic, so a chunk equals render_regs's register for the
// same pixel.
// ---------------------------------------------------------------------------
struct ChunkSrc {
  float h, w, amp;  // lane s: source s (amp = g * psf_scale * f)
  int klo, khi;     // chunks its window rows touch (klo > khi: none)
};

template <int MODEL>
__device__ __forceinline__ ChunkSrc chunk_sources(const DevModel& m, float sh, float sw, float sf,
                                                  int S, int lane) {
  ChunkSrc c;
  c.h = sh;
  c.w = sw;
  c.amp = m.g * psf_scale<MODEL>(m) * sf;
  const int fh = ifloor_clamped(sh), fw = ifloor_clamped(sw);
  const int r0 = max(fh - m.R, 0), r1 = min(fh + m.R, m.H - 1);
  const bool empty = lane >= S || r0 > r1 || fw + m.R < 0 || fw - m.R > m.W - 1;
  c.klo = empty ? 1 : (r0 * m.W) >> 6;
  c.khi = empty ? 0 : ((r1 + 1) * m.W - 1) >> 6;
  return c;
}

// rate at pixel p = 64k + lane (meaningful for p < H*W)
template <int MODEL>
__device__ __forceinline__ float chunk_rate(const DevModel& m, const ChunkSrc& c, int S, int k,
                                            int lane, float inv_w) {
  const int p = k * kWave + lane;
  const int ph = (int)(((float)p + 0.5f) * inv_w);  // exact: p < 2^16, W <= 2^16
  const int pw = p - ph * m.W;
  float lam = m.bg;
  for (int s = 0; s < S; ++s) {
    if (k < readlane(c.klo, s) || k > readlane(c.khi, s)) continue;
    const float h = readlane(c.h, s), w = readlane(c.w, s);
    const float amp = readlane(c.amp, s);
    const int fh = ifloor_clamped(h), fw = ifloor_clamped(w);
    const float dh = ((float)ph + 0.5f) - h;
    const float dw = ((float)pw + 0.5f) - w;
    const float v = amp * psf_raw<MODEL>(m, fmaf(dh, dh, dw * dw));
    const bool in = (unsigned)(ph - fh + m.R) <= 2u * (unsigned)m.R &&
                    (unsigned)(pw - fw + m.R) <= 2u * (unsigned)m.R;
    lam += in ? v : 0.0f;
  }
  return lam;
}

// full render into a rate image in global memory (lam[p], p < H*W)
template <int MODEL>
__device__ __forceinline__ void render_chunks(const DevModel& m, float* lam, float sh, float sw,
                                              float sf, int S, int lane) {
  const int HW = m.H * m.W;
  const float inv_w = 1.0f / (float)m.W;
  const ChunkSrc c = chunk_sources<MODEL>(m, sh, sw, sf, S, lane);
  for (int k = 0; k * kWave < HW; ++k) {
    const float v = chunk_rate<MODEL>(m, c, S, k, lane, inv_w);
    if (k * kWave + lane < HW) lam[k * kWave + lane] = v;
  }
  wave_sync();
}

// sum of the per-pixel log-likelihood without storing the rate image
template <int MODEL>
__device__ __forceinline__ double loglik_chunks(const DevModel& m, const float* __restrict__ x,
                                                float sh, float sw, float sf, int S, int lane) {
  const int HW = m.H * m.W;
  const float inv_w = 1.0f / (float)m.W;
  const ChunkSrc c = chunk_sources<MODEL>(m, sh, sw, sf, S, lane);
  float acc = 0.0f;
  for (int k = 0; k * kWave < HW; ++k) {
    const int p = k * kWave + lane;
    const float lam = chunk_rate<MODEL>(m, c, S, k, lane, inv_w);
    const float e = pix_loglik<MODEL>(m, x[p < HW ? p : HW - 1], 0.0f, lam);
    acc += p < HW ? e : 0.0f;
  }
  return wave_sum((double)acc);
}

template <int MODEL, int PPL>
__device__ __forceinline__ double pixel_sum_regs(const DevModel& m, const float* xs,
                                                 const float* lg, const float (&lamk)[PPL],
                                                 int lane) {
  const int HW = m.H * m.W;
  float acc = 0.0f;
#pragma unroll
  for (int k = 0; k < PPL; ++k) {
    const int p = k * kWave + lane;
    if (k * kWave < HW) {
      const int pp = p < HW ? p : 0;
      const float lgx = (MODEL == SMCDET_MODEL_POISSON) ? lg[pp] : 0.0f;
      const float e = pix_loglik<MODEL>(m, xs[pp], lgx, lamk[k]);
      acc += p < HW ? e : 0.0f;
    }
  }
  return wave_sum((double)acc);
}

template <int MODEL, int PPL>
__device__ __forceinline__ void store_regs(const DevModel& m, float* lam, const float (&lamk)[PPL],
                                           int lane) {
  const int HW = m.H * m.W;
#pragma unroll
  for (int k = 0; k < PPL; ++k) {
    const int p = k * kWave + lane;
    if (k * kWave < HW && p < HW) lam[p] = lamk[k];
  }
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
