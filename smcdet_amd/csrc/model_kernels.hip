// model_kernels.hip — image-model and prior kernels of the C ABI:
// smcdet_loglik, smcdet_render, smcdet_psf_dense, smcdet_sample_image,
// smcdet_log_prior, smcdet_prior_sample.
#include <math.h>

#include "render.h"

namespace smcdet {

constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWavesPerBlock * kWave;

static size_t model_lds_bytes(const smcdet_image_model_t& m, int per_wave_images) {
  const size_t HW = (size_t)m.H * m.W;
  const size_t img = (m.model == SMCDET_MODEL_POISSON ? 2 : 1) * HW;
  return (img + (size_t)kWavesPerBlock * per_wave_images * HW) * sizeof(float);
}

// ---------------------------------------------------------------------------
// loglikelihood: one particle per wave, image tile staged in LDS
// ---------------------------------------------------------------------------
template <int MODEL, int PPL>
__global__ __launch_bounds__(kBlock) void loglik_kernel(DevModel m, const float* __restrict__ img,
                                                        const float* __restrict__ locs,
                                                        const float* __restrict__ fluxes, int N,
                                                        int S, float* __restrict__ out) {
  extern __shared__ float smem[];
  const int HW = m.H * m.W;
  const int t = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* xs = smem;
  float* lg = smem + HW;
  float* lam = smem + (MODEL == SMCDET_MODEL_POISSON ? 2 : 1) * HW + wave * HW;
  stage_image<MODEL>(img + (size_t)t * HW, xs, lg, HW, threadIdx.x, kBlock);
  __syncthreads();
  const int n = blockIdx.x * kWavesPerBlock + wave;
  if (n >= N) return;
  const size_t pid = (size_t)t * N + n;
  double ll;
  if constexpr (PPL > 0) {
    float sh = 0.f, sw = 0.f, sf = 0.f;
    if (lane < S) {
      sh = locs[(pid * S + lane) * 2 + 0];
      sw = locs[(pid * S + lane) * 2 + 1];
      sf = fluxes[pid * S + lane];
    }
    float lamk[PPL > 0 ? PPL : 1];
    render_regs<MODEL, PPL>(m, lamk, sh, sw, sf, S, lane);
    ll = pixel_sum_regs<MODEL, PPL>(m, xs, lg, lamk, lane);
  } else {
    render_sources_mem<MODEL>(m, lam, locs + pid * S * 2, fluxes + pid * S, S, lane);
    ll = pixel_sum<MODEL>(m, xs, lg, lam, nullptr, lane);
  }
  if (lane == 0) out[pid] = (float)ll;
}

// tiles above the LDS budget (M71): the tile image stays in global memory
// (L2-resident), the rate image is rendered chunk by chunk in registers
template <int MODEL>
__global__ __launch_bounds__(kBlock) void loglik_global_kernel(DevModel m,
                                                               const float* __restrict__ img,
                                                               const float* __restrict__ locs,
                                                               const float* __restrict__ fluxes,
                                                               int N, int S,
                                                               float* __restrict__ out) {
  const int HW = m.H * m.W;
  const int t = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = blockIdx.x * kWavesPerBlock + wave;
  if (n >= N) return;
  const size_t pid = (size_t)t * N + n;
  float sh = 0.f, sw = 0.f, sf = 0.f;
  if (lane < S) {
    sh = locs[(pid * S + lane) * 2 + 0];
    sw = locs[(pid * S + lane) * 2 + 1];
    sf = fluxes[pid * S + lane];
  }
  const double ll = loglik_chunks<MODEL>(m, img + (size_t)t * HW, sh, sw, sf, S, lane);
  if (lane == 0) out[pid] = (float)ll;
}

template <int MODEL>
__global__ __launch_bounds__(kBlock) void render_global_kernel(DevModel m,
                                                               const float* __restrict__ locs,
                                                               const float* __restrict__ fluxes,
                                                               int N, int S,
                                                               float* __restrict__ rate) {
  const int HW = m.H * m.W;
  const int t = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = blockIdx.x * kWavesPerBlock + wave;
  if (n >= N) return;
  const size_t pid = (size_t)t * N + n;
  float sh = 0.f, sw = 0.f, sf = 0.f;
  if (lane < S) {
    sh = locs[(pid * S + lane) * 2 + 0];
    sw = locs[(pid * S + lane) * 2 + 1];
    sf = fluxes[pid * S + lane];
  }
  const ChunkSrc c = chunk_sources<MODEL>(m, sh, sw, sf, S, lane);
  const float inv_w = 1.0f / (float)m.W;
  for (int k = 0; k * kWave < HW; ++k) {
    const int p = k * kWave + lane;
    const float v = chunk_rate<MODEL>(m, c, S, k, lane, inv_w);
    if (p < HW) rate[((size_t)t * HW + p) * N + n] = v;
  }
}

// rate[T,H,W,N]
template <int MODEL>
__global__ __launch_bounds__(kBlock) void render_kernel(DevModel m, const float* __restrict__ locs,
                                                        const float* __restrict__ fluxes, int N,
                                                        int S, float* __restrict__ rate) {
  extern __shared__ float smem[];
  const int HW = m.H * m.W;
  const int t = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* lam = smem + wave * HW;
  const int n = blockIdx.x * kWavesPerBlock + wave;
  if (n >= N) return;
  const size_t pid = (size_t)t * N + n;
  render_sources_mem<MODEL>(m, lam, locs + pid * S * 2, fluxes + pid * S, S, lane);
  for (int p = lane; p < HW; p += kWave) rate[((size_t)t * HW + p) * N + n] = lam[p];
}

// psf[T,H,W,N,S] (zero-filled beforehand): thread per (t, n, s) window
template <int MODEL>
__global__ void psf_dense_kernel(DevModel m, const float* __restrict__ locs, int T, int N, int S,
                                 float* __restrict__ psf) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)T * N * S) return;
  const int s = (int)(i % S);
  const size_t tn = i / S;
  const int n = (int)(tn % N);
  const int t = (int)(tn / N);
  const float h = locs[i * 2 + 0], w = locs[i * 2 + 1];
  const int fh = ifloor_clamped(h), fw = ifloor_clamped(w);
  for (int ph = max(fh - m.R, 0); ph <= min(fh + m.R, m.H - 1); ++ph)
    for (int pw = max(fw - m.R, 0); pw <= min(fw + m.R, m.W - 1); ++pw) {
      const float dh = ((float)ph + 0.5f) - h, dw = ((float)pw + 0.5f) - w;
      psf[((((size_t)t * m.H + ph) * m.W + pw) * N + n) * S + s] =
          psf_eval<MODEL>(m, fmaf(dh, dh, dw * dw));
    }
}

// ---------------------------------------------------------------------------
// noise: Normal (M71, images.py:147-157) or Poisson (images.py:78-83)
// ---------------------------------------------------------------------------
__device__ float std_normal(uint32_t a, uint32_t b) {
  const float u1 = ((float)(a >> 8) + 0.5f) * 5.9604644775390625e-08f;  // (0,1)
  const float u2 = u01(b);
  return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

// PTRS (Hormann 1993) for lambda >= 10, multiplication method below
__device__ float poisson_draw(float lam, uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1) {
  if (!(lam > 0.f)) return 0.f;
  uint32_t ctr = 0;
  if (lam < 10.f) {
    const float L = expf(-lam);
    float p = 1.f;
    int k = -1;
    while (true) {
      U4 r = philox4x32(c0, c1, ctr++, kTagNoise + 1, k0, k1);
      const uint32_t ws[4] = {r.x, r.y, r.z, r.w};
      for (int i = 0; i < 4; ++i) {
        ++k;
        p *= u01(ws[i]);
        if (p <= L) return (float)k;
      }
      if (ctr > 4096) return (float)k;
    }
  }
  const float slam = sqrtf(lam), loglam = logf(lam);
  const float b = 0.931f + 2.53f * slam;
  const float a = -0.059f + 0.02483f * b;
  const float inv_alpha = 1.1239f + 1.1328f / (b - 3.4f);
  const float vr = 0.9277f - 3.6224f / (b - 2.f);
  while (ctr < 100000) {
    U4 r = philox4x32(c0, c1, ctr++, kTagNoise + 2, k0, k1);
    const float U = u01(r.x) - 0.5f;
    const float V = ((float)(r.y >> 8) + 0.5f) * 5.9604644775390625e-08f;
    const float us = 0.5f - fabsf(U);
    const float k = floorf((2.f * a / us + b) * U + lam + 0.43f);
    if (us >= 0.07f && V <= vr) return k;
    if (k < 0.f || (us < 0.013f && V > us)) continue;
    if (logf(V) + logf(inv_alpha) - logf(a / (us * us) + b) <= -lam + k * loglam - lgammaf(k + 1.f))
      return k;
  }
  return lam;
}

template <int MODEL>
__global__ void sample_image_kernel(DevModel m, const float* __restrict__ rate, int64_t count,
                                    uint32_t k0, uint32_t k1, uint64_t offset,
                                    float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const float lam = rate[i];
  const uint64_t c = offset + (uint64_t)i;
  if constexpr (MODEL == SMCDET_MODEL_M71) {
    U4 r = philox4x32((uint32_t)c, (uint32_t)(c >> 32), 0u, kTagNoise, k0, k1);
    const float sd = sqrtf(fmaf(m.eta, lam, m.s0sq));
    out[i] = fmaf(sd, std_normal(r.x, r.y), lam);
  } else {
    out[i] = poisson_draw(lam, k0, k1, (uint32_t)c, (uint32_t)(c >> 32));
  }
}

// ---------------------------------------------------------------------------
// priors
// ---------------------------------------------------------------------------
// M71Prior.log_prob (prior.py:220-226, :67-75) / ParetoStarPrior.log_prob
// (prior.py:183-189): thread per particle
// tile_boxes [T,4] (lo_h, lo_w, hi_h, hi_w), nullable: per-tile location boxes
// (a partition of the padded image, SMCDET_ABI 12); the Poisson count mean
// scales with the box area
__global__ void log_prior_kernel(DevPrior pr, const float* __restrict__ counts,
                                 const float* __restrict__ locs, const float* __restrict__ fluxes,
                                 int64_t TN, int N, int S, const float* __restrict__ boxes,
                                 float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= TN) return;
  const float c = counts[i];
  if (boxes) tile_box_prior(pr, boxes + 4 * (i / N));
  float lp;
  if (pr.kind == SMCDET_PRIOR_M71) {
    lp = c * pr.count_c0 - pr.count_c1 - lgammaf(c + 1.0f);  // Poisson.log_prob
  } else {
    const bool in = c >= (float)pr.min_objects && c <= (float)pr.max_objects;
    lp = in ? pr.count_c0 : -INFINITY;  // DiscreteUniform.log_prob
  }
  float sl = 0.f, sfl = 0.f;
  for (int s = 0; s < S; ++s) {
    if (!((float)s < c)) break;  // counts_mask
    const float h = locs[(i * S + s) * 2 + 0], w = locs[(i * S + s) * 2 + 1];
    const float lh = (h >= pr.lo && h < pr.hi_h) ? pr.loc_lp_h : -INFINITY;
    const float lw = (w >= pr.lo_w && w < pr.hi_w) ? pr.loc_lp_w : -INFINITY;
    sl += lh + lw;
    float f = fluxes[i * S + s];
    if (f == 0.f) f = pr.lower;
    sfl += pr.flux_c - pr.ap1 * logf(f);
  }
  out[i] = lp + sl + sfl;
}

// Prior.sample(stratify_by_count=True) (prior.py:47-64, :201-217): thread per (t,n,s)
__global__ void prior_sample_kernel(DevPrior pr, int T, int N, int n_per_count, int S,
                                    uint32_t k0, uint32_t k1, uint64_t offset,
                                    const float* __restrict__ uloc, const float* __restrict__ uflux,
                                    const float* __restrict__ boxes, float* __restrict__ counts,
                                    float* __restrict__ locs, float* __restrict__ fluxes) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)T * N * S) return;
  const int s = (int)(i % S);
  const int64_t tn = i / S;
  const int n = (int)(tn % N);
  if (boxes) tile_box_prior(pr, boxes + 4 * (tn / N));
  const float c = (float)(pr.min_objects + n / n_per_count);
  if (s == 0) counts[tn] = c;
  float uh, uw, uf;
  if (uloc) {
    uh = uloc[i * 2 + 0];
    uw = uloc[i * 2 + 1];
    uf = uflux[i];
  } else {
    // keyed by particle (t*N + n) with the source in the counter, as the
    // other kernels key theirs: a tile's draws do not depend on how many
    // tiles the grid has (a rank's shard reproduces the single-process run)
    const uint64_t ctr = offset + (uint64_t)s;
    U4 r = philox4x32((uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)tn, kTagPriorLoc, k0, k1);
    uh = u01(r.x);
    uw = u01(r.y);
    uf = u01(r.z);
  }
  const bool on = (float)s < c;
  // Uniform(low, high).rsample: low + u*(high - low)
  const float h = fmaf(uh, pr.hi_h - pr.lo, pr.lo);
  const float w = fmaf(uw, pr.hi_w - pr.lo_w, pr.lo_w);
  float f;
  if (pr.kind == SMCDET_PRIOR_M71) {
    // TruncatedPareto.sample (distributions.py:76-85)
    const float Ua = powf(pr.upper, pr.alpha), La = powf(pr.lower, pr.alpha);
    const float num = Ua - uf * Ua + uf * La;
    f = powf(num / (La * Ua), -1.0f / pr.alpha);
  } else {
    // Pareto(scale, alpha) by inverse CDF
    f = pr.lower * powf(1.0f - uf, -1.0f / pr.alpha);
  }
  locs[i * 2 + 0] = on ? h : 0.f;
  locs[i * 2 + 1] = on ? w : 0.f;
  fluxes[i] = on ? f : 0.f;
}

}  // namespace smcdet

using namespace smcdet;

#define SMCDET_DISPATCH_MODEL(mdl, KERNEL, ...)                              \
  ((mdl) == SMCDET_MODEL_M71 ? (KERNEL<SMCDET_MODEL_M71>)(__VA_ARGS__)      \
                             : (KERNEL<SMCDET_MODEL_POISSON>)(__VA_ARGS__))

extern "C" {

int smcdet_loglik(const smcdet_image_model_t* model, const float* tiled_image, const float* locs,
                  const float* fluxes, int32_t T, int32_t N, int32_t S, float* out,
                  void* stream) {
  int rc = validate_model(model, kMaxGlobalPixels);
  if (rc) return rc;
  if (!tiled_image || !locs || !fluxes || !out) return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || N <= 0 || S < 0)
    return set_error(SMCDET_EUNSUPPORTED, "T=%d N=%d S=%d (need T,N>0, S>=0)", T, N, S);
  if (T > 65535) return set_error(SMCDET_EUNSUPPORTED, "T=%d > 65535", T);
  const DevModel m = make_dev_model(*model);
  const dim3 grid((N + kWavesPerBlock - 1) / kWavesPerBlock, T);
  if (m.H * m.W > kMaxLdsPixels) {  // M71 (validate_model), global-memory path
    if (S > kWave) return set_error(SMCDET_EUNSUPPORTED, "S=%d > 64 above %d pixels", S,
                                    kMaxLdsPixels);
    hipLaunchKernelGGL(loglik_global_kernel<SMCDET_MODEL_M71>, grid, dim3(kBlock), 0,
                       (hipStream_t)stream, m, tiled_image, locs, fluxes, N, S, out);
    return check_launch("smcdet_loglik");
  }
  const size_t lds = model_lds_bytes(*model, 1);
  hipStream_t st = (hipStream_t)stream;
  const int HW = m.H * m.W;
  const int ppl = S > kWave ? 0 : (HW <= 64 ? 1 : (HW <= 256 ? 4 : (HW <= 1024 ? 16 : 0)));
#define SMCDET_LL_LAUNCH(MDL, P)                                                            \
  do {                                                                                       \
    rc = ensure_lds((const void*)loglik_kernel<MDL, P>, lds);                                \
    if (rc) return rc;                                                                       \
    hipLaunchKernelGGL((loglik_kernel<MDL, P>), grid, dim3(kBlock), lds, st, m, tiled_image, \
                       locs, fluxes, N, S, out);                                             \
  } while (0)
  if (m.model == SMCDET_MODEL_M71) {
    if (ppl == 1) SMCDET_LL_LAUNCH(SMCDET_MODEL_M71, 1);
    else if (ppl == 4) SMCDET_LL_LAUNCH(SMCDET_MODEL_M71, 4);
    else if (ppl == 16) SMCDET_LL_LAUNCH(SMCDET_MODEL_M71, 16);
    else SMCDET_LL_LAUNCH(SMCDET_MODEL_M71, 0);
  } else {
    if (ppl == 1) SMCDET_LL_LAUNCH(SMCDET_MODEL_POISSON, 1);
    else if (ppl == 4) SMCDET_LL_LAUNCH(SMCDET_MODEL_POISSON, 4);
    else if (ppl == 16) SMCDET_LL_LAUNCH(SMCDET_MODEL_POISSON, 16);
    else SMCDET_LL_LAUNCH(SMCDET_MODEL_POISSON, 0);
  }
#undef SMCDET_LL_LAUNCH
  return check_launch("smcdet_loglik");
}

int smcdet_render(const smcdet_image_model_t* model, const float* locs, const float* fluxes,
                  int32_t T, int32_t N, int32_t S, float* rate, void* stream) {
  int rc = validate_model(model, kMaxGlobalPixels);
  if (rc) return rc;
  if (!locs || !fluxes || !rate) return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || N <= 0 || S < 0 || T > 65535)
    return set_error(SMCDET_EUNSUPPORTED, "T=%d N=%d S=%d", T, N, S);
  const DevModel m = make_dev_model(*model);
  const dim3 grid((N + kWavesPerBlock - 1) / kWavesPerBlock, T);
  if (m.H * m.W > kMaxLdsPixels) {
    if (S > kWave) return set_error(SMCDET_EUNSUPPORTED, "S=%d > 64 above %d pixels", S,
                                    kMaxLdsPixels);
    hipLaunchKernelGGL(render_global_kernel<SMCDET_MODEL_M71>, grid, dim3(kBlock), 0,
                       (hipStream_t)stream, m, locs, fluxes, N, S, rate);
    return check_launch("smcdet_render");
  }
  const size_t lds = (size_t)kWavesPerBlock * m.H * m.W * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  rc = ensure_lds(m.model == SMCDET_MODEL_M71 ? (const void*)render_kernel<SMCDET_MODEL_M71>
                                              : (const void*)render_kernel<SMCDET_MODEL_POISSON>,
                  lds);
  if (rc) return rc;
  if (m.model == SMCDET_MODEL_M71)
    hipLaunchKernelGGL(render_kernel<SMCDET_MODEL_M71>, grid, dim3(kBlock), lds, st, m, locs,
                       fluxes, N, S, rate);
  else
    hipLaunchKernelGGL(render_kernel<SMCDET_MODEL_POISSON>, grid, dim3(kBlock), lds, st, m, locs,
                       fluxes, N, S, rate);
  return check_launch("smcdet_render");
}

int smcdet_psf_dense(const smcdet_image_model_t* model, const float* locs, int32_t T, int32_t N,
                     int32_t S, float* psf, void* stream) {
  int rc = validate_model(model, kMaxGlobalPixels);
  if (rc) return rc;
  if (!locs || !psf) return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || N <= 0 || S <= 0) return set_error(SMCDET_EUNSUPPORTED, "empty shape");
  const DevModel m = make_dev_model(*model);
  hipStream_t st = (hipStream_t)stream;
  const size_t total = (size_t)T * m.H * m.W * N * S;
  if (hipMemsetAsync(psf, 0, total * sizeof(float), st) != hipSuccess)
    return set_error(SMCDET_EHIP, "smcdet_psf_dense: memset failed");
  const size_t nthr = (size_t)T * N * S;
  const dim3 grid((unsigned)((nthr + 255) / 256));
  if (m.model == SMCDET_MODEL_M71)
    hipLaunchKernelGGL(psf_dense_kernel<SMCDET_MODEL_M71>, grid, dim3(256), 0, st, m, locs, T, N,
                       S, psf);
  else
    hipLaunchKernelGGL(psf_dense_kernel<SMCDET_MODEL_POISSON>, grid, dim3(256), 0, st, m, locs, T,
                       N, S, psf);
  return check_launch("smcdet_psf_dense");
}

int smcdet_sample_image(const smcdet_image_model_t* model, const float* rate, int64_t count,
                        uint64_t seed, uint64_t offset, float* image, void* stream) {
  int rc = validate_model(model, kMaxGlobalPixels);
  if (rc) return rc;
  if (!rate || !image || count < 0) return set_error(SMCDET_EINVAL, "bad buffer/count");
  if (count == 0) return SMCDET_OK;
  const DevModel m = make_dev_model(*model);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)((count + 255) / 256));
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  if (m.model == SMCDET_MODEL_M71)
    hipLaunchKernelGGL(sample_image_kernel<SMCDET_MODEL_M71>, grid, dim3(256), 0, st, m, rate,
                       count, k0, k1, offset, image);
  else
    hipLaunchKernelGGL(sample_image_kernel<SMCDET_MODEL_POISSON>, grid, dim3(256), 0, st, m, rate,
                       count, k0, k1, offset, image);
  return check_launch("smcdet_sample_image");
}

int smcdet_log_prior(const smcdet_prior_t* prior, const float* counts, const float* locs,
                     const float* fluxes, int32_t T, int32_t N, int32_t S,
                     const float* tile_boxes, float* out, void* stream) {
  int rc = validate_prior(prior);
  if (rc) return rc;
  if (!counts || !locs || !fluxes || !out) return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || N <= 0 || S < 0) return set_error(SMCDET_EUNSUPPORTED, "empty shape");
  const DevPrior d = make_dev_prior(*prior);
  const int64_t TN = (int64_t)T * N;
  hipLaunchKernelGGL(log_prior_kernel, dim3((unsigned)((TN + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, d, counts, locs, fluxes, TN, N, S, tile_boxes, out);
  return check_launch("smcdet_log_prior");
}

int smcdet_prior_sample(const smcdet_prior_t* prior, int32_t T, int32_t n_per_count,
                        uint64_t seed, uint64_t offset, const float* uloc, const float* uflux,
                        const float* tile_boxes, float* counts, float* locs, float* fluxes,
                        void* stream) {
  int rc = validate_prior(prior);
  if (rc) return rc;
  if (!counts || !locs || !fluxes) return set_error(SMCDET_EINVAL, "null buffer");
  if ((uloc == nullptr) != (uflux == nullptr))
    return set_error(SMCDET_EINVAL, "uloc and uflux must both be given or both null");
  if (T <= 0 || n_per_count <= 0) return set_error(SMCDET_EUNSUPPORTED, "empty shape");
  const DevPrior d = make_dev_prior(*prior);
  const int N = (prior->max_objects - prior->min_objects + 1) * n_per_count;
  const int S = prior->max_objects;
  const int64_t total = (int64_t)T * N * S;
  hipStream_t st = (hipStream_t)stream;
  if (S == 0) {
    // no sources: counts = min_objects = 0 everywhere
    if (hipMemsetAsync(counts, 0, (size_t)T * N * sizeof(float), st) != hipSuccess)
      return set_error(SMCDET_EHIP, "memset failed");
    return SMCDET_OK;
  }
  hipLaunchKernelGGL(prior_sample_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     d, T, N, n_per_count, S, (uint32_t)seed, (uint32_t)(seed >> 32), offset, uloc,
                     uflux, tile_boxes, counts, locs, fluxes);
  return check_launch("smcdet_prior_sample");
}

}  // extern "C"
