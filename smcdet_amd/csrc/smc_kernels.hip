// smc_kernels.hip — per-tile SMC bookkeeping on device: adaptive tempering
// (sampler.py:93-125), reweighting / log-evidence / ESS (sampler.py:181-196),
// systematic and multinomial resampling (sampler.py:127-169) and pruning
// (sampler.py:198-219).
//
// One 1024-thread workgroup per tile does temper -> reweight -> resample
// indices in one launch, so an SMC iteration needs no host round trip (the
// reference copies the log-likelihoods to the host and runs scipy brentq per
// tile).  The tempering root is found by the same Brent iteration as scipy's
// brentq (so the same root is picked when ESS(delta) crosses the threshold
// more than once), each f evaluation being a workgroup-wide reduction.
#include <math.h>

#include "device.h"

namespace smcdet {

constexpr int kTB = 256;            // threads per tile workgroup
constexpr int kTW = kTB / kWave;    // 4 waves

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
};

// Workgroup reductions with ONE barrier each: wave DPP reductions -> per-wave
// slots of a double-buffered LDS array -> every thread combines the kTW slots
// in a fixed order (deterministic; every thread ends with the same value).
// `parity` lives in registers and toggles identically in every thread, so a
// buffer is not rewritten before all threads passed the next call's barrier.
struct TileRed {
  double d[2][kTW][2];
  float f[2][kTW];
};
__device__ __forceinline__ void block_sum2(double& a, double& b, TileRed* r, int& parity) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  a = wave_sum(a);
  b = wave_sum(b);
  const int k = parity;
  parity ^= 1;
  if (lane == 0) {
    r->d[k][wave][0] = a;
    r->d[k][wave][1] = b;
  }
  __syncthreads();
  double sa = 0.0, sb = 0.0;
#pragma unroll
  for (int i = 0; i < kTW; ++i) {
    sa += r->d[k][i][0];
    sb += r->d[k][i][1];
  }
  a = sa;
  b = sb;
}
__device__ __forceinline__ float block_max(float v, TileRed* r, int& parity) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_max(v);
  const int k = parity;
  parity ^= 1;
  if (lane == 0) r->f[k][wave] = v;
  __syncthreads();
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < kTW; ++i) m = fmaxf(m, r->f[k][i]);
  return m;
}

// f(delta) = ESS(delta) - threshold, evaluated by the whole workgroup from the
// LDS-staged log-likelihoods: ESS = (sum e)^2 / sum e^2, e = exp(d*l - max(d*l)),
// d = float32(delta) (the reference multiplies its float32 log-likelihoods by
// the python float delta, i.e. at float32 precision; sampler.py:93-97).
__device__ double block_ess_objective(const float* ll, int N, float lmax, double delta,
                                      double thr, TileRed* red, int& parity) {
  const float df = (float)delta;
  const float m = df * lmax;  // = max_i fl(df*l_i): rounding is monotone
  double s1 = 0.0, s2 = 0.0;
  for (int i = threadIdx.x; i < N; i += kTB) {
    const double e = (double)fast_exp2((df * ll[i] - m) * kLog2e);
    s1 += e;
    s2 += e * e;
  }
  block_sum2(s1, s2, red, parity);
  return s1 * s1 / s2 - thr;
}

// scipy.optimize.brentq (scipy/optimize/Zeros/brentq.c, the algorithm the
// reference calls at sampler.py:114-120) with xtol = rtol = 1e-6, maxiter
// 100.  Every thread runs the (deterministic) control flow on identical
// values; the workgroup evaluates f together.
__device__ double block_brentq(const float* ll, int N, float lmax, double thr, double xa,
                               double xb, double fa, double fb, TileRed* red, int& parity) {
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
        stry = -fcur * (xcur - xpre) / (fcur - fpre);  // interpolate
      } else {                                         // extrapolate
        const double dpre = (fpre - fcur) / (xpre - xcur);
        const double dblk = (fblk - fcur) / (xblk - xcur);
        stry = -fcur * (fblk * dblk - fpre * dpre) / (dblk * dpre * (fblk - fpre));
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
    fcur = block_ess_objective(ll, N, lmax, xcur, thr, red, parity);
  }
  return xcur;
}

__global__ __launch_bounds__(kTB) void tile_kernel(TileArgs a) {
  extern __shared__ float buf[];  // N floats: log-likelihoods, then weights / cumsum
  __shared__ TileRed red;
  int parity = 0;
  const int t = blockIdx.x;
  const int N = a.N;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

  if (a.flags & (kDoTemper | kDoWeights)) {
    const float* llg = a.loglik + (size_t)t * N;
    for (int i = threadIdx.x; i < N; i += kTB) buf[i] = llg[i];
    __syncthreads();
  }

  // ------------------------------------------------------------------ temper
  if (a.flags & kDoTemper) {
    const float tau = a.temperature[t];
    float lm = -INFINITY;
    for (int i = threadIdx.x; i < N; i += kTB) lm = fmaxf(lm, buf[i]);
    lm = block_max(lm, &red, parity);
    const double top = 1.0 - (double)tau;
    // sampler.py:113-122: root-find only if ESS at delta = 1 - tau is below threshold
    const double ftop = block_ess_objective(buf, N, lm, top, a.ess_threshold, &red, parity);
    double delta = top;
    if (ftop < 0.0) {
      const double f0 = block_ess_objective(buf, N, lm, 0.0, a.ess_threshold, &red, parity);
      delta = block_brentq(buf, N, lm, a.ess_threshold, 0.0, top, f0, ftop, &red, parity);
    }
    if (threadIdx.x == 0) {
      const float d32 = (float)delta;  // delta tensor is float32 (sampler.py:105)
      a.temperature_prev[t] = tau;
      a.temperature[t] = tau + d32;
    }
    __syncthreads();
  }

  // ------------------------------------------------------------ update weights
  if (a.flags & kDoWeights) {
    const float d = a.temperature[t] - a.temperature_prev[t];
    float mx = -INFINITY;
    for (int i = threadIdx.x; i < N; i += kTB) {
      const float lw = nan_to_num(d * buf[i], -INFINITY);
      a.log_w[(size_t)t * N + i] = lw;
      mx = fmaxf(mx, lw);
    }
    mx = block_max(mx, &red, parity);
    double s = 0.0, unused = 0.0;
    for (int i = threadIdx.x; i < N; i += kTB)
      s += (double)expf(nan_to_num(d * buf[i], -INFINITY) - mx);
    block_sum2(s, unused, &red, parity);
    const float sf = (float)s;
    double q = 0.0;
    for (int i = threadIdx.x; i < N; i += kTB) {
      const float wv = expf(nan_to_num(d * buf[i], -INFINITY) - mx) / sf;
      a.weights[(size_t)t * N + i] = wv;
      buf[i] = wv;  // same thread, same index: no hazard
      q += (double)wv * (double)wv;
    }
    block_sum2(q, unused, &red, parity);
    if (threadIdx.x == 0) {
      a.ess[t] = (float)(1.0 / q);
      a.logZ[t] = (a.logZ[t] + mx) + logf(sf / (float)N);
    }
  }

  // ---------------------------------------------------------- resample index
  if (a.flags & kDoResample) {
    if (!(a.flags & kDoWeights)) {
      const float* W = a.weights + (size_t)t * N;
      for (int i = threadIdx.x; i < N; i += kTB) buf[i] = W[i];
    }
    __syncthreads();
    // bins = cumsum(W): float64 running sum rounded per element to float32
    // (what torch's CPU cumsum does), contiguous chunk per thread, in place
    const int chunk = (N + kTB - 1) / kTB;
    const int b0 = min((int)threadIdx.x * chunk, N), b1 = min(b0 + chunk, N);
    double part = 0.0;
    for (int i = b0; i < b1; ++i) part += (double)buf[i];
    double incl = part;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double y = __shfl_up(incl, o, kWave);
      if (lane >= o) incl += y;
    }
    const int k = parity;
    parity ^= 1;
    if (lane == 63) red.d[k][wave][0] = incl;
    __syncthreads();
    double base = 0.0;
    for (int i = 0; i < wave; ++i) base += red.d[k][i][0];
    double run = base + incl - part;
    for (int i = b0; i < b1; ++i) {
      run += (double)buf[i];
      buf[i] = (float)run;
    }
    __syncthreads();
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
    const float total = buf[N - 1];
    for (int n = threadIdx.x; n < N; n += kTB) {
      int lo = 0, hi = N;  // first i with pred(bins[i])
      if (a.method == SMCDET_RESAMPLE_SYSTEMATIC) {
        // u = (n + U) / N in float32 (sampler.py:144); bucketize right=False
        const float un = ((float)n + U) / (float)N;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (buf[mid] >= un) hi = mid; else lo = mid + 1;
        }
      } else {
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
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (buf[mid] > target) hi = mid; else lo = mid + 1;
        }
      }
      a.idx[(size_t)t * N + n] = (int64_t)min(lo, N - 1);
    }
  }
}

// gather: thread per (t, n, s)
__global__ void gather_kernel(const int64_t* __restrict__ idx, int T, int N, int S,
                              const float* __restrict__ cin, const float* __restrict__ lin,
                              const float* __restrict__ fin, float* __restrict__ cout,
                              float* __restrict__ lout, float* __restrict__ fout) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)T * N * (S > 0 ? S : 1);
  if (i >= total) return;
  const int Sx = S > 0 ? S : 1;
  const int s = (int)(i % Sx);
  const int64_t tn = i / Sx;
  const int64_t t = tn / N;
  const int64_t src = t * N + idx[tn];
  if (s == 0) cout[tn] = cin[src];
  if (S > 0) {
    lout[(tn * S + s) * 2 + 0] = lin[(src * S + s) * 2 + 0];
    lout[(tn * S + s) * 2 + 1] = lin[(src * S + s) * 2 + 1];
    fout[tn * S + s] = fin[src * S + s];
  }
}

// prune: thread per particle (sampler.py:198-219)
__global__ void prune_kernel(const float* __restrict__ locs, const float* __restrict__ fluxes,
                             int64_t TN, int S, float tile_dim, float thr,
                             int64_t* __restrict__ cnt, float* __restrict__ lout,
                             float* __restrict__ fout) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= TN) return;
  int k = 0;
  for (int s = 0; s < S; ++s) {
    const float h = locs[(i * S + s) * 2 + 0], w = locs[(i * S + s) * 2 + 1];
    const float f = fluxes[i * S + s];
    if (h > 0.f && h < tile_dim && w > 0.f && w < tile_dim && f > thr) {
      lout[(i * S + k) * 2 + 0] = h;
      lout[(i * S + k) * 2 + 1] = w;
      fout[i * S + k] = f;
      ++k;
    }
  }
  cnt[i] = k;
  for (int s = k; s < S; ++s) {
    lout[(i * S + s) * 2 + 0] = 0.f;
    lout[(i * S + s) * 2 + 1] = 0.f;
    fout[i * S + s] = 0.f;
  }
}

static int launch_tile(const TileArgs& a, hipStream_t st) {
  const size_t lds = (size_t)a.N * sizeof(float);
  int rc = ensure_lds((const void*)tile_kernel, lds + sizeof(TileRed));
  if (rc) return rc;
  hipLaunchKernelGGL(tile_kernel, dim3(a.T), dim3(kTB), lds, st, a);
  return check_launch("smcdet tile kernel");
}

}  // namespace smcdet

using namespace smcdet;

extern "C" {

int smcdet_temper(const float* loglik, float* temperature, float* temperature_prev, int32_t T,
                  int32_t N, double ess_threshold, void* stream) {
  if (!loglik || !temperature || !temperature_prev) return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || N <= 0) return set_error(SMCDET_EUNSUPPORTED, "T=%d N=%d", T, N);
  TileArgs a{};
  a.flags = kDoTemper;
  a.T = T;
  a.N = N;
  a.ess_threshold = ess_threshold;
  a.loglik = loglik;
  a.temperature = temperature;
  a.temperature_prev = temperature_prev;
  return launch_tile(a, (hipStream_t)stream);
}

int smcdet_update_weights(const float* loglik, const float* temperature,
                          const float* temperature_prev, float* log_weights_unnorm,
                          float* weights, float* ess, float* log_norm_const, int32_t T,
                          int32_t N, void* stream) {
  if (!loglik || !temperature || !temperature_prev || !log_weights_unnorm || !weights || !ess ||
      !log_norm_const)
    return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || N <= 0) return set_error(SMCDET_EUNSUPPORTED, "T=%d N=%d", T, N);
  TileArgs a{};
  a.flags = kDoWeights;
  a.T = T;
  a.N = N;
  a.loglik = loglik;
  a.temperature = const_cast<float*>(temperature);
  a.temperature_prev = const_cast<float*>(temperature_prev);
  a.log_w = log_weights_unnorm;
  a.weights = weights;
  a.ess = ess;
  a.logZ = log_norm_const;
  return launch_tile(a, (hipStream_t)stream);
}

int smcdet_resample_index(const float* weights, int32_t T, int32_t N, int32_t method,
                          uint64_t seed, uint64_t offset, const float* u, int64_t* idx,
                          void* stream) {
  if (!weights || !idx) return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || N <= 0) return set_error(SMCDET_EUNSUPPORTED, "T=%d N=%d", T, N);
  if (method != SMCDET_RESAMPLE_MULTINOMIAL && method != SMCDET_RESAMPLE_SYSTEMATIC)
    return set_error(SMCDET_EINVAL, "unknown resample method %d", method);
  TileArgs a{};
  a.flags = kDoResample;
  a.T = T;
  a.N = N;
  a.weights = const_cast<float*>(weights);
  a.method = method;
  a.k0 = (uint32_t)seed;
  a.k1 = (uint32_t)(seed >> 32);
  a.offset = offset;
  a.u = u;
  a.idx = idx;
  return launch_tile(a, (hipStream_t)stream);
}

int smcdet_temper_reweight(const float* loglik, float* temperature, float* temperature_prev,
                           float* log_weights_unnorm, float* weights, float* ess,
                           float* log_norm_const, int32_t T, int32_t N, double ess_threshold,
                           int32_t resample_method, uint64_t seed, uint64_t offset, int64_t* idx,
                           void* stream) {
  if (!loglik || !temperature || !temperature_prev || !log_weights_unnorm || !weights || !ess ||
      !log_norm_const)
    return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || N <= 0) return set_error(SMCDET_EUNSUPPORTED, "T=%d N=%d", T, N);
  if (idx && resample_method != SMCDET_RESAMPLE_MULTINOMIAL &&
      resample_method != SMCDET_RESAMPLE_SYSTEMATIC)
    return set_error(SMCDET_EINVAL, "unknown resample method %d", resample_method);
  TileArgs a{};
  a.flags = kDoTemper | kDoWeights | (idx ? kDoResample : 0u);
  a.T = T;
  a.N = N;
  a.ess_threshold = ess_threshold;
  a.loglik = loglik;
  a.temperature = temperature;
  a.temperature_prev = temperature_prev;
  a.log_w = log_weights_unnorm;
  a.weights = weights;
  a.ess = ess;
  a.logZ = log_norm_const;
  a.method = resample_method;
  a.k0 = (uint32_t)seed;
  a.k1 = (uint32_t)(seed >> 32);
  a.offset = offset;
  a.idx = idx;
  return launch_tile(a, (hipStream_t)stream);
}

int smcdet_gather(const int64_t* idx, int32_t T, int32_t N, int32_t S, const float* counts_in,
                  const float* locs_in, const float* fluxes_in, float* counts_out,
                  float* locs_out, float* fluxes_out, void* stream) {
  if (!idx || !counts_in || !counts_out || (S > 0 && (!locs_in || !fluxes_in || !locs_out ||
                                                      !fluxes_out)))
    return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || N <= 0 || S < 0) return set_error(SMCDET_EUNSUPPORTED, "T=%d N=%d S=%d", T, N, S);
  if (counts_in == counts_out || locs_in == locs_out || fluxes_in == fluxes_out)
    return set_error(SMCDET_EINVAL, "gather needs distinct in/out buffers");
  const int64_t total = (int64_t)T * N * (S > 0 ? S : 1);
  hipLaunchKernelGGL(gather_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, idx, T, N, S, counts_in, locs_in, fluxes_in, counts_out,
                     locs_out, fluxes_out);
  return check_launch("smcdet_gather");
}

int smcdet_prune(const float* locs, const float* fluxes, int32_t T, int32_t N, int32_t S,
                 float tile_dim, float flux_threshold, int64_t* counts_out, float* locs_out,
                 float* fluxes_out, void* stream) {
  if (!locs || !fluxes || !counts_out || !locs_out || !fluxes_out)
    return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || N <= 0 || S < 0) return set_error(SMCDET_EUNSUPPORTED, "T=%d N=%d S=%d", T, N, S);
  if (locs == locs_out || fluxes == fluxes_out)
    return set_error(SMCDET_EINVAL, "prune needs distinct in/out buffers");
  const int64_t TN = (int64_t)T * N;
  hipLaunchKernelGGL(prune_kernel, dim3((unsigned)((TN + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, locs, fluxes, TN, S, tile_dim, flux_threshold,
                     counts_out, locs_out, fluxes_out);
  return check_launch("smcdet_prune");
}

}  // extern "C"
