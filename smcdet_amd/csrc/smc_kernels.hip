// smc_kernels.hip — per-tile SMC bookkeeping launches: temper / reweight /
// resample index (tile.h's tile_work, one 512-thread workgroup per tile; the
// reference copies the log-likelihoods to the host and runs scipy brentq per
// tile), gather, pruning (sampler.py:198-219), the CS-SMC count posterior and
// the aggregation temper / reweight kernels.
#include <math.h>
#include <stdlib.h>

#include <type_traits>

#include "tile.h"

namespace smcdet {


// One workgroup of NT threads per tile, on tile.h's 512-thread virtual
// layout, so either NT gives the same results bit for bit (the MH sweep's
// fused tail runs the same work on its 256 threads).  512 by default;
// SMCDET_TILE_THREADS=256 in the environment selects the 256-thread
// instantiation (A/B: fewer waves at each Brent barrier, two virtual threads
// per thread).
template <int NT, int PER>
__global__ __launch_bounds__(NT) void tile_kernel(TileArgs a) {
  if (a.go && *a.go == 0) return;  // speculatively enqueued iteration that must not run
  extern __shared__ float buf[];  // N floats: weights / cumsum, then N+1 resample slots
  __shared__ TileRed red;
  const int t = blockIdx.x;
  tile_work<NT, PER>(a, t, buf, red, threadIdx.x < kWave ? t : -1);
}

// 512 threads; the 256-thread tile kernel (measured slower)
// is the diagnostic build's A/B (SMCDET_TILE_THREADS=256)
static int tile_threads() {
#ifdef SMCDET_DIAG
  static const int nt = [] {
    const char* e = getenv("SMCDET_TILE_THREADS");
    return (e && atoi(e) == 256) ? 256 : 512;
  }();
  return nt;
#else
  return 512;
#endif
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

// ---------------------------------------------------------------------------
// CS-SMC combination (manuscript.tex:344-354): one workgroup per image tile.
// p(s|x) in double from the strata's log evidences and the count prior; the
// stratum of output catalog n by inverse CDF (same float64 arithmetic as the
// oracle, oracle/smc_oracle.py count_posterior_draw), then a uniform particle
// of that stratum, gathered straight to the output.
// ---------------------------------------------------------------------------
constexpr int kMaxStrata = 1024;

struct CountPostArgs {
  int T, NS, N, S, n_out, method;
  uint32_t k0, k1;
  uint64_t offset;
  const float* logZ;
  const float* lcp;          // [NS], or [T,NS] with lcp_per_tile
  int lcp_per_tile;
  const float* u_strata;
  const float* u_pick;
  const float* cin;
  const float* lin;
  const float* fin;
  float* probs;
  int64_t* idx;
  float* cout;
  float* lout;
  float* fout;
};

__global__ __launch_bounds__(256) void count_posterior_kernel(CountPostArgs a) {
  __shared__ double cdf[kMaxStrata];
  __shared__ double U;
  const int t = blockIdx.x;
  const int NS = a.NS;
  const float* lcp = a.lcp + (a.lcp_per_tile ? (size_t)t * NS : 0);
  if (threadIdx.x == 0) {
    double m = -INFINITY;
    for (int k = 0; k < NS; ++k)
      m = fmax(m, (double)a.logZ[(size_t)t * NS + k] + (double)lcp[k]);
    double s = 0.0;
    for (int k = 0; k < NS; ++k) s += exp((double)a.logZ[(size_t)t * NS + k] + (double)lcp[k] - m);
    double c = 0.0;
    for (int k = 0; k < NS; ++k) {
      const double p = exp((double)a.logZ[(size_t)t * NS + k] + (double)lcp[k] - m) / s;
      a.probs[(size_t)t * NS + k] = (float)p;
      c += p;
      cdf[k] = c;
    }
    if (a.method == SMCDET_RESAMPLE_SYSTEMATIC) {
      if (a.u_strata) {
        U = (double)a.u_strata[t];
      } else {
        const U4 r = philox4x32((uint32_t)a.offset, (uint32_t)(a.offset >> 32), (uint32_t)t,
                                kTagStrata, a.k0, a.k1);
        U = (double)u01(r.y);
      }
    }
  }
  __syncthreads();
  const int N = a.N, S = a.S;
  for (int n = threadIdx.x; n < a.n_out; n += blockDim.x) {
    const size_t on = (size_t)t * a.n_out + n;
    const uint64_t c = a.offset + (uint64_t)n;
    U4 r{0u, 0u, 0u, 0u};
    if (!a.u_strata || !a.u_pick)
      r = philox4x32((uint32_t)c, (uint32_t)(c >> 32), (uint32_t)t, kTagStrata + 1, a.k0, a.k1);
    double u;
    if (a.method == SMCDET_RESAMPLE_SYSTEMATIC) u = ((double)n + U) / (double)a.n_out;
    else u = a.u_strata ? (double)a.u_strata[on] : (double)u01(r.x);
    int k = 0;
    while (k < NS - 1 && cdf[k] < u) ++k;
    const float v = a.u_pick ? a.u_pick[on] : u01(r.y);
    const int m = min((int)(v * (float)N), N - 1);
    a.idx[on] = (int64_t)k * N + m;
    const size_t src = ((size_t)t * NS + k) * N + m;
    a.cout[on] = a.cin[src];
    for (int s = 0; s < S; ++s) {
      a.lout[(on * S + s) * 2 + 0] = a.lin[(src * S + s) * 2 + 0];
      a.lout[(on * S + s) * 2 + 1] = a.lin[(src * S + s) * 2 + 1];
      a.fout[on * S + s] = a.fin[src * S + s];
    }
  }
}

// ---------------------------------------------------------------------------
// Tile aggregation (smcdet/aggregate.py:140-174 temper, :439-483
// update_weights, :485-521 resample_intracount): the particles of a joint
// tile are sorted by count, and each count group ("segment": tile, first
// particle, length) is its own SMC population.  One 512-thread workgroup per
// segment: pass A solves the segment's tempering increment with the same
// Brent iteration as tile_kernel (ESS target ess_prop * group size); the
// tile's increment is the minimum over its segments (a scatter-min by the
// caller); pass B reweights each segment at the new temperature (softmax
// within the group, log evidence of the group) and draws the intracount
// multinomial resampling indices for the next iteration.  The
// log-likelihood increment is loglik_parent - loglik_children (:539-541).
// ---------------------------------------------------------------------------
struct AggTileArgs {
  int T, N, G;
  double ess_prop;
  const float* ll_parent;   // [T,N]
  const float* ll_child;    // [T,N]
  const int32_t* seg_tile;  // [G]
  const int32_t* seg_start; // [G] first particle (within the tile)
  const int32_t* seg_len;   // [G]
  const float* temperature; // [T]
  const float* temperature_prev; // [T]
  float* delta;             // [G]
  float* log_w;             // [T,N]
  float* w_intra;           // [T,N]
  float* lnc;               // [G] in/out
  float* ess;               // [G]
  uint32_t k0, k1;
  uint64_t offset;
  const float* u;           // [T,N] replayed uniforms or null
  int64_t* idx;             // [T,N] or null (tile-local particle indices)
};

// the segment's (tile, first particle, length), clamped into [0,T) x [0,N)
__device__ __forceinline__ void agg_segment(const AggTileArgs& a, int g, int& t, int& s0,
                                            int& n) {
  t = min(max(a.seg_tile[g], 0), a.T - 1);
  s0 = min(max(a.seg_start[g], 0), a.N);
  n = min(max(a.seg_len[g], 0), a.N - s0);
}

template <int PER>
__global__ __launch_bounds__(kTB) void agg_temper_kernel(AggTileArgs a) {
  __shared__ TileRed red;
  int parity = 0;
  const int g = blockIdx.x;
  int t, s0, n;
  agg_segment(a, g, t, s0, n);
  if (n == 0) {
    if (threadIdx.x == 0) a.delta[g] = 1.0f;  // an empty group imposes nothing
    return;
  }
  const size_t base = (size_t)t * a.N + s0;
  TileLL<kTB, PER> ll;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = threadIdx.x + j * kTB;
    ll.l[0][j] = ll.valid(0, j, n) ? a.ll_parent[base + i] - a.ll_child[base + i] : 0.f;
  }
  float lm = -INFINITY;
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (ll.valid(0, j, n)) lm = fmaxf(lm, ll.l[0][j]);
  lm = block_max(lm, &red, parity);
  const double thr = a.ess_prop * (double)n;
  auto f = [&](double x) { return block_ess_objective(ll, n, lm, x, thr, &red, parity); };
  const double top = 1.0 - (double)a.temperature[t];
  const double ftop = f(top);
  double delta = top;
  if (ftop < 0.0) delta = block_brentq(f, 0.0, top, (double)n - thr, ftop);
  if (threadIdx.x == 0) a.delta[g] = (float)delta;
}

// inclusive cumsum of buf[0..n) in place: float64 running sum rounded per
// element to float32 (torch's CPU cumsum), contiguous chunk per thread
__device__ __forceinline__ void block_cumsum(float* buf, int n, TileRed* red, int& parity) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int chunk = (n + kTB - 1) / kTB;
  const int b0 = min((int)threadIdx.x * chunk, n), b1 = min(b0 + chunk, n);
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
  if (lane == 63) red->d[k][wave][0] = incl;
  __syncthreads();
  double run = incl - part;
  for (int i = 0; i < wave; ++i) run += red->d[k][i][0];
  for (int i = b0; i < b1; ++i) {
    run += (double)buf[i];
    buf[i] = (float)run;
  }
  __syncthreads();
}

__global__ __launch_bounds__(kTB) void agg_reweight_kernel(AggTileArgs a) {
  extern __shared__ float buf[];  // n floats
  __shared__ TileRed red;
  int parity = 0;
  const int g = blockIdx.x;
  int t, s0, n;
  agg_segment(a, g, t, s0, n);
  // temperature - temperature_prev, float32 tensors (aggregate.py:440-442)
  const float d = a.temperature[t] - a.temperature_prev[t];
  if (n == 0) return;
  const size_t base = (size_t)t * a.N + s0;
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < n; i += kTB) {
    const float e = d * (a.ll_parent[base + i] - a.ll_child[base + i]);
    a.log_w[base + i] = e;
    buf[i] = e;
    mx = fmaxf(mx, e);
  }
  mx = block_max(mx, &red, parity);
  double s = 0.0, unused = 0.0;
  for (int i = threadIdx.x; i < n; i += kTB) {
    const float e = expf(buf[i] - mx);
    buf[i] = e;
    s += (double)e;
  }
  block_sum2(s, unused, &red, parity);
  const float sf = (float)s;
  double q = 0.0;
  for (int i = threadIdx.x; i < n; i += kTB) {
    const float w = buf[i] / sf;  // softmax within the group (:452-454)
    a.w_intra[base + i] = w;
    buf[i] = w;
    q += (double)w * (double)w;
  }
  block_sum2(q, unused, &red, parity);
  if (threadIdx.x == 0) {
    a.ess[g] = (float)(1.0 / q);
    // (wt - wt.max()).exp().mean().log() + wt.max(), added to the group's log Z (:456-465)
    a.lnc[g] = a.lnc[g] + (logf(sf / (float)n) + mx);
  }
  if (!a.idx) return;
  // ---- intracount multinomial resampling (:506-515), tile-local indices -----
  block_cumsum(buf, n, &red, parity);
  const float total = buf[n - 1];
  for (int i = threadIdx.x; i < n; i += kTB) {
    float un;
    if (a.u) {
      un = a.u[base + i];
    } else {
      const uint64_t c = a.offset + (uint64_t)(s0 + i);
      const U4 r = philox4x32((uint32_t)c, (uint32_t)(c >> 32), (uint32_t)t, kTagAggResample,
                              a.k0, a.k1);
      un = u01(r.x);
    }
    const float target = un * total;
    int lo = 0, hi = n;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (buf[mid] > target) hi = mid; else lo = mid + 1;
    }
    a.idx[base + i] = (int64_t)(s0 + min(lo, n - 1));
  }
}

int launch_tile(const TileArgs& a, hipStream_t st) {
  if (a.N > kMaxN)
    return set_error(SMCDET_EUNSUPPORTED, "N=%d particles per tile > %d", a.N, kMaxN);
  // weights / bins, then (systematic resampling) N+1 slots
  const size_t lds = (size_t)(2 * a.N + 1) * sizeof(float);
  const int per = (a.N + kTB - 1) / kTB;
  const int nt = tile_threads();
  auto pick = [per](auto NT) -> const void* {
    constexpr int n = decltype(NT)::value;
    return per <= 1 ? (const void*)tile_kernel<n, 1>
         : per <= 2 ? (const void*)tile_kernel<n, 2>
         : per <= 4 ? (const void*)tile_kernel<n, 4>
         : per <= 8 ? (const void*)tile_kernel<n, 8>
         : per <= 16 ? (const void*)tile_kernel<n, 16>
                     : (const void*)tile_kernel<n, 32>;
  };
#ifdef SMCDET_DIAG
  const void* fn = nt == 256 ? pick(std::integral_constant<int, 256>{})
                             : pick(std::integral_constant<int, 512>{});
#else
  (void)nt;
  const void* fn = pick(std::integral_constant<int, 512>{});
#endif
  int rc = ensure_lds(fn, lds + sizeof(TileRed));
  if (rc) return rc;
  void* args[] = {const_cast<TileArgs*>(&a)};
  hipError_t e;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (timing_tiles() && timing_next(&e0, &e1))  // events on the dispatch packet (launch_sweep)
    e = hipExtLaunchKernel(fn, dim3(a.T), dim3(nt), args, lds, st, e0, e1, 0);
  else
    e = hipLaunchKernel(fn, dim3(a.T), dim3(nt), args, lds, st);
  if (e != hipSuccess) return set_error(SMCDET_EHIP, "tile kernel launch: %s", hipGetErrorString(e));
  return check_launch("smcdet tile kernel");
}

// bins -> indices: one wave per particle (bins_ancestor), 4 per workgroup
__global__ __launch_bounds__(256) void bins_index_kernel(const float* __restrict__ bins, int T,
                                                         int N, int64_t* __restrict__ idx) {
  const int t = blockIdx.y;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  const float* coarse = bins + (size_t)T * (N + 1) + (size_t)t * kBinsCoarse;
  const int a = bins_ancestor(bins + (size_t)t * N, coarse, N, bins[(size_t)T * N + t], n);
  if ((threadIdx.x & 63) == 0) idx[(size_t)t * N + n] = a;
}

}  // namespace smcdet

using namespace smcdet;

SMCDET_TRACE_READER(smcdet_trace_read_tile)

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
                           uint32_t flags, int32_t* finished_iter, int32_t iter, int32_t* live,
                           const int32_t* go, int32_t* live_host, void* stream) {
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
  a.smc_flags = flags;
  a.fin_iter = finished_iter;
  a.iter = iter;
  if ((uintptr_t)live & 7) return set_error(SMCDET_EINVAL, "live must be 8-byte aligned");
  a.live = live;
  a.go = go;
  a.live_host = live ? live_host : nullptr;
  return launch_tile(a, (hipStream_t)stream);
}

int smcdet_bins_index(const float* bins, int32_t T, int32_t N, int64_t* idx, void* stream) {
  if (!bins || !idx) return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || N <= 0 || T > 65535) return set_error(SMCDET_EUNSUPPORTED, "T=%d N=%d", T, N);
  hipLaunchKernelGGL(bins_index_kernel, dim3((unsigned)((N + 3) / 4), (unsigned)T), dim3(256), 0,
                     (hipStream_t)stream, bins, T, N, idx);
  return check_launch("smcdet_bins_index");
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

int smcdet_count_posterior(const float* log_norm_const, const float* log_count_prior,
                           int32_t lcp_per_tile, int32_t T, int32_t NS, int32_t N, int32_t S,
                           int32_t n_out,
                           int32_t resample_method, uint64_t seed, uint64_t offset,
                           const float* u_strata, const float* u_pick, const float* counts_in,
                           const float* locs_in, const float* fluxes_in, float* probs,
                           int64_t* idx, float* counts_out, float* locs_out, float* fluxes_out,
                           void* stream) {
  if (!log_norm_const || !log_count_prior || !counts_in || !probs || !idx || !counts_out ||
      (S > 0 && (!locs_in || !fluxes_in || !locs_out || !fluxes_out)))
    return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || T > 65535 || N <= 0 || n_out <= 0 || S < 0 || NS <= 0 || NS > kMaxStrata)
    return set_error(SMCDET_EUNSUPPORTED, "T=%d NS=%d N=%d S=%d n_out=%d", T, NS, N, S, n_out);
  if (resample_method != SMCDET_RESAMPLE_MULTINOMIAL &&
      resample_method != SMCDET_RESAMPLE_SYSTEMATIC)
    return set_error(SMCDET_EINVAL, "unknown resample method %d", resample_method);
  if ((u_strata == nullptr) != (u_pick == nullptr))
    return set_error(SMCDET_EINVAL, "u_strata and u_pick must be given together");
  CountPostArgs a{};
  a.T = T;
  a.NS = NS;
  a.N = N;
  a.S = S;
  a.n_out = n_out;
  a.method = resample_method;
  a.k0 = (uint32_t)seed;
  a.k1 = (uint32_t)(seed >> 32);
  a.offset = offset;
  a.logZ = log_norm_const;
  a.lcp = log_count_prior;
  a.lcp_per_tile = lcp_per_tile != 0;
  a.u_strata = u_strata;
  a.u_pick = u_pick;
  a.cin = counts_in;
  a.lin = locs_in;
  a.fin = fluxes_in;
  a.probs = probs;
  a.idx = idx;
  a.cout = counts_out;
  a.lout = locs_out;
  a.fout = fluxes_out;
  hipLaunchKernelGGL(count_posterior_kernel, dim3(T), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("smcdet_count_posterior");
}

static int agg_tile_common(AggTileArgs& a, const float* loglik_parent,
                           const float* loglik_children, const float* temperature, int32_t T,
                           int32_t N, int32_t G, const int32_t* seg_tile,
                           const int32_t* seg_start, const int32_t* seg_len) {
  if (!loglik_parent || !loglik_children || !temperature || !seg_tile || !seg_start || !seg_len)
    return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || N <= 0 || G <= 0 || G > 65535 * 64)
    return set_error(SMCDET_EUNSUPPORTED, "T=%d N=%d G=%d", T, N, G);
  if (N > kMaxN) return set_error(SMCDET_EUNSUPPORTED, "N=%d particles per tile > %d", N, kMaxN);
  a.T = T;
  a.N = N;
  a.G = G;
  a.ll_parent = loglik_parent;
  a.ll_child = loglik_children;
  a.temperature = temperature;
  a.seg_tile = seg_tile;
  a.seg_start = seg_start;
  a.seg_len = seg_len;
  return SMCDET_OK;
}

int smcdet_aggregate_temper(const float* loglik_parent, const float* loglik_children,
                            const float* temperature, int32_t T, int32_t N, int32_t G,
                            const int32_t* seg_tile, const int32_t* seg_start,
                            const int32_t* seg_len, double ess_threshold_prop, float* delta,
                            void* stream) {
  AggTileArgs a{};
  int rc = agg_tile_common(a, loglik_parent, loglik_children, temperature, T, N, G, seg_tile,
                           seg_start, seg_len);
  if (rc) return rc;
  if (!delta) return set_error(SMCDET_EINVAL, "null buffer");
  a.ess_prop = ess_threshold_prop;
  a.delta = delta;
  const int per = (N + kTB - 1) / kTB;
  const void* fn = per <= 1 ? (const void*)agg_temper_kernel<1>
                 : per <= 2 ? (const void*)agg_temper_kernel<2>
                 : per <= 4 ? (const void*)agg_temper_kernel<4>
                 : per <= 8 ? (const void*)agg_temper_kernel<8>
                 : per <= 16 ? (const void*)agg_temper_kernel<16>
                             : (const void*)agg_temper_kernel<32>;
  void* args[] = {&a};
  hipError_t e = hipLaunchKernel(fn, dim3(G), dim3(kTB), args, 0, (hipStream_t)stream);
  if (e != hipSuccess)
    return set_error(SMCDET_EHIP, "aggregate temper launch: %s", hipGetErrorString(e));
  return check_launch("smcdet_aggregate_temper");
}

int smcdet_aggregate_reweight(const float* loglik_parent, const float* loglik_children,
                              const float* temperature, const float* temperature_prev, int32_t T,
                              int32_t N, int32_t G, const int32_t* seg_tile,
                              const int32_t* seg_start, const int32_t* seg_len,
                              float* log_weights_unnorm, float* weights_intracount,
                              float* log_norm_const, float* ess, uint64_t seed, uint64_t offset,
                              const float* u, int64_t* idx, void* stream) {
  AggTileArgs a{};
  int rc = agg_tile_common(a, loglik_parent, loglik_children, temperature, T, N, G, seg_tile,
                           seg_start, seg_len);
  if (rc) return rc;
  if (!temperature_prev || !log_weights_unnorm || !weights_intracount || !log_norm_const || !ess)
    return set_error(SMCDET_EINVAL, "null buffer");
  a.temperature_prev = temperature_prev;
  a.log_w = log_weights_unnorm;
  a.w_intra = weights_intracount;
  a.lnc = log_norm_const;
  a.ess = ess;
  a.k0 = (uint32_t)seed;
  a.k1 = (uint32_t)(seed >> 32);
  a.offset = offset;
  a.u = u;
  a.idx = idx;
  const size_t lds = (size_t)N * sizeof(float);
  rc = ensure_lds((const void*)agg_reweight_kernel, lds + sizeof(TileRed));
  if (rc) return rc;
  hipLaunchKernelGGL(agg_reweight_kernel, dim3(G), dim3(kTB), lds, (hipStream_t)stream, a);
  return check_launch("smcdet_aggregate_reweight");
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
