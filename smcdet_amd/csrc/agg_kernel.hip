// agg_kernel.hip — the MH sweep of the tile-aggregation SMC
// (smcdet/aggregate.py:105-130 log_target, :176-187 mutate through
// smcdet/kernel.py:26-130 SingleComponentMH.run).
//
// A joint tile (two neighbouring tiles joined along `axis`, aggregate.py:217-263)
// is sampled under the bridging target
//   log pi_tau(z) = log p(z) + (1 - tau) * [l_c1(z_1) + l_c2(z_2)] + tau * l_p(z)
// where l_p is the image log-likelihood of the joint tile rendered from every
// source and l_c1 / l_c2 those of the two child halves, each rendered only from
// the sources whose axis coordinate puts them in that half (unjoin,
// aggregate.py:265-324: loc_axis <= dim/2 -> first child).  Pixel p of the
// joint tile lies in exactly one child, so the children's log-likelihoods sum
// to the pixel sum over a "child composite" rate image lamC, in which pixel p
// only receives the sources of p's own half.  One particle per wave keeps both
// rate images (lamP, lamC) in LDS; a move of source j from half A to half B
// changes lamP by dl = g f' psf_new - g f psf_old over the union of its PSF
// windows, and lamC by the new term on B's pixels minus the old term on A's.
//
// Differences from the fixed-count sweep (mh_kernel.hip), by design:
//   * the catalog lives in LDS ([S][3] floats per wave), not one source per
//     lane: joint tiles hold up to SMCDET_AGG_MAX_SOURCES sources;
//   * the moved component is drawn from 0..count-1 (count-grouped
//     populations padded to S sources, zero flux past the count);
//   * every sweep starts from a fresh render of both images, and the returned
//     log-likelihoods (parent and children) come from a fresh render of the
//     final state, so the tempering weights carry no incremental drift.
// Accept rule, truncated-normal proposals and the upper-edge freeze are the
// fixed-count sweep's (kernel.py:114-125).
#include <math.h>

#include "render.h"

namespace smcdet {

constexpr int kAggMaxWaves = 4;

// Normal(mu, 1/isig): Phi(lb) and the log-mass in the box (distributions.py:33-35)
__device__ __forceinline__ void phl_lz(float mu, float isig, float lb, float ub, float& phl,
                                       float& lZ) {
  phl = normal_cdf(lb, mu, isig);
  lZ = nan_to_num(fast_log(normal_cdf(ub, mu, isig) - phl), 0.0f);
}

struct AggArgs {
  DevModel m;  // joint tile: m.H x m.W
  DevPrior pr;
  int K, T, N, S;
  int axis;        // 0: children stacked along h, 1: along w
  int halfpix;     // pixels with coordinate < halfpix belong to the first child
  float half;      // sources with coordinate <= half belong to the first child
  float sl, isl, sf, isf;
  float lb_h, lb_w, ub_h, ub_w, lb_f, ub_f;
  uint32_t k0, k1;
  uint64_t offset;
  int nw;          // waves (particles) per workgroup
  const float* img;
  const float* temperature;
  const int64_t* ancestors;
  const float* counts_in;
  const float* locs_in;
  const float* fluxes_in;
  float* counts_out;
  float* locs_out;
  float* fluxes_out;
  float* ll_parent;
  float* ll_child;
  int32_t* acc_count;
  float* acc_rate;
  const float* boxes;  // [T,4] per-joint-tile location boxes (or null)
  const int32_t* r_comp;
  const float* r_uloc;
  const float* r_uflux;
  const float* r_uacc;
  float* work;         // GL: per-particle [2*H*W + 3*S] scratch (rate images, catalog)
};

// Both rate images from the LDS catalog: lamP = B + sum_s g f_s psf_s,
// lamC = B + sum over the sources of each pixel's own half.
template <int MODEL>
__device__ __forceinline__ void agg_render(const AggArgs& a, float* lamP, float* lamC,
                                           const float* cat, int lane) {
  const DevModel& m = a.m;
  const int HW = m.H * m.W;
  for (int p = lane; p < HW; p += kWave) {
    lamP[p] = m.bg;
    lamC[p] = m.bg;
  }
  wave_sync();
  const float scale = m.g * psf_scale<MODEL>(m);
  for (int s = 0; s < a.S; ++s) {
    const float h = cat[3 * s], w = cat[3 * s + 1], f = cat[3 * s + 2];
    if (f == 0.0f) continue;  // empty slot (wave-uniform)
    const int fh = ifloor_clamped(h), fw = ifloor_clamped(w);
    const int r0 = max(fh - m.R, 0), r1 = min(fh + m.R, m.H - 1);
    const int c0 = max(fw - m.R, 0), c1 = min(fw + m.R, m.W - 1);
    if (r0 > r1 || c0 > c1) continue;
    const int bw = c1 - c0 + 1, npos = (r1 - r0 + 1) * bw;
    const float inv_bw = 1.0f / (float)bw;
    const float amp = scale * f;
    const int side = ((a.axis == 0 ? h : w) > a.half) ? 1 : 0;
    for (int q = lane; q < npos; q += kWave) {
      const int aa = (int)(((float)q + 0.5f) * inv_bw);
      const int ph = r0 + aa, pw = c0 + (q - aa * bw);
      const float dh = ((float)ph + 0.5f) - h, dw = ((float)pw + 0.5f) - w;
      const float v = amp * psf_raw<MODEL>(m, fmaf(dh, dh, dw * dw));
      const int p = ph * m.W + pw;
      lamP[p] += v;
      const int pside = ((a.axis == 0 ? ph : pw) >= a.halfpix) ? 1 : 0;
      if (pside == side) lamC[p] += v;
    }
    wave_sync();
  }
}

// One union-window position of a move (h, w, amp_o) -> (hn, wn, amp_n): the
// parent and child-composite rate changes at pixel (ph, pw).
template <int MODEL>
__device__ __forceinline__ void agg_position(const AggArgs& a, int ph, int pw, float h, float w,
                                             float hn, float wn, int fh0, int fw0, int fh1,
                                             int fw1, float amp_o, float amp_n, int side_o,
                                             int side_n, float& dlP, float& dlC) {
  const DevModel& m = a.m;
  const float fph = (float)ph + 0.5f, fpw = (float)pw + 0.5f;
  const float dho = fph - h, dwo = fpw - w, dhn = fph - hn, dwn = fpw - wn;
  const unsigned span = 2u * (unsigned)m.R;
  const bool in_o = (unsigned)(ph - fh0 + m.R) <= span && (unsigned)(pw - fw0 + m.R) <= span;
  const bool in_n = (unsigned)(ph - fh1 + m.R) <= span && (unsigned)(pw - fw1 + m.R) <= span;
  const float vo = in_o ? amp_o * psf_raw<MODEL>(m, fmaf(dho, dho, dwo * dwo)) : 0.f;
  const float vn = in_n ? amp_n * psf_raw<MODEL>(m, fmaf(dhn, dhn, dwn * dwn)) : 0.f;
  dlP = vn - vo;
  const int pside = ((a.axis == 0 ? ph : pw) >= a.halfpix) ? 1 : 0;
  dlC = (pside == side_n ? vn : 0.f) - (pside == side_o ? vo : 0.f);
}

// GL: joint tiles above the LDS budget -- tile image read from global memory,
// both rate images and the catalog in the caller's workspace (row per particle)
template <int MODEL, bool REPLAY, bool GL = false>
__global__ __launch_bounds__(kAggMaxWaves* kWave) void agg_sweep_kernel(AggArgs a) {
  extern __shared__ float smem[];
  __shared__ int wg_acc, wg_done;
  const DevModel& m = a.m;
  const int HW = m.H * m.W;
  const int HWp = HW + kWave;
  const int t = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int kImg = (MODEL == SMCDET_MODEL_POISSON) ? 2 : 1;
  float* xs = smem;
  float* lg = smem + HWp;
  const int per_wave = 2 * HWp + 3 * a.S;
  float* lamP = smem + kImg * HWp + wave * per_wave;
  float* lamC = lamP + HWp;
  float* cat = lamC + HWp;
  if constexpr (GL) {
    xs = const_cast<float*>(a.img) + (size_t)t * HW;
    lg = nullptr;
  } else {
    stage_image<MODEL>(a.img + (size_t)t * HW, xs, lg, HW, threadIdx.x, a.nw * kWave);
  }
  if (threadIdx.x == 0) {
    wg_acc = 0;
    wg_done = 0;
  }
  __syncthreads();
  const int n = blockIdx.x * a.nw + wave;
  if (n >= a.N) return;

  const int N = a.N, S = a.S;
  const size_t pid = (size_t)t * N + n;
  const size_t src = a.ancestors ? (size_t)t * N + (size_t)a.ancestors[pid] : pid;
  if constexpr (GL) {
    lamP = a.work + pid * (2 * (size_t)HW + 3 * (size_t)S);
    lamC = lamP + HW;
    cat = lamC + HW;
  }
  const float count = a.counts_in[src];
  if (a.counts_out && lane == 0) a.counts_out[pid] = count;
  const int Sj = min(max((int)count, 0), S);
  const float tau = a.temperature[t];
  const int K = Sj > 0 ? a.K : 0;
  for (int s = lane; s < S; s += kWave) {
    cat[3 * s] = a.locs_in[(src * S + s) * 2 + 0];
    cat[3 * s + 1] = a.locs_in[(src * S + s) * 2 + 1];
    cat[3 * s + 2] = a.fluxes_in[src * S + s];
  }
  wave_sync();
  agg_render<MODEL>(a, lamP, lamC, cat, lane);

  // lane d < 3 proposes dimension d (h, w, flux); lanes >= 3 shadow dimension 2
  const int d = min(lane, 2);
  const float isig = d < 2 ? a.isl : a.isf, sig = d < 2 ? a.sl : a.sf;
  float lb = d == 0 ? a.lb_h : (d == 1 ? a.lb_w : a.lb_f);
  float ub = d == 0 ? a.ub_h : (d == 1 ? a.ub_w : a.ub_f);
  if (a.boxes && d < 2) {  // the joint tile's own box (partition of the padded image)
    lb = a.boxes[4 * t + d];
    ub = a.boxes[4 * t + 2 + d];
  }
  const float scale = m.g * psf_scale<MODEL>(m);
  const float omt = 1.0f - tau;

  float ru0 = 0.f, ru1 = 0.f, ru2 = 0.f, ru3 = 0.f, ru4 = 0.f;
  int rcomp = 0;
  int accept = 0;
  for (int k = 0; k < K; ++k) {
    const int kl = k & 63;
    if (kl == 0) {  // draws of iterations k..k+63, lane i holds iteration k+i
      const int kk = k + lane;
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
        const U4 r0 = philox4x32(c0, c1, (uint32_t)pid, kTagAgg0, a.k0, a.k1);
        const U4 r1 = philox4x32(c0, c1, (uint32_t)pid, kTagAgg1, a.k0, a.k1);
        ru0 = u01(r0.x);
        ru1 = u01(r0.y);
        ru2 = u01(r0.z);
        ru3 = u01(r0.w);
        ru4 = u01(r1.x);
      }
    }
    int j;
    if constexpr (REPLAY) j = min(max(readlane(rcomp, kl), 0), Sj - 1);
    else j = min((int)(readlane(ru0, kl) * (float)Sj), Sj - 1);
    const float u = d == 0 ? readlane(ru1, kl) : (d == 1 ? readlane(ru2, kl) : readlane(ru3, kl));
    const float log_u = fast_log(readlane(ru4, kl));

    // ---- proposal (distributions.py:40-48) and Hastings + prior terms -------
    const float mu = cat[3 * j + d];
    float c_ph, c_lZ, n_ph, n_lZ;
    phl_lz(mu, isig, lb, ub, c_ph, c_lZ);
    const float pc = fminf(fmaxf(u, 1e-6f), 0.999999f);
    float pt = c_ph + pc * fast_exp(c_lZ);
    pt = fminf(fmaxf(pt, 1e-6f), 0.999999f);
    float xn = mu + sig * erfinv_fast(2.0f * pt - 1.0f) * kSqrt2;
    xn = fminf(fmaxf(xn, lb), ub);
    phl_lz(xn, isig, lb, ub, n_ph, n_lZ);
    float hd = c_lZ - n_lZ;
    // a location clamped onto the box's upper edge has log prior -inf
    // (Uniform.log_prob(high)): rejected, and the reference's cached NaN
    // target freezes the particle for the rest of the sweep (kernel.py:125)
    if (d < 2 && xn >= ub) hd = -INFINITY;
    // flux prior term (prior.py:220-226 / :183-189): -(alpha+1) log(f'/f)
    if (d == 2) hd += -a.pr.ap1 * (fast_log(xn) - fast_log(mu));
    const float h = readlane(mu, 0), w = readlane(mu, 1), f = readlane(mu, 2);
    const float hn = readlane(xn, 0), wn = readlane(xn, 1), fn = readlane(xn, 2);
    const float hast = (readlane(hd, 0) + readlane(hd, 1)) + readlane(hd, 2);

    // ---- parent / child-composite log-likelihood changes over the union window
    const int fh0 = ifloor16(h), fw0 = ifloor16(w), fh1 = ifloor16(hn), fw1 = ifloor16(wn);
    const int r0 = max(min(fh0, fh1) - m.R, 0), r1 = min(max(fh0, fh1) + m.R, m.H - 1);
    const int c0 = max(min(fw0, fw1) - m.R, 0), c1 = min(max(fw0, fw1) + m.R, m.W - 1);
    const int bw = max(c1 - c0 + 1, 1);
    const int npos = (r1 >= r0 && c1 >= c0) ? (r1 - r0 + 1) * bw : 0;
    const float inv_bw = 1.0f / (float)bw;
    const float amp_o = scale * f, amp_n = scale * fn;
    const int side_o = ((a.axis == 0 ? h : w) > a.half) ? 1 : 0;
    const int side_n = ((a.axis == 0 ? hn : wn) > a.half) ? 1 : 0;
    float eP = 0.f, eC = 0.f;
    for (int q = lane; q < npos; q += kWave) {
      const int aa = (int)(((float)q + 0.5f) * inv_bw);
      const int ph = r0 + aa, pw = c0 + (q - aa * bw);
      float dlP, dlC;
      agg_position<MODEL>(a, ph, pw, h, w, hn, wn, fh0, fw0, fh1, fw1, amp_o, amp_n, side_o,
                          side_n, dlP, dlC);
      const int p = ph * m.W + pw;
      const float x = xs[p];
      const float lgx = (MODEL == SMCDET_MODEL_POISSON) ? lg[p] : 0.0f;
      eP += pix_delta<MODEL>(m, x, lgx, lamP[p], dlP);
      eC += (dlC != 0.f) ? pix_delta<MODEL>(m, x, lgx, lamC[p], dlC) : 0.f;
    }
    const float dllP = wave_sum(eP), dllC = wave_sum(eC);

    // ---- accept / reject (kernel.py:114-122) --------------------------------
    const float loga = hast + fmaf(omt, dllC, tau * dllP);
    accept = __builtin_amdgcn_readfirstlane((loga >= log_u) ? 1 : 0);
    if (hast == -INFINITY) break;  // edge hit: rejected, the sweep is over
    if (accept) {
      for (int q = lane; q < npos; q += kWave) {
        const int aa = (int)(((float)q + 0.5f) * inv_bw);
        const int ph = r0 + aa, pw = c0 + (q - aa * bw);
        float dlP, dlC;
        agg_position<MODEL>(a, ph, pw, h, w, hn, wn, fh0, fw0, fh1, fw1, amp_o, amp_n, side_o,
                            side_n, dlP, dlC);
        const int p = ph * m.W + pw;
        lamP[p] += dlP;
        lamC[p] += dlC;
      }
      if (lane < 3) cat[3 * j + lane] = xn;
      wave_sync();
    }
  }

  // ---- write back; log-likelihoods of a fresh render of the final state ------
  for (int s = lane; s < S; s += kWave) {
    a.locs_out[(pid * S + s) * 2 + 0] = cat[3 * s];
    a.locs_out[(pid * S + s) * 2 + 1] = cat[3 * s + 1];
    a.fluxes_out[pid * S + s] = cat[3 * s + 2];
  }
  if (a.ll_parent || a.ll_child) {
    if (K > 0) agg_render<MODEL>(a, lamP, lamC, cat, lane);
    const double lp = pixel_sum<MODEL>(m, xs, lg, lamP, nullptr, lane);
    const double lc = pixel_sum<MODEL>(m, xs, lg, lamC, nullptr, lane);
    if (lane == 0) {
      if (a.ll_parent) a.ll_parent[pid] = (float)lp;
      if (a.ll_child) a.ll_child[pid] = (float)lc;
    }
  }
  // ---- acceptance rate of the last iteration (kernel.py:130), per tile ------
  if (lane == 0 && a.acc_rate) {
    const int nw = min(a.nw, N - (int)blockIdx.x * a.nw);
    if (accept && a.K > 0) atomicAdd(&wg_acc, 1);
    __threadfence_block();
    if (atomicAdd(&wg_done, 1) == nw - 1) {
      int32_t* cnt = a.acc_count + t;
      int32_t* ticket = a.acc_count + a.T + t;
      atomicAdd(cnt, atomicAdd(&wg_acc, 0));
      __threadfence();
      if (atomicAdd(ticket, 1) == (int)gridDim.x - 1) {
        const int total = atomicExch(cnt, 0);
        atomicExch(ticket, 0);
        a.acc_rate[t] = (float)total / (float)N;
      }
    }
  }
}

}  // namespace smcdet

using namespace smcdet;

// fewest waves per workgroup the LDS aggregation sweep runs with (above: the
// workspace variant, M71 only)
static int agg_min_lds_waves(int model) { return model == SMCDET_MODEL_M71 ? 2 : 1; }

extern "C" int64_t smcdet_aggregate_workspace(const smcdet_image_model_t* model, int32_t T,
                                              int32_t N, int32_t S) {
  int rc = validate_model(model, kMaxGlobalPixels);
  if (rc) return rc;
  if (T <= 0 || N <= 0 || T > 65535) return set_error(SMCDET_EUNSUPPORTED, "T=%d N=%d", T, N);
  if (S < 1 || S > SMCDET_AGG_MAX_SOURCES)
    return set_error(SMCDET_EUNSUPPORTED, "S=%d outside 1..%d", S, SMCDET_AGG_MAX_SOURCES);
  const size_t HWp = (size_t)model->H * model->W + kWave;
  const size_t img_b = (model->model == SMCDET_MODEL_POISSON ? 2 : 1) * HWp * sizeof(float);
  const size_t wave_b = (2 * HWp + 3 * (size_t)S) * sizeof(float);
  // LDS path at the largest wave count (4..kAggMinLdsWaves) whose workgroup
  // fits; the workspace only beyond that (M71: the global-memory variant
  // keeps 4 waves per workgroup where LDS would hold one, i.e. one wave per
  // CU; the Poisson model has no such variant and goes down to one wave)
  if (img_b + agg_min_lds_waves(model->model) * wave_b <= 160 * 1024) return 0;
  if (model->model != SMCDET_MODEL_M71)
    return set_error(SMCDET_EUNSUPPORTED, "joint tile %dx%d with S=%d exceeds LDS (M71 only "
                     "beyond)", model->H, model->W, S);
  return (int64_t)T * N * (2 * (int64_t)model->H * model->W + 3 * (int64_t)S);
}

extern "C" int smcdet_aggregate_sweep(
    const smcdet_image_model_t* model, const smcdet_prior_t* prior, const smcdet_mh_t* mh,
    int32_t axis, const float* tiled_image, const float* temperature, int32_t T, int32_t N,
    int32_t S, const int64_t* ancestors, const float* counts_in, const float* locs_in,
    const float* fluxes_in, float* counts_out, float* locs_out, float* fluxes_out, uint64_t seed,
    uint64_t offset, const smcdet_mh_replay_t* replay, float* loglik_parent,
    float* loglik_children, float* acc_rate, int32_t* acc_count, const float* tile_boxes,
    float* workspace, void* stream) {
  const int64_t need = smcdet_aggregate_workspace(model, T, N, S);
  if (need < 0) return (int)need;
  int rc = validate_prior(prior);
  if (rc) return rc;
  if (!mh) return set_error(SMCDET_EINVAL, "mh params are null");
  if (!tiled_image || !temperature || !counts_in || !locs_in || !fluxes_in || !locs_out ||
      !fluxes_out)
    return set_error(SMCDET_EINVAL, "null buffer");
  const bool gl = need > 0;
  if (gl && !workspace)
    return set_error(SMCDET_EINVAL, "joint tile %dx%d with S=%d needs a workspace of %lld floats",
                     model->H, model->W, S, (long long)need);
  if (acc_rate && !acc_count) return set_error(SMCDET_EINVAL, "acc_rate needs acc_count");
  if (axis != 0 && axis != 1) return set_error(SMCDET_EINVAL, "axis %d not 0 or 1", axis);
  const int dim = axis == 0 ? model->H : model->W;
  if (dim % 2) return set_error(SMCDET_EUNSUPPORTED, "joint tile side %d is odd", dim);
  if (mh->num_iters < 0) return set_error(SMCDET_EINVAL, "num_iters < 0");
  if (!(mh->locs_stdev > 0.f) || !(mh->fluxes_stdev > 0.f))
    return set_error(SMCDET_EINVAL, "proposal standard deviations must be > 0");
  if (ancestors && (locs_in == locs_out || fluxes_in == fluxes_out ||
                    (counts_out && counts_in == counts_out)))
    return set_error(SMCDET_EINVAL, "ancestor gather needs distinct in/out buffers");
  if (replay && (!replay->comp || !replay->uloc || !replay->uflux || !replay->uacc))
    return set_error(SMCDET_EINVAL, "incomplete replay buffers");

  AggArgs a{};
  a.m = make_dev_model(*model);
  a.pr = make_dev_prior(*prior);
  a.K = mh->num_iters;
  a.T = T;
  a.N = N;
  a.S = S;
  a.axis = axis;
  a.halfpix = dim / 2;
  a.half = (float)dim / 2.0f;
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
  a.ll_parent = loglik_parent;
  a.ll_child = loglik_children;
  a.acc_count = acc_count;
  a.acc_rate = acc_rate;
  a.boxes = tile_boxes;
  if (replay) {
    a.r_comp = replay->comp;
    a.r_uloc = replay->uloc;
    a.r_uflux = replay->uflux;
    a.r_uacc = replay->uacc;
  }
  a.work = workspace;
  hipStream_t st = (hipStream_t)stream;
  if (gl) {  // M71 (smcdet_aggregate_workspace), 4 waves, no dynamic LDS
    a.nw = kAggMaxWaves;
    const dim3 grid((N + a.nw - 1) / a.nw, T), block(a.nw * kWave);
    if (replay)
      hipLaunchKernelGGL((agg_sweep_kernel<SMCDET_MODEL_M71, true, true>), grid, block, 0, st, a);
    else
      hipLaunchKernelGGL((agg_sweep_kernel<SMCDET_MODEL_M71, false, true>), grid, block, 0, st, a);
    return check_launch("smcdet_aggregate_sweep");
  }
  // the largest wave count per workgroup (4..1) whose LDS fits
  // (smcdet_aggregate_workspace sends joint tiles where not even one wave fits
  // to the global-memory path, M71 only)
  const size_t HWp = (size_t)model->H * model->W + kWave;
  const size_t img_b = (model->model == SMCDET_MODEL_POISSON ? 2 : 1) * HWp * sizeof(float);
  const size_t wave_b = (2 * HWp + 3 * (size_t)S) * sizeof(float);
  int nw = kAggMaxWaves;
  while (nw > agg_min_lds_waves(model->model) && img_b + nw * wave_b > 160 * 1024) --nw;
  const size_t lds = img_b + nw * wave_b;
  a.nw = nw;
  const dim3 grid((N + nw - 1) / nw, T), block(nw * kWave);
  const bool m71 = a.m.model == SMCDET_MODEL_M71;
  const void* fn =
      replay ? (m71 ? (const void*)agg_sweep_kernel<SMCDET_MODEL_M71, true>
                    : (const void*)agg_sweep_kernel<SMCDET_MODEL_POISSON, true>)
             : (m71 ? (const void*)agg_sweep_kernel<SMCDET_MODEL_M71, false>
                    : (const void*)agg_sweep_kernel<SMCDET_MODEL_POISSON, false>);
  rc = ensure_lds(fn, lds);
  if (rc) return rc;
  if (replay) {
    if (m71) hipLaunchKernelGGL((agg_sweep_kernel<SMCDET_MODEL_M71, true>), grid, block, lds, st, a);
    else hipLaunchKernelGGL((agg_sweep_kernel<SMCDET_MODEL_POISSON, true>), grid, block, lds, st, a);
  } else {
    if (m71) hipLaunchKernelGGL((agg_sweep_kernel<SMCDET_MODEL_M71, false>), grid, block, lds, st, a);
    else hipLaunchKernelGGL((agg_sweep_kernel<SMCDET_MODEL_POISSON, false>), grid, block, lds, st, a);
  }
  return check_launch("smcdet_aggregate_sweep");
}
