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
//   * accept iff U <= min(1, exp(log alpha)) (kernel.py:114-116).
// The rate image is rebuilt from scratch at the start of each sweep and the
// returned loglik_out comes from a fresh full render of the final state.
#include <math.h>

#include "render.h"

namespace smcdet {

constexpr int kMhWaves = 4;
constexpr int kMhBlock = kMhWaves * kWave;
constexpr int kSlots = 8;  // register-resident window passes (8*64 = 512 positions)

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
  const float* img;                  // [T,H,W]
  const float* temperature;          // [T]
  const int64_t* ancestors;          // [T,N] or null
  const float* counts_in;
  const float* locs_in;
  const float* fluxes_in;
  float* counts_out;
  float* locs_out;
  float* fluxes_out;
  float* loglik_out;                 // [T,N] or null
  int32_t* acc_count;                // [T]
  const int32_t* r_comp;             // replay (or null)
  const float* r_uloc;
  const float* r_uflux;
  const float* r_uacc;
};

// truncated-normal cache at mean mu: Phi(lb), Z = Phi(ub) - Phi(lb), log Z
// (distributions.py:33-35)
__device__ __forceinline__ void tn_cache(float mu, float isig, float lb, float ub, float& phl,
                                         float& Z, float& lZ) {
  phl = normal_cdf(lb, mu, isig);
  Z = normal_cdf(ub, mu, isig) - phl;
  lZ = nan_to_num(fast_log(Z), 0.0f);
}

template <int MODEL, bool REPLAY, bool FULL>
__global__ __launch_bounds__(kMhBlock) void mh_sweep_kernel(MhArgs a) {
  extern __shared__ float smem[];
  const DevModel& m = a.m;
  const int HW = m.H * m.W;
  const int t = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int kImg = (MODEL == SMCDET_MODEL_POISSON) ? 2 : 1;
  float* xs = smem;
  float* lg = smem + HW;
  float* lam = smem + kImg * HW + wave * HW;

  stage_image<MODEL>(a.img + (size_t)t * HW, xs, lg, HW, threadIdx.x, kMhBlock);
  __syncthreads();
  const int n = blockIdx.x * kMhWaves + wave;
  if (n >= a.N) return;

  const int N = a.N, S = a.S;
  const size_t pid = (size_t)t * N + n;
  const size_t src = a.ancestors ? (size_t)t * N + (size_t)a.ancestors[pid] : pid;
  const float count = a.counts_in[src];
  if (a.counts_out && lane == 0) a.counts_out[pid] = count;

  // ---- particle state: lane s holds source s --------------------------------
  float sh = 0.f, sw = 0.f, sfx = 0.f;
  if (lane < S) {
    sh = a.locs_in[(src * S + lane) * 2 + 0];
    sw = a.locs_in[(src * S + lane) * 2 + 1];
    sfx = a.fluxes_in[src * S + lane];
  }
  // per-source proposal caches at the current values
  float ph_h, Z_h, lZ_h, ph_w, Z_w, lZ_w, ph_f, Z_f, lZ_f;
  tn_cache(sh, a.isl, a.lb_h, a.ub_h, ph_h, Z_h, lZ_h);
  tn_cache(sw, a.isl, a.lb_w, a.ub_w, ph_w, Z_w, lZ_w);
  tn_cache(sfx, a.isf, a.lb_f, a.ub_f, ph_f, Z_f, lZ_f);
  float lfx = fast_log(sfx);

  const float tau = a.temperature[t];
  render_sources<MODEL>(m, lam, sh, sw, sfx, S, lane);
  double cur_ll = pixel_sum<MODEL>(m, xs, lg, lam, nullptr, lane);

  // lanes 0,1,2 handle proposal dimension d = h, w, flux
  const int d = lane < 3 ? lane : 2;
  const float p_isig = d < 2 ? a.isl : a.isf;
  const float p_sig = d < 2 ? a.sl : a.sf;
  const float p_lb = d == 0 ? a.lb_h : (d == 1 ? a.lb_w : a.lb_f);
  const float p_ub = d == 0 ? a.ub_h : (d == 1 ? a.ub_w : a.ub_f);

  float ru0 = 0.f, ru1 = 0.f, ru2 = 0.f, ru3 = 0.f, ru4 = 0.f;
  int rcomp = 0;
  bool accept = false;

  for (int k = 0; k < a.K; ++k) {
    const int kl = k & 63;
    if (kl == 0) {
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
        const U4 r0 = philox4x32(c0, c1, (uint32_t)pid, kTagMH0, a.k0, a.k1);
        const U4 r1 = philox4x32(c0, c1, (uint32_t)pid, kTagMH1, a.k0, a.k1);
        ru0 = u01(r0.x);
        ru1 = u01(r0.y);
        ru2 = u01(r0.z);
        ru3 = u01(r0.w);
        ru4 = u01(r1.x);
      }
    }
    int j;
    if constexpr (REPLAY) {
      j = readlane(rcomp, kl);
    } else {
      j = min((int)(readlane(ru0, kl) * (float)S), S - 1);
    }
    const float uacc = readlane(ru4, kl);

    // ---- current values and caches of source j -------------------------------
    const float h = readlane(sh, j), w = readlane(sw, j), f = readlane(sfx, j);
    const float lf = readlane(lfx, j);
    const float c_ph = d == 0 ? readlane(ph_h, j) : (d == 1 ? readlane(ph_w, j) : readlane(ph_f, j));
    const float c_lZ = d == 0 ? readlane(lZ_h, j) : (d == 1 ? readlane(lZ_w, j) : readlane(lZ_f, j));
    const float mu = d == 0 ? h : (d == 1 ? w : f);
    const float u = d == 0 ? readlane(ru1, kl) : (d == 1 ? readlane(ru2, kl) : readlane(ru3, kl));

    // ---- truncated-normal proposal, lanes 0..2 (distributions.py:40-48) ------
    float xn, n_ph, n_Z, n_lZ, hast_d, n_lf;
    if (a.ablate & SMCDET_MH_ABLATE_PROPOSAL) {
      // timing-only stand-in: a small deterministic move, no special functions
      xn = fminf(fmaxf(mu + (u - 0.5f) * p_sig, p_lb), p_ub);
      n_ph = c_ph;
      n_Z = 1.f;
      n_lZ = c_lZ;
      hast_d = 0.f;
      n_lf = xn;
    } else {
      const float pc = fminf(fmaxf(u, 1e-6f), 0.999999f);
      float pt = c_ph + pc * fast_exp(c_lZ);
      pt = fminf(fmaxf(pt, 1e-6f), 0.999999f);
      xn = mu + p_sig * erfinv_fast(2.0f * pt - 1.0f) * kSqrt2;
      xn = fminf(fmaxf(xn, p_lb), p_ub);
      tn_cache(xn, p_isig, p_lb, p_ub, n_ph, n_Z, n_lZ);
      hast_d = c_lZ - n_lZ;  // log q(z|z') - log q(z'|z), this dimension
      n_lf = fast_log(xn);
    }

    const float hn = readlane(xn, 0), wn = readlane(xn, 1), fn = readlane(xn, 2);
    const float hast = readlane(hast_d, 0) + readlane(hast_d, 1) + readlane(hast_d, 2);
    const float lfn = readlane(n_lf, 2);
    // prior: uniform locations are constant in the box; flux density term
    const float dprior = ((float)j < count) ? -a.pr.ap1 * (lfn - lf) : 0.0f;

    // ---- likelihood difference -----------------------------------------------
    float dll;
    double new_ll = 0.0;
    const float amp_o = m.g * f, amp_n = m.g * fn;
    // register slots for the incremental path
    float s_lam[kSlots];
    int s_pix[kSlots];
    int r0 = 0, c0 = 0, bw = 1, npos = 0;
    int fh0 = 0, fw0 = 0, fh1 = 0, fw1 = 0;
    float inv_bw = 1.f;
    if constexpr (FULL) {
      const float ch = lane == j ? hn : sh, cw = lane == j ? wn : sw, cf = lane == j ? fn : sfx;
      render_sources<MODEL>(m, lam, ch, cw, cf, S, lane);
      new_ll = pixel_sum<MODEL>(m, xs, lg, lam, nullptr, lane);
      dll = (float)(new_ll - cur_ll);
    } else {
      fh0 = ifloor_clamped(h);
      fw0 = ifloor_clamped(w);
      fh1 = ifloor_clamped(hn);
      fw1 = ifloor_clamped(wn);
      r0 = max(min(fh0, fh1) - m.R, 0);
      const int r1 = min(max(fh0, fh1) + m.R, m.H - 1);
      c0 = max(min(fw0, fw1) - m.R, 0);
      const int c1 = min(max(fw0, fw1) + m.R, m.W - 1);
      bw = c1 - c0 + 1;
      npos = (r1 >= r0 && c1 >= c0 && !(a.ablate & SMCDET_MH_ABLATE_LIKELIHOOD))
                 ? (r1 - r0 + 1) * bw : 0;
      inv_bw = 1.0f / (float)bw;
      float dsum = 0.f;
#pragma unroll
      for (int i = 0; i < kSlots; ++i) {
        s_pix[i] = -1;
        if (i * kWave < npos) {
          const int q = i * kWave + lane;
          if (q < npos) {
            const int aa = (int)(((float)q + 0.5f) * inv_bw);
            const int bb = q - aa * bw;
            const int ph = r0 + aa, pw = c0 + bb;
            const int p = ph * m.W + pw;
            const float fph = (float)ph + 0.5f, fpw = (float)pw + 0.5f;
            float psi_o = 0.f, psi_n = 0.f;
            if (abs(ph - fh0) <= m.R && abs(pw - fw0) <= m.R) {
              const float dh = fph - h, dw = fpw - w;
              psi_o = psf_eval<MODEL>(m, fmaf(dh, dh, dw * dw));
            }
            if (abs(ph - fh1) <= m.R && abs(pw - fw1) <= m.R) {
              const float dh = fph - hn, dw = fpw - wn;
              psi_n = psf_eval<MODEL>(m, fmaf(dh, dh, dw * dw));
            }
            const float dl = fmaf(amp_n, psi_n, -amp_o * psi_o);
            const float lo = lam[p];
            const float lgx = (MODEL == SMCDET_MODEL_POISSON) ? lg[p] : 0.0f;
            dsum += pix_delta<MODEL>(m, xs[p], lgx, lo, dl);
            s_lam[i] = lo + dl;
            s_pix[i] = p;
          }
        }
      }
      // rare: union window larger than the register slots (a jump of several px)
      for (int q = kSlots * kWave + lane; q < npos; q += kWave) {
        const int aa = (int)(((float)q + 0.5f) * inv_bw);
        const int bb = q - aa * bw;
        const int ph = r0 + aa, pw = c0 + bb;
        const int p = ph * m.W + pw;
        const float fph = (float)ph + 0.5f, fpw = (float)pw + 0.5f;
        float psi_o = 0.f, psi_n = 0.f;
        if (abs(ph - fh0) <= m.R && abs(pw - fw0) <= m.R) {
          const float dh = fph - h, dw = fpw - w;
          psi_o = psf_eval<MODEL>(m, fmaf(dh, dh, dw * dw));
        }
        if (abs(ph - fh1) <= m.R && abs(pw - fw1) <= m.R) {
          const float dh = fph - hn, dw = fpw - wn;
          psi_n = psf_eval<MODEL>(m, fmaf(dh, dh, dw * dw));
        }
        const float dl = fmaf(amp_n, psi_n, -amp_o * psi_o);
        const float lgx = (MODEL == SMCDET_MODEL_POISSON) ? lg[p] : 0.0f;
        dsum += pix_delta<MODEL>(m, xs[p], lgx, lam[p], dl);
      }
      dll = wave_sum(dsum);
    }

    // ---- accept / reject (kernel.py:114-128) ----------------------------------
    const float loga = dprior + tau * dll + hast;
    const float e = fast_exp(loga);
    const float alpha = e > 1.0f ? 1.0f : e;  // clamp(max=1) keeps NaN
    accept = uacc <= alpha;
    if (accept) {
      if constexpr (FULL) {
        cur_ll = new_ll;
      } else {
#pragma unroll
        for (int i = 0; i < kSlots; ++i) {
          if (i * kWave < npos && s_pix[i] >= 0) {
            lam[s_pix[i]] = s_lam[i];
          }
        }
        for (int q = kSlots * kWave + lane; q < npos; q += kWave) {
          const int aa = (int)(((float)q + 0.5f) * inv_bw);
          const int bb = q - aa * bw;
          const int ph = r0 + aa, pw = c0 + bb;
          const int p = ph * m.W + pw;
          const float fph = (float)ph + 0.5f, fpw = (float)pw + 0.5f;
          float psi_o = 0.f, psi_n = 0.f;
          if (abs(ph - fh0) <= m.R && abs(pw - fw0) <= m.R) {
            const float dh = fph - h, dw = fpw - w;
            psi_o = psf_eval<MODEL>(m, fmaf(dh, dh, dw * dw));
          }
          if (abs(ph - fh1) <= m.R && abs(pw - fw1) <= m.R) {
            const float dh = fph - hn, dw = fpw - wn;
            psi_n = psf_eval<MODEL>(m, fmaf(dh, dh, dw * dw));
          }
          lam[p] += fmaf(amp_n, psi_n, -amp_o * psi_o);
        }
        cur_ll += (double)dll;
        wave_sync();
      }
      const float nph_h = readlane(n_ph, 0), nZ_h = readlane(n_Z, 0), nlZ_h = readlane(n_lZ, 0);
      const float nph_w = readlane(n_ph, 1), nZ_w = readlane(n_Z, 1), nlZ_w = readlane(n_lZ, 1);
      const float nph_f = readlane(n_ph, 2), nZ_f = readlane(n_Z, 2), nlZ_f = readlane(n_lZ, 2);
      if (lane == j) {
        sh = hn;
        sw = wn;
        sfx = fn;
        lfx = lfn;
        ph_h = nph_h; Z_h = nZ_h; lZ_h = nlZ_h;
        ph_w = nph_w; Z_w = nZ_w; lZ_w = nlZ_w;
        ph_f = nph_f; Z_f = nZ_f; lZ_f = nlZ_f;
      }
    }
  }
  (void)Z_h; (void)Z_w; (void)Z_f;

  // ---- write back --------------------------------------------------------------
  if (lane < S) {
    a.locs_out[(pid * S + lane) * 2 + 0] = sh;
    a.locs_out[(pid * S + lane) * 2 + 1] = sw;
    a.fluxes_out[pid * S + lane] = sfx;
  }
  if (a.loglik_out) {
    render_sources<MODEL>(m, lam, sh, sw, sfx, S, lane);
    const double ll = pixel_sum<MODEL>(m, xs, lg, lam, nullptr, lane);
    if (lane == 0) a.loglik_out[pid] = (float)ll;
  }
  if (lane == 0 && accept && a.K > 0) atomicAdd(a.acc_count + t, 1);
}

__global__ void acc_finalize_kernel(const int32_t* __restrict__ cnt, int T, int N,
                                    float* __restrict__ rate) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < T) rate[t] = (float)cnt[t] / (float)N;
}

template <int MODEL, bool REPLAY, bool FULL>
static int launch_mh1(const MhArgs& a, dim3 grid, size_t lds, hipStream_t st) {
  const void* fn = (const void*)mh_sweep_kernel<MODEL, REPLAY, FULL>;
  int rc = ensure_lds(fn, lds);
  if (rc) return rc;
  hipLaunchKernelGGL((mh_sweep_kernel<MODEL, REPLAY, FULL>), grid, dim3(kMhBlock), lds, st, a);
  return SMCDET_OK;
}

template <int MODEL>
static int launch_mh(const MhArgs& a, bool replay, bool full, dim3 grid, size_t lds,
                     hipStream_t st) {
  if (replay)
    return full ? launch_mh1<MODEL, true, true>(a, grid, lds, st)
                : launch_mh1<MODEL, true, false>(a, grid, lds, st);
  return full ? launch_mh1<MODEL, false, true>(a, grid, lds, st)
              : launch_mh1<MODEL, false, false>(a, grid, lds, st);
}

}  // namespace smcdet

using namespace smcdet;

extern "C" int smcdet_mh_sweep(const smcdet_image_model_t* model, const smcdet_prior_t* prior,
                               const smcdet_mh_t* mh, const float* tiled_image,
                               const float* temperature, int32_t T, int32_t N, int32_t S,
                               const int64_t* ancestors, const float* counts_in,
                               const float* locs_in, const float* fluxes_in, float* counts_out,
                               float* locs_out, float* fluxes_out, uint64_t seed,
                               uint64_t offset, const smcdet_mh_replay_t* replay, uint32_t flags,
                               float* loglik_out, float* acc_rate, int32_t* acc_count,
                               void* stream) {
  int rc = validate_model(model);
  if (rc) return rc;
  rc = validate_prior(prior);
  if (rc) return rc;
  if (!mh) return set_error(SMCDET_EINVAL, "mh params are null");
  if (!tiled_image || !temperature || !counts_in || !locs_in || !fluxes_in || !locs_out ||
      !fluxes_out || !acc_rate || !acc_count)
    return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || N <= 0 || T > 65535) return set_error(SMCDET_EUNSUPPORTED, "T=%d N=%d", T, N);
  if (S < 1 || S > 64) return set_error(SMCDET_EUNSUPPORTED, "S=%d outside 1..64", S);
  if (mh->num_iters < 0) return set_error(SMCDET_EINVAL, "num_iters < 0");
  if (ancestors && (locs_in == locs_out || fluxes_in == fluxes_out ||
                    (counts_out && counts_in == counts_out)))
    return set_error(SMCDET_EINVAL, "ancestor gather needs distinct in/out buffers");
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
  a.acc_count = acc_count;
  if (replay) {
    a.r_comp = replay->comp;
    a.r_uloc = replay->uloc;
    a.r_uflux = replay->uflux;
    a.r_uacc = replay->uacc;
  }
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(acc_count, 0, (size_t)T * sizeof(int32_t), st) != hipSuccess)
    return set_error(SMCDET_EHIP, "smcdet_mh_sweep: memset failed");
  const size_t HW = (size_t)model->H * model->W;
  const size_t lds =
      ((model->model == SMCDET_MODEL_POISSON ? 2 : 1) * HW + (size_t)kMhWaves * HW) *
      sizeof(float);
  const dim3 grid((N + kMhWaves - 1) / kMhWaves, T);
  const bool full = (flags & SMCDET_MH_FULL_RECOMPUTE) != 0;
  a.ablate = flags & (SMCDET_MH_ABLATE_LIKELIHOOD | SMCDET_MH_ABLATE_PROPOSAL);
  rc = a.m.model == SMCDET_MODEL_M71
           ? launch_mh<SMCDET_MODEL_M71>(a, replay != nullptr, full, grid, lds, st)
           : launch_mh<SMCDET_MODEL_POISSON>(a, replay != nullptr, full, grid, lds, st);
  if (rc) return rc;
  rc = check_launch("smcdet_mh_sweep");
  if (rc) return rc;
  hipLaunchKernelGGL(acc_finalize_kernel, dim3((T + 255) / 256), dim3(256), 0, st, acc_count, T,
                     N, acc_rate);
  return check_launch("smcdet_mh_sweep(finalize)");
}
