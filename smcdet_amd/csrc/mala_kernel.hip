// mala_kernel.hip — the fused single-component MALA sweep (restates
// smcdet/kernel.py:133-275, SingleComponentMALA.run, with the log_target of
// smcdet/sampler.py:87-91 and its torch.autograd.grad gradient evaluated
// in-kernel).
//
// Same execution model as the MH sweep (mh_kernel.hip): one particle per
// 64-lane wavefront, 4 particles of one tile per workgroup sharing the tile
// image in LDS, all K iterations in one launch, the particle's state in
// registers (lane s holds source s) and its rate image in the wave's LDS
// slice.  Per iteration:
//   * gradient at the current state w.r.t. the chosen source's (h, w, f):
//     d log_target / d rate per pixel (M71: (x-l)/v + eta (x-l)^2/(2v^2) -
//     eta/(2v); Poisson: x/l - 1) times d rate / d(h, w, f) = g psf, g f
//     dpsf/dh, g f dpsf/dw, summed over the source's clipped PSF window (one
//     pass, <= (2R+1)^2 positions), plus the flux prior's -(alpha+1)/f;
//   * proposal (kernel.py:168-190): truncated normals around x + step^2/2 *
//     grad, lanes 0/1/2 one dimension each, in the reference's float32
//     operation order (distributions.py:22-52): Normal.cdf saturates to 0/1
//     a few sigma outside the box, log(mass in box) then becomes -FLT_MAX
//     (nan_to_num) and the reference's float32 sums (kernel.py:220-251)
//     absorb the log target; these regimes are reproduced exactly;
//   * one pass over the new window (delta log-likelihood, the rate after the
//     move, the gradient at the proposal) and one over the old window's
//     remaining positions (delta log-likelihood); the moved rates go to an
//     LDS scratch and are written back on accept; the source's PSF at its
//     current place comes from an LDS cache filled by the gradient pass;
//   * accept iff U <= min(1, exp(log alpha)); log alpha in the finite regime
//     is the exact difference (delta log target + Hastings terms, no float32
//     absorption of a ~1e3-1e4 log target), proposals on the location box's
//     upper edge have log prior -inf (torch Uniform.log_prob at `high`) and
//     are rejected.
#include <math.h>

#include "mcmc.h"

namespace smcdet {

constexpr int kMalaWaves = 4;
constexpr int kMalaBlock = kMalaWaves * kWave;

struct MalaArgs {
  DevModel m;
  DevPrior pr;
  int K, T, N, S;
  float sl, rsl, sf, rsf;            // step sizes and float32 reciprocals
  float cl, cf;                      // 0.5 * step^2 (float32, as the reference)
  float lb_h, lb_w, ub_h, ub_w;      // proposal box (locs)
  float lb_f, ub_f;                  // proposal box (fluxes)
  uint32_t k0, k1;                   // Philox key
  uint64_t offset;                   // Philox counter base (iterations)
  int by_count, skip_done;
  int W2;                            // (2R+1)^2: scratch positions per window
  const float* img;
  const float* temperature;
  const int64_t* ancestors;
  const float* counts_in;
  const float* locs_in;
  const float* fluxes_in;
  float* counts_out;
  float* locs_out;
  float* fluxes_out;
  float* loglik_out;
  const float* rate_in;
  float* rate_out;
  const int32_t* go;                 // predicate: skip the launch when *go == 0 (or null)
  int32_t* acc_count;
  float* acc_rate;
  const int32_t* r_comp;
  const float* r_uloc;
  const float* r_uflux;
  const float* r_uacc;
};

constexpr int kKeep = 5;  // register-resident new-window slots (5*64 >= 17*17)

template <int MODEL, bool REPLAY>
__global__ __launch_bounds__(kMalaBlock, 4) void mala_sweep_kernel(MalaArgs a) {
  extern __shared__ float smem[];
  __shared__ int wg_acc, wg_done;
  if (a.go && *a.go == 0) return;
  const DevModel& m = a.m;
  const int HW = m.H * m.W;
  const int HWp = HW + kWave;
  const int t = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int kImg = (MODEL == SMCDET_MODEL_POISSON) ? 2 : 1;
  float* xs = smem;
  float* lg = smem + HWp;
  float* lam = smem + kImg * HWp + wave * (HWp + 3 * a.W2);
  float* scr = lam + HWp;  // moved rates: new window [0, W2), old-only [W2, 2 W2)
  float* psc = scr + 2 * a.W2;  // raw psf of the moved source at its current place, per old-window position

  stage_image<MODEL>(a.img + (size_t)t * HW, xs, lg, HW, threadIdx.x, kMalaBlock);
  if (threadIdx.x == 0) {
    wg_acc = 0;
    wg_done = 0;
  }
  __syncthreads();
  const int n = blockIdx.x * kMalaWaves + wave;
  if (n >= a.N) return;

  const int N = a.N, S = a.S;
  const size_t pid = (size_t)t * N + n;
  const size_t src = a.ancestors ? (size_t)t * N + (size_t)a.ancestors[pid] : pid;
  const float count = a.counts_in[src];
  if (a.counts_out && lane == 0) a.counts_out[pid] = count;
  const int Sj = a.by_count ? min(max((int)count, 0), S) : S;
  const float tau = a.temperature[t];
  const int K = (Sj > 0 && !(a.skip_done && tau >= 1.0f)) ? a.K : 0;

  float sh = 0.f, sw = 0.f, sfx = 0.f;
  if (lane < S) {
    sh = a.locs_in[(src * S + lane) * 2 + 0];
    sw = a.locs_in[(src * S + lane) * 2 + 1];
    sfx = a.fluxes_in[src * S + lane];
  }
  if (a.rate_in) {
    const float* rin = a.rate_in + src * (size_t)HW;
    for (int p = lane; p < HW; p += kWave) lam[p] = rin[p];
    wave_sync();
  } else {
    render_sources<MODEL>(m, lam, sh, sw, sfx, S, lane);
  }

  // lane d < 3 owns proposal dimension d (h, w, flux)
  const int d = lane % 3;  // proposal dimension of this lane (lanes 3.. replicate 0..2)
  const float dsig = d < 2 ? a.sl : a.sf, drs = d < 2 ? a.rsl : a.rsf;
  const float dc = d < 2 ? a.cl : a.cf;
  const float dlb = d == 0 ? a.lb_h : (d == 1 ? a.lb_w : a.lb_f);
  const float dub = d == 0 ? a.ub_h : (d == 1 ? a.ub_w : a.ub_f);
  const float gs = m.g * psf_scale<MODEL>(m);  // rate per unit flux per raw psf

  // draws: lane i holds iteration (block*64 + i)
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
      const U4 r0 = philox4x32(c0, c1, (uint32_t)pid, kTagMALA0, a.k0, a.k1);
      const U4 r1 = philox4x32(c0, c1, (uint32_t)pid, kTagMALA1, a.k0, a.k1);
      ru0 = u01(r0.x);
      ru1 = u01(r0.y);
      ru2 = u01(r0.z);
      ru3 = u01(r0.w);
      ru4 = u01(r1.x);
    }
  };

  // raw gradient sums of the image log-likelihood for a source at (h, w):
  // sum e dpsi dh, sum e dpsi dw, sum e psi with e = d loglik / d rate over
  // the rates in `lam` (wave-uniform results in gr[3])
  auto grad_at = [&](float h, float w, const Window& q, float (&gr)[3]) {
    float gh = 0.f, gw = 0.f, gf = 0.f;
    for (int i = lane; i < q.npos; i += kWave) {
      int ph, pw;
      window_pos(q, i, ph, pw);
      const float dh = ((float)ph + 0.5f) - h, dw = ((float)pw + 0.5f) - w;
      float dpsi;
      const float psi = psf_raw_d<MODEL>(m, fmaf(dh, dh, dw * dw), dpsi);
      psc[i] = psi;  // reused by the delta passes (the same value bit for bit)
      const int p = ph * m.W + pw;
      const float e = dll_drate<MODEL>(m, xs[p], lam[p]);
      gf = fmaf(e, psi, gf);
      const float ed = e * dpsi;
      gh = fmaf(ed, dh, gh);
      gw = fmaf(ed, dw, gw);
    }
    gr[0] = wave_sum(gh);
    gr[1] = wave_sum(gw);
    gr[2] = wave_sum(gf);
    wave_sync();  // psc[] written by all lanes before the delta passes read it
  };

  int accept = 0;
  for (int k = 0; k < K; ++k) {
    const int kl = k & 63;
    if (kl == 0) refill(k);
    int j;
    if constexpr (REPLAY) j = readlane(rcomp, kl);
    else j = min((int)(readlane(ru0, kl) * (float)Sj), Sj - 1);
    const float uacc = readlane(ru4, kl);
    const float ud = d == 0 ? readlane(ru1, kl) : (d == 1 ? readlane(ru2, kl) : readlane(ru3, kl));
    const float h = readlane(sh, j), w = readlane(sw, j), f = readlane(sfx, j);
    const bool active = (float)j < count;
    const float ft = f == 0.f ? a.pr.lower : f;  // prior.py:189, :226

    // ---- gradient at the current state (kernel.py:157-166) ------------------
    const Window qo = window_of(m, h, w);
    float g0[3];
    grad_at(h, w, qo, g0);
    const float gh = tau * ((gs * f) * (-2.0f * g0[0]));
    const float gw = tau * ((gs * f) * (-2.0f * g0[1]));
    const float gf = tau * (gs * g0[2]) - (active ? a.pr.ap1 / ft : 0.f);

    // ---- proposal (kernel.py:168-190), lane d: dimension d -------------------
    const float cur = d == 0 ? h : (d == 1 ? w : f);
    const float gd = d == 0 ? gh : (d == 1 ? gw : gf);
    float mu;
    {
#pragma clang fp contract(off)
      mu = cur + dc * gd;
    }
    const TnBox bf = t_box_lanes(mu, drs, dlb, dub, lane);
    const float xn = t_sample_box(mu, dsig, dlb, dub, ud, bf);
    const float q_fwd = t_logprob_box(xn, mu, dsig, bf);
    const float hn = readlane(xn, 0), wn = readlane(xn, 1), fn = readlane(xn, 2);

    // ---- new window: delta log-likelihood, moved rates, gradient at the proposal
    const Window qn = window_of(m, hn, wn);
    const float amp_o = gs * f, amp_n = gs * fn;
    float dsum = 0.f, pgh = 0.f, pgw = 0.f, pgf = 0.f;
    // one new-window position: accumulates the delta and the gradient, returns
    // the moved rate (same per-lane order over i as a plain strided loop)
    auto new_pos = [&](int i, int& p) -> float {
      int ph, pw;
      window_pos(qn, i, ph, pw);
      const float fph = (float)ph + 0.5f, fpw = (float)pw + 0.5f;
      const float dhn = fph - hn, dwn = fpw - wn;
      float dpsi;
      const float psi_n = psf_raw_d<MODEL>(m, fmaf(dhn, dhn, dwn * dwn), dpsi);
      float psi_o = 0.f;
      if (in_window(m, qo.fh, qo.fw, ph, pw)) psi_o = psc[(ph - qo.r0) * qo.bw + (pw - qo.c0)];
      const float dl = fmaf(amp_n, psi_n, -amp_o * psi_o);
      p = ph * m.W + pw;
      const float lo = lam[p], x = xs[p];
      const float lgx = (MODEL == SMCDET_MODEL_POISSON) ? lg[p] : 0.0f;
      dsum += pix_delta<MODEL>(m, x, lgx, lo, dl);
      const float l1 = lo + dl;
      const float e = dll_drate<MODEL>(m, x, l1);
      pgf = fmaf(e, psi_n, pgf);
      const float ed = e * dpsi;
      pgh = fmaf(ed, dhn, pgh);
      pgw = fmaf(ed, dwn, pgw);
      return l1;
    };
    // the first kKeep positions per lane keep their moved rates in registers
    // (a whole 17x17 window), further ones go to the LDS scratch
    float kv[kKeep];
    int kp[kKeep];
#pragma unroll
    for (int s_ = 0; s_ < kKeep; ++s_) {
      const int i = lane + s_ * kWave;
      kp[s_] = 0;
      kv[s_] = 0.f;
      if (i < qn.npos) kv[s_] = new_pos(i, kp[s_]);
    }
    for (int i = lane + kKeep * kWave; i < qn.npos; i += kWave) {
      int p;
      scr[i] = new_pos(i, p);
    }
    // old window positions outside the new window: the source's rate leaves
    // (no walk when the old window's clipped box lies inside the new window)
    const bool old_only = has_old_only(m, qo, qn);
    for (int i = lane; old_only && i < qo.npos; i += kWave) {
      int ph, pw;
      window_pos(qo, i, ph, pw);
      if (in_window(m, qn.fh, qn.fw, ph, pw)) continue;
      const float dl = -amp_o * psc[i];
      const int p = ph * m.W + pw;
      const float lo = lam[p];
      const float lgx = (MODEL == SMCDET_MODEL_POISSON) ? lg[p] : 0.0f;
      dsum += pix_delta<MODEL>(m, xs[p], lgx, lo, dl);
      scr[a.W2 + i] = lo + dl;
    }
    const float dll = wave_sum(dsum);
    const float fnt = fn == 0.f ? a.pr.lower : fn;
    const float pgh_ = tau * ((gs * fn) * (-2.0f * wave_sum(pgh)));
    const float pgw_ = tau * ((gs * fn) * (-2.0f * wave_sum(pgw)));
    const float pgf_ = tau * (gs * wave_sum(pgf)) - (active ? a.pr.ap1 / fnt : 0.f);

    // ---- reverse proposal density q(z | z') (kernel.py:199-224) -------------
    const float pgd = d == 0 ? pgh_ : (d == 1 ? pgw_ : pgf_);
    float mur;
    {
#pragma clang fp contract(off)
      mur = xn + dc * pgd;
    }
    const float q_rev = t_logprob_box(cur, mur, dsig, t_box_lanes(mur, drs, dlb, dub, lane));
    const float f0 = readlane(q_fwd, 0), f1 = readlane(q_fwd, 1), f2 = readlane(q_fwd, 2);
    const float b0 = readlane(q_rev, 0), b1 = readlane(q_rev, 1), b2 = readlane(q_rev, 2);

    // ---- accept / reject (kernel.py:226-266) ---------------------------------
    // log prior change: -(alpha+1) log(f'/f) for an active source; a location
    // at or beyond the uniform prior's `high` has log prior -inf (nan for a
    // masked source): both reject
    const bool outside = hn >= a.pr.hi_h || wn >= a.pr.hi_w || hn < a.pr.lo || wn < a.pr.lo;
    const float dprior = active ? -a.pr.ap1 * (fast_log(fnt) - fast_log(ft)) : 0.f;
    const float dlt = dprior + tau * dll;
    const float big = 1e30f;
    float la;
    if (fabsf(f0) < big && fabsf(f1) < big && fabsf(f2) < big && fabsf(b0) < big &&
        fabsf(b1) < big && fabsf(b2) < big) {
      la = dlt + ((b0 - f0) + (b1 - f1)) + (b2 - f2);
    } else {
      // saturated mass-in-box terms: the reference's float32 sums, in its
      // order; the (finite) log target itself is absorbed
#pragma clang fp contract(off)
      const float num = (dlt + (b0 + b1)) + b2;
      const float den = (f0 + f1) + f2;
      la = num - den;
    }
    const float e = expf(la);
    const float alpha = e > 1.0f ? 1.0f : e;  // clamp(max=1) keeps nan
    accept = __builtin_amdgcn_readfirstlane((!outside && uacc <= alpha) ? 1 : 0);
    if (accept) {
#pragma unroll
      for (int s_ = 0; s_ < kKeep; ++s_)
        if (lane + s_ * kWave < qn.npos) lam[kp[s_]] = kv[s_];
      for (int i = lane + kKeep * kWave; i < qn.npos; i += kWave) {
        int ph, pw;
        window_pos(qn, i, ph, pw);
        lam[ph * m.W + pw] = scr[i];
      }
      for (int i = lane; old_only && i < qo.npos; i += kWave) {
        int ph, pw;
        window_pos(qo, i, ph, pw);
        if (!in_window(m, qn.fh, qn.fw, ph, pw)) lam[ph * m.W + pw] = scr[a.W2 + i];
      }
      sh = writelane(hn, j, sh);
      sw = writelane(wn, j, sw);
      sfx = writelane(fn, j, sfx);
    }
    wave_sync();
  }

  // ---- write back ---------------------------------------------------------------
  if (lane < S) {
    a.locs_out[(pid * S + lane) * 2 + 0] = sh;
    a.locs_out[(pid * S + lane) * 2 + 1] = sw;
    a.fluxes_out[pid * S + lane] = sfx;
  }
  if (a.loglik_out) {
    const double ll = pixel_sum<MODEL>(m, xs, lg, lam, nullptr, lane);
    if (lane == 0) a.loglik_out[pid] = (float)ll;
  }
  if (a.rate_out) {
    float* rout = a.rate_out + pid * (size_t)HW;
    for (int p = lane; p < HW; p += kWave) rout[p] = lam[p];
  }
  // acceptance rate of the last iteration (kernel.py:275), as mh_kernel.hip
  if (lane == 0) {
    const int nw = min(kMalaWaves, N - (int)blockIdx.x * kMalaWaves);
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

template <int MODEL>
static int launch_mala(const MalaArgs& a, bool replay, dim3 grid, size_t lds, hipStream_t st) {
  const void* fn = replay ? (const void*)mala_sweep_kernel<MODEL, true>
                          : (const void*)mala_sweep_kernel<MODEL, false>;
  int rc = ensure_lds(fn, lds);
  if (rc) return rc;
  if (replay)
    launch_sweep(mala_sweep_kernel<MODEL, true>, grid, dim3(kMalaBlock), lds, st, a);
  else
    launch_sweep(mala_sweep_kernel<MODEL, false>, grid, dim3(kMalaBlock), lds, st, a);
  return SMCDET_OK;
}

}  // namespace smcdet

using namespace smcdet;

extern "C" int smcdet_mala_sweep(const smcdet_image_model_t* model, const smcdet_prior_t* prior,
                                 const smcdet_mh_t* mala, const float* tiled_image,
                                 const float* temperature, int32_t T, int32_t N, int32_t S,
                                 const int64_t* ancestors, const float* counts_in,
                                 const float* locs_in, const float* fluxes_in, float* counts_out,
                                 float* locs_out, float* fluxes_out, const float* rate_in,
                                 float* rate_out, uint64_t seed, uint64_t offset,
                                 const smcdet_mh_replay_t* replay, uint32_t flags,
                                 float* loglik_out, float* acc_rate, int32_t* acc_count,
                                 const int32_t* go, void* stream) {
  int rc = validate_model(model);
  if (rc) return rc;
  rc = validate_prior(prior);
  if (rc) return rc;
  if (!mala) return set_error(SMCDET_EINVAL, "mala params are null");
  if (!tiled_image || !temperature || !counts_in || !locs_in || !fluxes_in || !locs_out ||
      !fluxes_out || !acc_rate || !acc_count)
    return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || N <= 0 || T > 65535) return set_error(SMCDET_EUNSUPPORTED, "T=%d N=%d", T, N);
  if (S < 1 || S > 64) return set_error(SMCDET_EUNSUPPORTED, "S=%d outside 1..64", S);
  if (mala->num_iters < 0) return set_error(SMCDET_EINVAL, "num_iters < 0");
  if (ancestors && (locs_in == locs_out || fluxes_in == fluxes_out ||
                    (counts_out && counts_in == counts_out)))
    return set_error(SMCDET_EINVAL, "ancestor gather needs distinct in/out buffers");
  if (ancestors && rate_in && rate_in == rate_out)
    return set_error(SMCDET_EINVAL, "ancestor gather needs distinct rate_in/rate_out buffers");
  if (replay && (!replay->comp || !replay->uloc || !replay->uflux || !replay->uacc))
    return set_error(SMCDET_EINVAL, "incomplete replay buffers");
  if (!(mala->locs_stdev > 0.f) || !(mala->fluxes_stdev > 0.f))
    return set_error(SMCDET_EINVAL, "step sizes must be > 0");
  if (flags & ~(SMCDET_MH_COMPONENT_BY_COUNT | SMCDET_MH_SKIP_DONE))
    return set_error(SMCDET_EUNSUPPORTED, "unsupported MALA flags 0x%x", flags);

  MalaArgs a{};
  a.m = make_dev_model(*model);
  a.pr = make_dev_prior(*prior);
  a.K = mala->num_iters;
  a.T = T;
  a.N = N;
  a.S = S;
  a.sl = mala->locs_stdev;
  a.sf = mala->fluxes_stdev;
  a.rsl = 1.0f / a.sl;
  a.rsf = 1.0f / a.sf;
  a.cl = 0.5f * (a.sl * a.sl);
  a.cf = 0.5f * (a.sf * a.sf);
  a.lb_h = mala->locs_min_h;
  a.lb_w = mala->locs_min_w;
  a.ub_h = mala->locs_max_h;
  a.ub_w = mala->locs_max_w;
  a.lb_f = mala->fluxes_min;
  a.ub_f = mala->fluxes_max;
  a.k0 = (uint32_t)seed;
  a.k1 = (uint32_t)(seed >> 32);
  a.offset = offset;
  a.by_count = (flags & SMCDET_MH_COMPONENT_BY_COUNT) != 0;
  a.skip_done = (flags & SMCDET_MH_SKIP_DONE) != 0;
  a.W2 = (2 * model->psf_radius + 1) * (2 * model->psf_radius + 1);
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
  if (replay) {
    a.r_comp = replay->comp;
    a.r_uloc = replay->uloc;
    a.r_uflux = replay->uflux;
    a.r_uacc = replay->uacc;
  }
  const size_t HWp = (size_t)model->H * model->W + kWave;
  const size_t lds = ((model->model == SMCDET_MODEL_POISSON ? 2 : 1) * HWp +
                      (size_t)kMalaWaves * (HWp + 3 * (size_t)a.W2)) *
                     sizeof(float);
  const dim3 grid((N + kMalaWaves - 1) / kMalaWaves, T);
  hipStream_t st = (hipStream_t)stream;
  rc = a.m.model == SMCDET_MODEL_M71 ? launch_mala<SMCDET_MODEL_M71>(a, replay != nullptr, grid, lds, st)
                                     : launch_mala<SMCDET_MODEL_POISSON>(a, replay != nullptr, grid, lds, st);
  if (rc) return rc;
  return check_launch("smcdet_mala_sweep");
}
