// chain_kernel.hip — MHsampler.run (smcdet/sampler.py:420-486): one
// single-component MH chain per tile at temperature 1, recording the kept
// samples (burn-in discarded, every keep-th sample) in-kernel.
//
// The reference runs one chain per tile for 50,000 iterations on the CPU,
// image after image (experiments/m71/run_mcmc.py:95-132).  Here one chain is
// one 64-lane wavefront (lane s holds source s, the chain's rate image in the
// wave's LDS slice) and C chains per tile x T tiles run as one grid, so a
// batch of independent images (tiles) advances together; iterations
// [k_begin, k_end) run in one launch and the state is carried in
// locs_state / fluxes_state between launches.  Per iteration: the truncated
// normal proposals of the chosen source (lanes 0/1/2, torch's float32 order,
// mean = current value so the mass-in-box never saturates), the delta
// log-likelihood over its new window and the old-only positions, the
// Hastings terms as the differences of the two truncated-normal log
// densities (kernel.py's and sampler.py:455-495's log_prob pairs), accept iff
// U <= min(1, exp(log alpha)).
#include "mcmc.h"

namespace smcdet {

constexpr int kChainWaves = 4;
constexpr int kChainBlock = kChainWaves * kWave;
constexpr int kChainBatch = 8;  // proposals computed together (6 lanes each)

struct ChainArgs {
  DevModel m;
  DevPrior pr;
  int T, C, S;
  int k_begin, k_end;                // iterations of this launch
  int total, burnin, keep, M;        // samples, burn-in, thinning, kept samples
  float sl, rsl, sf, rsf;
  float lb_h, lb_w, ub_h, ub_w, lb_f, ub_f;
  uint32_t k0, k1;
  uint64_t offset;
  int W2;
  const float* img;                  // [T,H,W]
  const float* counts;               // [T,C]
  float* locs_state;                 // [T,C,S,2] in/out
  float* fluxes_state;               // [T,C,S]   in/out
  float* locs_out;                   // [T,C,M,S,2] kept samples
  float* fluxes_out;                 // [T,C,M,S]
  int32_t* accept_out;               // [T,C,total-1] or null
  int32_t* frozen;                   // [T,C] chain stopped by an edge hit (in/out) or null
  const int32_t* r_comp;             // replay [total-1,T,C] (or null)
  const float* r_uloc;
  const float* r_uflux;
  const float* r_uacc;
};

__global__ __launch_bounds__(kChainBlock, 4) void mh_chain_kernel(ChainArgs a) {
  extern __shared__ float smem[];
  const DevModel& m = a.m;
  const int HW = m.H * m.W;
  const int HWp = HW + kWave;
  const int t = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool poisson = m.model == SMCDET_MODEL_POISSON;
  float* xs = smem;
  float* lg = smem + HWp;
  float* lam = smem + 2 * HWp + wave * (HWp + 2 * a.W2);
  float* scr = lam + HWp;
  if (poisson)
    stage_image<SMCDET_MODEL_POISSON>(a.img + (size_t)t * HW, xs, lg, HW, threadIdx.x, kChainBlock);
  else
    stage_image<SMCDET_MODEL_M71>(a.img + (size_t)t * HW, xs, lg, HW, threadIdx.x, kChainBlock);
  __syncthreads();
  const int c = blockIdx.x * kChainWaves + wave;
  if (c >= a.C) return;
  const int S = a.S;
  const size_t pid = (size_t)t * a.C + c;
  const float count = a.counts[pid];

  float sh = 0.f, sw = 0.f, sfx = 0.f;
  if (lane < S) {
    sh = a.locs_state[(pid * S + lane) * 2 + 0];
    sw = a.locs_state[(pid * S + lane) * 2 + 1];
    sfx = a.fluxes_state[pid * S + lane];
  }
  if (poisson)
    render_sources<SMCDET_MODEL_POISSON>(m, lam, sh, sw, sfx, S, lane);
  else
    render_sources<SMCDET_MODEL_M71>(m, lam, sh, sw, sfx, S, lane);

  auto record = [&](int mi) {  // sample mi (state after iteration mi - 1)
    if (mi < a.burnin || (mi - a.burnin) % a.keep != 0) return;
    const size_t slot = pid * (size_t)a.M + (size_t)((mi - a.burnin) / a.keep);
    if (lane < S) {
      a.locs_out[(slot * S + lane) * 2 + 0] = sh;
      a.locs_out[(slot * S + lane) * 2 + 1] = sw;
      a.fluxes_out[slot * S + lane] = sfx;
    }
  };
  if (a.k_begin == 0) record(0);

  const float gs = m.g * (poisson ? psf_scale<SMCDET_MODEL_POISSON>(m)
                                  : psf_scale<SMCDET_MODEL_M71>(m));
  const int K = a.total - 1;

  float ru0 = 0.f, ru1 = 0.f, ru2 = 0.f, ru3 = 0.f, ru4 = 0.f;
  int rcomp = 0;
  auto refill = [&](int k0) {
    const int kk = k0 + lane;
    if (a.r_comp) {
      if (kk < K) {
        const size_t r = (size_t)kk * a.T * a.C + pid;
        rcomp = a.r_comp[r];
        ru1 = a.r_uloc[r * 2 + 0];
        ru2 = a.r_uloc[r * 2 + 1];
        ru3 = a.r_uflux[r];
        ru4 = a.r_uacc[r];
      }
    } else {
      const uint64_t ctr = a.offset + (uint64_t)kk;
      const uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32);
      const U4 r0 = philox4x32(c0, c1, (uint32_t)pid, kTagChain0, a.k0, a.k1);
      const U4 r1 = philox4x32(c0, c1, (uint32_t)pid, kTagChain1, a.k0, a.k1);
      ru0 = u01(r0.x);
      ru1 = u01(r0.y);
      ru2 = u01(r0.z);
      ru3 = u01(r0.w);
      ru4 = u01(r1.x);
    }
  };

  // ---- proposals and Hastings terms (sampler.py:435-495), batched off the
  // chain's critical path: lane 6b+r computes dimension r % 3 of iteration
  // batch_k0 + b (r < 3: cdf at the lower bound, r >= 3: at the upper bound,
  // exchanged within the group), from the state at batch time.  An entry goes
  // stale only if an earlier accepted iteration of the batch moved the same
  // source (tracked in `dirty`); the batch is then recomputed from there.
  // Each proposal is the same arithmetic on the same inputs as one computed
  // at its own iteration.
  const int gb = lane / 6, gr = lane - 6 * gb, gd = gr % 3;
  const float gsig = gd < 2 ? a.sl : a.sf, grs = gd < 2 ? a.rsl : a.rsf;
  const float glb = gd == 0 ? a.lb_h : (gd == 1 ? a.lb_w : a.lb_f);
  const float gub = gd == 0 ? a.ub_h : (gd == 1 ? a.ub_w : a.ub_f);
  float bcur = 0.f, bxn = 0.f, bqf = 0.f, bqr = 0.f;
  int bj = 0, batch_k0 = 0, batch_n = 0;
  uint64_t dirty = 0;
  auto compute_batch = [&](int k0) {
    const int off = (k0 - a.k_begin) & 63;
    const int n_ = min(min(kChainBatch, kWave - off), a.k_end - k0);
    const int b = min(gb, n_ - 1);
    const int kl = off + b;
    const int j = a.r_comp ? __shfl(rcomp, kl, kWave)
                           : min((int)(__shfl(ru0, kl, kWave) * (float)S), S - 1);
    const float u1 = __shfl(ru1, kl, kWave), u2 = __shfl(ru2, kl, kWave);
    const float u3 = __shfl(ru3, kl, kWave);
    const float ud = gd == 0 ? u1 : (gd == 1 ? u2 : u3);
    const float h = __shfl(sh, j, kWave), w = __shfl(sw, j, kWave), f = __shfl(sfx, j, kWave);
    const float cur = gd == 0 ? h : (gd == 1 ? w : f);
    const int src = 6 * b + gd;
    const TnBox bc = t_box_group(cur, grs, glb, gub, gr, src);
    const float xn = t_sample_box(cur, gsig, glb, gub, ud, bc);
    bqf = t_logprob_box(xn, cur, gsig, bc);
    bqr = t_logprob_box(cur, xn, gsig, t_box_group(xn, grs, glb, gub, gr, src));
    bxn = xn;
    bcur = cur;
    bj = j;
    batch_k0 = k0;
    batch_n = n_;
    dirty = 0;
  };

  // A chain whose proposal landed on the prior box's upper edge is frozen
  // for the rest of the run (below); a later launch continues it frozen.
  int k_end = (a.frozen && a.frozen[pid]) ? a.k_begin : a.k_end;
  int k = a.k_begin;
  for (; k < k_end; ++k) {
    const int kl = (k - a.k_begin) & 63;
    if (kl == 0) refill(k);
    if (k >= batch_k0 + batch_n) compute_batch(k);
    int b = k - batch_k0;
    int j = readlane(bj, 6 * b);
    if ((dirty >> j) & 1ull) {
      compute_batch(k);
      b = 0;
      j = readlane(bj, 0);
    }
    const float uacc = readlane(ru4, kl);
    const float h = readlane(bcur, 6 * b), w = readlane(bcur, 6 * b + 1);
    const float f = readlane(bcur, 6 * b + 2);
    const float hn = readlane(bxn, 6 * b), wn = readlane(bxn, 6 * b + 1);
    const float fn = readlane(bxn, 6 * b + 2);

    // ---- delta log-likelihood over the new window and the old-only positions
    const Window qo = window_of(m, h, w), qn = window_of(m, hn, wn);
    const float amp_o = gs * f, amp_n = gs * fn;
    float dsum = 0.f;
    // the moved rates of the lane's first new-window position stay in
    // registers (all of them on tiles of <= 64 pixels); further ones go to scr
    float v0 = 0.f;
    int p0 = 0;
    for (int i = lane; i < qn.npos; i += kWave) {
      int ph, pw;
      window_pos(qn, i, ph, pw);
      const float fph = (float)ph + 0.5f, fpw = (float)pw + 0.5f;
      const float dhn = fph - hn, dwn = fpw - wn;
      float psi_n, psi_o = 0.f;
      const bool old = in_window(m, qo.fh, qo.fw, ph, pw);
      const float dho = fph - h, dwo = fpw - w;
      if (poisson) {
        psi_n = psf_raw<SMCDET_MODEL_POISSON>(m, fmaf(dhn, dhn, dwn * dwn));
        if (old) psi_o = psf_raw<SMCDET_MODEL_POISSON>(m, fmaf(dho, dho, dwo * dwo));
      } else {
        psi_n = psf_raw<SMCDET_MODEL_M71>(m, fmaf(dhn, dhn, dwn * dwn));
        if (old) psi_o = psf_raw<SMCDET_MODEL_M71>(m, fmaf(dho, dho, dwo * dwo));
      }
      const float dl = fmaf(amp_n, psi_n, -amp_o * psi_o);
      const int p = ph * m.W + pw;
      const float lo = lam[p];
      dsum += poisson ? pix_delta<SMCDET_MODEL_POISSON>(m, xs[p], lg[p], lo, dl)
                      : pix_delta<SMCDET_MODEL_M71>(m, xs[p], 0.f, lo, dl);
      if (i < kWave) {
        v0 = lo + dl;
        p0 = p;
      } else {
        scr[i] = lo + dl;
      }
    }
    // old-only positions exist unless the old window's clipped box lies inside
    // the new window (same anchors, or both cover a small tile): skip the walk
    const bool old_only = has_old_only(m, qo, qn);
    for (int i = lane; old_only && i < qo.npos; i += kWave) {
      int ph, pw;
      window_pos(qo, i, ph, pw);
      if (in_window(m, qn.fh, qn.fw, ph, pw)) continue;
      const float dho = ((float)ph + 0.5f) - h, dwo = ((float)pw + 0.5f) - w;
      const float r2 = fmaf(dho, dho, dwo * dwo);
      const float dl = -amp_o * (poisson ? psf_raw<SMCDET_MODEL_POISSON>(m, r2)
                                         : psf_raw<SMCDET_MODEL_M71>(m, r2));
      const int p = ph * m.W + pw;
      const float lo = lam[p];
      dsum += poisson ? pix_delta<SMCDET_MODEL_POISSON>(m, xs[p], lg[p], lo, dl)
                      : pix_delta<SMCDET_MODEL_M71>(m, xs[p], 0.f, lo, dl);
      scr[a.W2 + i] = lo + dl;
    }
    const float dll = wave_sum(dsum);

    // ---- accept / reject (sampler.py:481-486) --------------------------------
    const bool active = (float)j < count;
    const float ft = f == 0.f ? a.pr.lower : f, fnt = fn == 0.f ? a.pr.lower : fn;
    const float dprior = active ? -a.pr.ap1 * (fast_log(fnt) - fast_log(ft)) : 0.f;
    const bool outside = hn >= a.pr.hi_h || wn >= a.pr.hi_w || hn < a.pr.lo || wn < a.pr.lo;
    const float la = (dprior + dll) +
                     (((readlane(bqr, 6 * b) - readlane(bqf, 6 * b)) +
                       (readlane(bqr, 6 * b + 1) - readlane(bqf, 6 * b + 1))) +
                      (readlane(bqr, 6 * b + 2) - readlane(bqf, 6 * b + 2)));
    const float e = expf(la);
    const float alpha = e > 1.0f ? 1.0f : e;
    const int accept = __builtin_amdgcn_readfirstlane((!outside && uacc <= alpha) ? 1 : 0);
    if (accept) {
      if (lane < qn.npos) lam[p0] = v0;
      for (int i = lane + kWave; i < qn.npos; i += kWave) {
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
      dirty |= 1ull << j;
    }
    wave_sync();
    if (a.accept_out && lane == 0) a.accept_out[pid * (size_t)K + k] = accept;
    record(k + 1);
    // An edge hit (Uniform.log_prob(high) = -inf, prior.py:73) is rejected,
    // and the reference caches log_num_target * 0 = NaN as the current log
    // target (sampler.py:522-526): every later proposal of the chain is
    // rejected, for the rest of the run.
    if (outside) {
      ++k;
      if (a.frozen && lane == 0) a.frozen[pid] = 1;
      break;
    }
  }
  // the frozen remainder: rejections, the same state recorded as the samples
  for (; k < a.k_end; ++k) {
    if (a.accept_out && lane == 0) a.accept_out[pid * (size_t)K + k] = 0;
    record(k + 1);
  }
  if (lane < S) {
    a.locs_state[(pid * S + lane) * 2 + 0] = sh;
    a.locs_state[(pid * S + lane) * 2 + 1] = sw;
    a.fluxes_state[pid * S + lane] = sfx;
  }
}

}  // namespace smcdet

using namespace smcdet;

extern "C" int smcdet_mh_chain(const smcdet_image_model_t* model, const smcdet_prior_t* prior,
                               const smcdet_mh_t* mh, const float* tiled_image, int32_t T,
                               int32_t C, int32_t S, const float* counts, float* locs_state,
                               float* fluxes_state, int32_t num_samples_total,
                               int32_t num_samples_burnin, int32_t keep_every_k,
                               int32_t k_begin, int32_t k_end, uint64_t seed, uint64_t offset,
                               const smcdet_mh_replay_t* replay, float* locs_out,
                               float* fluxes_out, int32_t* accept_out, int32_t* frozen,
                               void* stream) {
  int rc = validate_model(model);
  if (rc) return rc;
  rc = validate_prior(prior);
  if (rc) return rc;
  if (!mh || !tiled_image || !counts || !locs_state || !fluxes_state || !locs_out ||
      !fluxes_out)
    return set_error(SMCDET_EINVAL, "null buffer");
  if (T <= 0 || C <= 0 || T > 65535) return set_error(SMCDET_EUNSUPPORTED, "T=%d C=%d", T, C);
  if (S < 1 || S > 64) return set_error(SMCDET_EUNSUPPORTED, "S=%d outside 1..64", S);
  if (num_samples_total < 1 || num_samples_burnin < 0 || keep_every_k < 1 ||
      num_samples_burnin >= num_samples_total)
    return set_error(SMCDET_EINVAL, "bad sample counts total=%d burnin=%d keep=%d",
                     num_samples_total, num_samples_burnin, keep_every_k);
  if (k_begin < 0 || k_end < k_begin || k_end > num_samples_total - 1)
    return set_error(SMCDET_EINVAL, "iteration range [%d, %d) outside [0, %d)", k_begin, k_end,
                     num_samples_total - 1);
  if (replay && (!replay->comp || !replay->uloc || !replay->uflux || !replay->uacc))
    return set_error(SMCDET_EINVAL, "incomplete replay buffers");
  if (!(mh->locs_stdev > 0.f) || !(mh->fluxes_stdev > 0.f))
    return set_error(SMCDET_EINVAL, "proposal standard deviations must be > 0");
  if (k_end == k_begin && k_begin != 0) return SMCDET_OK;

  ChainArgs a{};
  a.m = make_dev_model(*model);
  a.pr = make_dev_prior(*prior);
  a.T = T;
  a.C = C;
  a.S = S;
  a.k_begin = k_begin;
  a.k_end = k_end;
  a.total = num_samples_total;
  a.burnin = num_samples_burnin;
  a.keep = keep_every_k;
  a.M = (num_samples_total - num_samples_burnin + keep_every_k - 1) / keep_every_k;
  a.sl = mh->locs_stdev;
  a.sf = mh->fluxes_stdev;
  a.rsl = 1.0f / a.sl;
  a.rsf = 1.0f / a.sf;
  a.lb_h = mh->locs_min_h;
  a.lb_w = mh->locs_min_w;
  a.ub_h = mh->locs_max_h;
  a.ub_w = mh->locs_max_w;
  a.lb_f = mh->fluxes_min;
  a.ub_f = mh->fluxes_max;
  a.k0 = (uint32_t)seed;
  a.k1 = (uint32_t)(seed >> 32);
  a.offset = offset;
  a.W2 = (2 * model->psf_radius + 1) * (2 * model->psf_radius + 1);
  a.img = tiled_image;
  a.counts = counts;
  a.locs_state = locs_state;
  a.fluxes_state = fluxes_state;
  a.locs_out = locs_out;
  a.fluxes_out = fluxes_out;
  a.accept_out = accept_out;
  a.frozen = frozen;
  if (replay) {
    a.r_comp = replay->comp;
    a.r_uloc = replay->uloc;
    a.r_uflux = replay->uflux;
    a.r_uacc = replay->uacc;
  }
  const size_t HWp = (size_t)model->H * model->W + kWave;
  const size_t lds = (2 * HWp + (size_t)kChainWaves * (HWp + 2 * (size_t)a.W2)) * sizeof(float);
  rc = ensure_lds((const void*)mh_chain_kernel, lds);
  if (rc) return rc;
  const dim3 grid((C + kChainWaves - 1) / kChainWaves, T);
  hipLaunchKernelGGL(mh_chain_kernel, grid, dim3(kChainBlock), lds, (hipStream_t)stream, a);
  return check_launch("smcdet_mh_chain");
}
