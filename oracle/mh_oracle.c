/*
 * mh_oracle.c — CPU ORACLE / CPU BASELINE (test infrastructure only).
 *
 * Plain-C float64 restatement of the reference's MH sweep (and, below, of its
 * MALA sweep, smcdet/kernel.py:133-275) with the reference's
 * arithmetic: every proposal re-renders every source and re-evaluates every
 * pixel (smcdet/kernel.py:26-130 -> sampler.py:87-91 -> images.py:28-76 +
 * :159-175 / :85-102, prior.py:67-75/:183-189/:220-226,
 * distributions.py:22-58).  Particles are independent and run in parallel
 * with OpenMP.  Used (a) by tests, checked against the reference's recorded
 * MH draws, and (b) as bench.py's `cpu_baseline` ("port") on the GPU box's
 * host cores.  Never linked into the product library.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
  int model; /* 1 = M71 (Gaussian noise), 2 = basic (Poisson) */
  int H, W, R;
  double bg, g;
  double s1, s2, sp, beta, b, p0, norm; /* M71 PSF */
  double psf_stdev;                     /* basic PSF */
  double s0sq, eta;                     /* M71 noise */
} om_model_t;

typedef struct {
  int kind; /* 1 = M71Prior (truncated Pareto), 2 = ParetoStarPrior */
  double alpha;
  double lower;                      /* flux substituted for f == 0 (prior.py:189, :226) */
  double loc_low, loc_high_h, loc_high_w;
} om_prior_t;

typedef struct {
  int K;
  double sl, sf, lb_h, lb_w, ub_h, ub_w, lb_f, ub_f;
} om_mh_t;

static double psf_value(const om_model_t* m, double r2) {
  if (m->model == 1) {
    const double t1 = exp(-r2 / (2 * m->s1));
    const double t2 = m->b * exp(-r2 / (2 * m->s2));
    const double t3 = m->p0 * pow(1 + r2 / (m->beta * m->sp), -m->beta / 2);
    return (t1 + t2 + t3) / (1 + m->b + m->p0) / m->norm;
  }
  const double s = m->psf_stdev;
  return exp(-r2 / (2 * s * s) - log(s) - 0.5 * log(2 * M_PI));
}

/* images.py:28-76 + :159-175 / :85-102 */
static double loglik(const om_model_t* m, const float* x, const double* h, const double* w,
                     const double* f, int S, double* rate, const double* lgx) {
  const int H = m->H, W = m->W, R = m->R;
  for (int p = 0; p < H * W; ++p) rate[p] = 0.0;
  for (int s = 0; s < S; ++s) {
    const int fh = (int)floor(h[s]), fw = (int)floor(w[s]);
    const int r0 = fh - R < 0 ? 0 : fh - R, r1 = fh + R > H - 1 ? H - 1 : fh + R;
    const int c0 = fw - R < 0 ? 0 : fw - R, c1 = fw + R > W - 1 ? W - 1 : fw + R;
    for (int ph = r0; ph <= r1; ++ph)
      for (int pw = c0; pw <= c1; ++pw) {
        const double dh = ph + 0.5 - h[s], dw = pw + 0.5 - w[s];
        rate[ph * W + pw] += psf_value(m, dh * dh + dw * dw) * (m->g * f[s]);
      }
  }
  double ll = 0.0;
  for (int p = 0; p < H * W; ++p) {
    const double lam = rate[p] + m->bg, xp = x[p];
    if (m->model == 1) {
      const double v = m->s0sq + m->eta * lam;
      ll += -(xp - lam) * (xp - lam) / (2 * v) - 0.5 * log(v) - 0.5 * log(2 * M_PI);
    } else if (lam > 50000.0) {
      ll += -(xp - lam) * (xp - lam) / (2 * lam) - 0.5 * log(lam) - 0.5 * log(2 * M_PI);
    } else {
      ll += (xp == 0 ? 0.0 : xp * log(lam)) - lam - lgx[p];
    }
  }
  return ll;
}

static double Phi(double z) { return 0.5 * (1 + erf(z / sqrt(2.0))); }

/* inverse error function: Giles (2010) initial guess + two Newton steps */
static double erfinv_d(double y) {
  if (y <= -1) return -INFINITY;
  if (y >= 1) return INFINITY;
  double w = -log((1.0 - y) * (1.0 + y)), x;
  if (w < 6.25) {
    w -= 3.125;
    x = -3.6444120640178196996e-21;
    x = -1.685059138182016589e-19 + x * w;
    x = 1.2858480715256400167e-18 + x * w;
    x = 1.115787767802518096e-17 + x * w;
    x = -1.333171662854620906e-16 + x * w;
    x = 2.0972767875968561637e-17 + x * w;
    x = 6.6376381343583238325e-15 + x * w;
    x = -4.0545662729752068639e-14 + x * w;
    x = -8.1519341976054721522e-14 + x * w;
    x = 2.6335093153082322977e-12 + x * w;
    x = -1.2975133253453532498e-11 + x * w;
    x = -5.4154120542946279317e-11 + x * w;
    x = 1.051212273321532285e-09 + x * w;
    x = -4.1126339803469836976e-09 + x * w;
    x = -2.9070369957882005086e-08 + x * w;
    x = 4.2347877827932403518e-07 + x * w;
    x = -1.3654692000834678645e-06 + x * w;
    x = -1.3882523362786468719e-05 + x * w;
    x = 0.0001867342080340571352 + x * w;
    x = -0.00074070253416626697512 + x * w;
    x = -0.0060336708714301490533 + x * w;
    x = 0.24015818242558961693 + x * w;
    x = 1.6536545626831027356 + x * w;
  } else if (w < 16.0) {
    w = sqrt(w) - 3.25;
    x = 2.2137376921775787049e-09;
    x = 9.0756561938885390979e-08 + x * w;
    x = -2.7517406297064545428e-07 + x * w;
    x = 1.8239629214389227755e-08 + x * w;
    x = 1.5027403968909827627e-06 + x * w;
    x = -4.013867526981545969e-06 + x * w;
    x = 2.9234449089955446044e-06 + x * w;
    x = 1.2475304481671778723e-05 + x * w;
    x = -4.7318229009055733981e-05 + x * w;
    x = 6.8284851459573175448e-05 + x * w;
    x = 2.4031110387097893999e-05 + x * w;
    x = -0.0003550375203628474796 + x * w;
    x = 0.00095328937973738049703 + x * w;
    x = -0.0016882755560235047313 + x * w;
    x = 0.0024914420961078508066 + x * w;
    x = -0.0037512085075692412107 + x * w;
    x = 0.005370914553590063617 + x * w;
    x = 1.0052589676941592334 + x * w;
    x = 3.0838856104922207635 + x * w;
  } else {
    w = sqrt(w) - 5.0;
    x = -2.7109920616438573243e-11;
    x = -2.5556418169965252055e-10 + x * w;
    x = 1.5076572693500548083e-09 + x * w;
    x = -3.7894654401267369937e-09 + x * w;
    x = 7.6157012080783393804e-09 + x * w;
    x = -1.4960026627149240478e-08 + x * w;
    x = 2.9147953450901080826e-08 + x * w;
    x = -6.7711997758452339498e-08 + x * w;
    x = 2.2900482228026654717e-07 + x * w;
    x = -9.9298272942317002539e-07 + x * w;
    x = 4.5260625972231537039e-06 + x * w;
    x = -1.9681778105531670567e-05 + x * w;
    x = 7.5995277030017761139e-05 + x * w;
    x = -0.00021503011930044477347 + x * w;
    x = -0.00013871931833623122026 + x * w;
    x = 1.0103004648645343977 + x * w;
    x = 4.8499064014085844221 + x * w;
  }
  x *= y;
  for (int it = 0; it < 2; ++it) x -= (erf(x) - y) / (2.0 / sqrt(M_PI) * exp(-x * x));
  return x;
}

static double clampd(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }

static double tn_logZ(double mu, double sig, double lb, double ub) {
  double z = log(Phi((ub - mu) / sig) - Phi((lb - mu) / sig));
  if (isnan(z)) return 0.0;
  if (isinf(z)) return z > 0 ? 3.4028234663852886e38 : -3.4028234663852886e38;
  return z;
}

/* distributions.py:40-48 */
static double tn_sample(double mu, double sig, double lb, double ub, double u) {
  const double p = clampd(u, 1e-6, 1 - 1e-6);
  double pt = Phi((lb - mu) / sig) + p * exp(tn_logZ(mu, sig, lb, ub));
  pt = clampd(pt, 1e-6, 1 - 1e-6);
  return clampd(mu + sig * sqrt(2.0) * erfinv_d(2 * pt - 1), lb, ub);
}

static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static double urand(uint64_t* s) { return (double)(splitmix(s) >> 40) * (1.0 / 16777216.0); }

/*
 * Image log-likelihood of T*N particles (images.py:159-175 / :85-102), float64
 * accumulation as loglik() above: out[T*N].  For the oracle SMC runs
 * (tests/golden/make_oracle_stats.py).  Returns 0.
 */
int mh_oracle_loglik(const om_model_t* m, const float* image, const float* locs,
                     const float* fluxes, int T, int N, int S, int threads, double* out) {
  const int HW = m->H * m->W;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
  {
    double* h = malloc(sizeof(double) * S * 3);
    double* w = h + S;
    double* f = w + S;
    double* rate = malloc(sizeof(double) * HW * 2);
    double* lgx = rate + HW;
#pragma omp for schedule(static)
    for (long pid = 0; pid < (long)T * N; ++pid) {
      const float* x = image + (size_t)(pid / N) * HW;
      for (int p = 0; p < HW; ++p) lgx[p] = lgamma((double)x[p] + 1.0);
      for (int s = 0; s < S; ++s) {
        h[s] = locs[(pid * S + s) * 2 + 0];
        w[s] = locs[(pid * S + s) * 2 + 1];
        f[s] = fluxes[pid * S + s];
      }
      out[pid] = loglik(m, x, h, w, f, S, rate, lgx);
    }
    free(h);
    free(rate);
  }
  return 0;
}

/*
 * One MH sweep over T*N particles.  image [T,H,W], counts [T,N], locs
 * [T,N,S,2] and fluxes [T,N,S] updated in place; tau [T].  Draws come from
 * the replay arrays (comp [K,T,N], uloc [K,T,N,2], uflux/uacc [K,T,N]) when
 * non-null, else from splitmix64 seeded by (seed, particle).  acc_last [T,N]
 * receives the accept flag of the last iteration (2: the particle was frozen
 * by an upper-edge proposal, a rejection).  Returns 0.
 */
int mh_oracle_sweep(const om_model_t* m, const om_prior_t* pr, const om_mh_t* mh,
                    const float* image, const float* counts, float* locs, float* fluxes,
                    const float* tau, int T, int N, int S, const int32_t* comp,
                    const float* uloc, const float* uflux, const float* uacc, uint64_t seed,
                    int threads, uint8_t* acc_last) {
  const int HW = m->H * m->W;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
  {
    double* h = malloc(sizeof(double) * S * 3);
    double* w = h + S;
    double* f = w + S;
    double* rate = malloc(sizeof(double) * HW * 2);
    double* lgx = rate + HW;
#pragma omp for schedule(dynamic, 4)
    for (long pid = 0; pid < (long)T * N; ++pid) {
      const int t = (int)(pid / N);
      const float* x = image + (size_t)t * HW;
      for (int p = 0; p < HW; ++p) lgx[p] = lgamma((double)x[p] + 1.0);
      for (int s = 0; s < S; ++s) {
        h[s] = locs[(pid * S + s) * 2 + 0];
        w[s] = locs[(pid * S + s) * 2 + 1];
        f[s] = fluxes[pid * S + s];
      }
      const double cnt = counts[pid];
      uint64_t st = seed ^ (0xA5A5A5A5ull * (uint64_t)(pid + 1));
      double ll = loglik(m, x, h, w, f, S, rate, lgx);
      int acc = 0;
      for (int k = 0; k < mh->K; ++k) {
        int j;
        double uh, uw, uf, ua;
        if (comp) {
          const size_t r = ((size_t)k * T + t) * N + (pid % N);
          j = comp[r];
          uh = uloc[r * 2];
          uw = uloc[r * 2 + 1];
          uf = uflux[r];
          ua = uacc[r];
        } else {
          j = (int)(urand(&st) * S);
          if (j >= S) j = S - 1;
          uh = urand(&st);
          uw = urand(&st);
          uf = urand(&st);
          ua = urand(&st);
        }
        const double oh = h[j], ow = w[j], of = f[j];
        /* proposals as the reference's float32 state holds them */
        const double nh = (float)tn_sample(oh, mh->sl, mh->lb_h, mh->ub_h, uh);
        const double nw = (float)tn_sample(ow, mh->sl, mh->lb_w, mh->ub_w, uw);
        const double nf = (float)tn_sample(of, mh->sf, mh->lb_f, mh->ub_f, uf);
        /* a location on the box's upper edge has log prior -inf
         * (Uniform.log_prob(high), prior.py:73): rejected, and the reference's
         * cached target becomes -inf * 0 = NaN (kernel.py:125), which rejects
         * every remaining proposal of the sweep */
        if (nh >= pr->loc_high_h || nw >= pr->loc_high_w) {
          acc = 2; /* rejected, and frozen (reported as acc_last = 2) */
          break;
        }
        /* Hastings: the Normal log-densities cancel; log-mass-in-box terms remain */
        const double hast = tn_logZ(oh, mh->sl, mh->lb_h, mh->ub_h) -
                            tn_logZ(nh, mh->sl, mh->lb_h, mh->ub_h) +
                            tn_logZ(ow, mh->sl, mh->lb_w, mh->ub_w) -
                            tn_logZ(nw, mh->sl, mh->lb_w, mh->ub_w) +
                            tn_logZ(of, mh->sf, mh->lb_f, mh->ub_f) -
                            tn_logZ(nf, mh->sf, mh->lb_f, mh->ub_f);
        const double dprior = (j < cnt) ? -(pr->alpha + 1) * (log(nf) - log(of)) : 0.0;
        h[j] = nh;
        w[j] = nw;
        f[j] = nf;
        const double nll = loglik(m, x, h, w, f, S, rate, lgx);
        const double loga = dprior + tau[t] * (nll - ll) + hast;
        const double e = exp(loga);
        const double alpha = e > 1.0 ? 1.0 : e;
        acc = ua <= alpha;
        if (acc) {
          ll = nll;
        } else {
          h[j] = oh;
          w[j] = ow;
          f[j] = of;
        }
      }
      for (int s = 0; s < S; ++s) {
        locs[(pid * S + s) * 2 + 0] = (float)h[s];
        locs[(pid * S + s) * 2 + 1] = (float)w[s];
        fluxes[pid * S + s] = (float)f[s];
      }
      if (acc_last) acc_last[pid] = (uint8_t)acc;
    }
    free(h);
    free(rate);
  }
  return 0;
}

/* ------------------------------------------------------------------------
 * SingleComponentMALA.run (smcdet/kernel.py:133-275).
 *
 * The image log-likelihood, its gradient and the prior are float64 (the
 * gradient analytic: d loglik / d rate per pixel times d rate / d (h, w, f)
 * over the moved source's PSF window, as torch.autograd.grad computes it,
 * kernel.py:160-166 / :190-197).  The proposal machinery is float32 in the
 * reference's operation order (distributions.py:22-52 on torch float32
 * tensors), because its saturation points decide outcomes: Normal.cdf
 * saturates to exactly 0 or 1 a few sigma outside the box, the mass-in-box
 * log becomes -FLT_MAX (nan_to_num), and the float32 sums of kernel.py:220-251
 * then absorb the log target.  Location proposals clamped to the box's upper
 * edge have log prior -inf (torch Uniform.log_prob is -inf at `high`).
 * ---------------------------------------------------------------------- */
static const float kFltMax = 3.4028234663852886e38f;

static float cdf_f(float v, float mu, float rsig) {
  return 0.5f * (1.0f + erff((v - mu) * rsig / 1.41421356237309504880f));
}
static float nan_to_num_f(float x) {
  if (isnan(x)) return 0.0f;
  if (isinf(x)) return x > 0 ? kFltMax : -kFltMax;
  return x;
}
static float tn_logZ_f(float mu, float rsig, float lb, float ub) {
  return nan_to_num_f(logf(cdf_f(ub, mu, rsig) - cdf_f(lb, mu, rsig)));
}
static float tn_sample_f(float mu, float sig, float rsig, float lb, float ub, float u) {
  const float p = u < 1e-6f ? 1e-6f : (u > (float)(1.0 - 1e-6) ? (float)(1.0 - 1e-6) : u);
  float pt = cdf_f(lb, mu, rsig) + p * expf(tn_logZ_f(mu, rsig, lb, ub));
  pt = pt < 1e-6f ? 1e-6f : (pt > (float)(1.0 - 1e-6) ? (float)(1.0 - 1e-6) : pt);
  float x = mu + sig * (float)erfinv_d(2.0f * pt - 1.0f) * 1.41421356237309504880f;
  return x < lb ? lb : (x > ub ? ub : x);
}
/* Normal(mu, sig).log_prob(v) - log_prob_in_box, torch's operation order */
static float tn_logprob_f(float v, float mu, float sig, float rsig, float lb, float ub) {
  const float d = v - mu;
  const float lp = -(d * d) / (2.0f * (sig * sig)) - logf(sig) -
                   (float)0.91893853320467274178;
  return lp - tn_logZ_f(mu, rsig, lb, ub);
}

/* d phi / d r2 of the normalised PSF */
static double psf_dr2(const om_model_t* m, double r2) {
  if (m->model == 1) {
    const double t1 = exp(-r2 / (2 * m->s1)) / (2 * m->s1);
    const double t2 = m->b * exp(-r2 / (2 * m->s2)) / (2 * m->s2);
    const double t3 = m->p0 * 0.5 / m->sp * pow(1 + r2 / (m->beta * m->sp), -m->beta / 2 - 1);
    return -(t1 + t2 + t3) / (1 + m->b + m->p0) / m->norm;
  }
  return -psf_value(m, r2) / (2 * m->psf_stdev * m->psf_stdev);
}

/* d (per-pixel log-likelihood) / d rate */
static double dll_drate(const om_model_t* m, double x, double lam) {
  const double d = x - lam;
  if (m->model == 1) {
    const double v = m->s0sq + m->eta * lam;
    return d / v + m->eta * d * d / (2 * v * v) - m->eta / (2 * v);
  }
  if (lam > 50000.0) return d / lam + d * d / (2 * lam * lam) - 1 / (2 * lam);
  return x / lam - 1;
}

/* gradient of log_target w.r.t. (h_j, w_j, f_j); rate excludes background */
static void mala_grad(const om_model_t* m, const om_prior_t* pr, const float* x,
                      const double* rate, double h, double w, double f, int active,
                      double tau, double* g) {
  const int H = m->H, W = m->W, R = m->R;
  const int fh = (int)floor(h), fw = (int)floor(w);
  double gh = 0, gw = 0, gf = 0;
  for (int ph = fh - R; ph <= fh + R; ++ph)
    for (int pw = fw - R; pw <= fw + R; ++pw) {
      if (ph < 0 || ph >= H || pw < 0 || pw >= W) continue;
      const double dh = ph + 0.5 - h, dw = pw + 0.5 - w, r2 = dh * dh + dw * dw;
      const double e = dll_drate(m, x[ph * W + pw], rate[ph * W + pw] + m->bg) * m->g;
      const double dp = psf_dr2(m, r2);
      gf += e * psf_value(m, r2);
      gh += e * f * dp * (-2 * dh);
      gw += e * f * dp * (-2 * dw);
    }
  g[0] = tau * gh;
  g[1] = tau * gw;
  g[2] = tau * gf;
  if (active) g[2] -= (pr->alpha + 1) / (f == 0 ? pr->lower : f);
}

/* the state-dependent part of Prior.log_prob (prior.py:67-75 + :183-189 /
 * :220-226): -(alpha+1) log f per active source, the uniform location
 * density's support (-inf at or beyond `high`; -inf * 0 = nan for masked
 * sources) -- the count and normalising constants cancel in every ratio */
static double log_prior_var(const om_prior_t* pr, const double* h, const double* w,
                            const double* f, int S, double cnt) {
  double lp = 0;
  for (int s = 0; s < S; ++s) {
    const double act = s < cnt ? 1.0 : 0.0;
    const int in = h[s] >= pr->loc_low && h[s] < pr->loc_high_h && w[s] >= pr->loc_low &&
                   w[s] < pr->loc_high_w;
    lp += (in ? 0.0 : -INFINITY) * act;
    lp += -(pr->alpha + 1) * log(f[s] == 0 ? pr->lower : f[s]) * act;
  }
  return lp;
}

/*
 * One MALA sweep; arguments as mh_oracle_sweep (mh->sl / mh->sf are the
 * location / flux step sizes).  grad_out (nullable) [K,T,N,3] receives the
 * gradient at the current state w.r.t. the chosen source's (h, w, f) each
 * iteration, prop_out (nullable) [K,T,N,3] the proposal.
 */
int mala_oracle_sweep(const om_model_t* m, const om_prior_t* pr, const om_mh_t* mh,
                      const float* image, const float* counts, float* locs, float* fluxes,
                      const float* tau, int T, int N, int S, const int32_t* comp,
                      const float* uloc, const float* uflux, const float* uacc, uint64_t seed,
                      int threads, uint8_t* acc_last, float* grad_out, float* prop_out) {
  const int HW = m->H * m->W;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
  {
    double* h = malloc(sizeof(double) * S * 3);
    double* w = h + S;
    double* f = w + S;
    double* rate = malloc(sizeof(double) * HW * 3);
    double* rate_p = rate + HW;
    double* lgx = rate_p + HW;
    const float sl = (float)mh->sl, sf = (float)mh->sf;
    const float rsl = 1.0f / sl, rsf = 1.0f / sf;
    const float cl = 0.5f * (sl * sl), cf = 0.5f * (sf * sf);
    const float lbh = (float)mh->lb_h, lbw = (float)mh->lb_w, ubh = (float)mh->ub_h;
    const float ubw = (float)mh->ub_w, lbf = (float)mh->lb_f, ubf = (float)mh->ub_f;
#pragma omp for schedule(dynamic, 4)
    for (long pid = 0; pid < (long)T * N; ++pid) {
      const int t = (int)(pid / N);
      const float* x = image + (size_t)t * HW;
      for (int p = 0; p < HW; ++p) lgx[p] = lgamma((double)x[p] + 1.0);
      for (int s = 0; s < S; ++s) {
        h[s] = locs[(pid * S + s) * 2 + 0];
        w[s] = locs[(pid * S + s) * 2 + 1];
        f[s] = fluxes[pid * S + s];
      }
      const double cnt = counts[pid];
      const double tk = tau[t];
      uint64_t st = seed ^ (0x5A5A5A5Aull * (uint64_t)(pid + 1));
      double ll = loglik(m, x, h, w, f, S, rate, lgx);
      int acc = 0;
      for (int k = 0; k < mh->K; ++k) {
        int j;
        float uh, uw, uf, ua;
        const size_t r = ((size_t)k * T + t) * N + (pid % N);
        if (comp) {
          j = comp[r];
          uh = uloc[r * 2];
          uw = uloc[r * 2 + 1];
          uf = uflux[r];
          ua = uacc[r];
        } else {
          j = (int)(urand(&st) * S);
          if (j >= S) j = S - 1;
          uh = (float)urand(&st);
          uw = (float)urand(&st);
          uf = (float)urand(&st);
          ua = (float)urand(&st);
        }
        const int active = j < cnt;
        const double lp = log_prior_var(pr, h, w, f, S, cnt);
        const float lt = (float)(lp + tk * ll);
        double g[3];
        mala_grad(m, pr, x, rate, h[j], w[j], f[j], active, tk, g);
        const float oh = (float)h[j], ow = (float)w[j], of = (float)f[j];
        /* kernel.py:168-190: mean = x + 0.5 step^2 grad */
        const float mh_ = oh + cl * (float)g[0], mw_ = ow + cl * (float)g[1];
        const float mf_ = of + cf * (float)g[2];
        const float nh = tn_sample_f(mh_, sl, rsl, lbh, ubh, uh);
        const float nw = tn_sample_f(mw_, sl, rsl, lbw, ubw, uw);
        const float nf = tn_sample_f(mf_, sf, rsf, lbf, ubf, uf);
        if (grad_out)
          for (int d = 0; d < 3; ++d) grad_out[r * 3 + d] = (float)g[d];
        if (prop_out) {
          prop_out[r * 3 + 0] = nh;
          prop_out[r * 3 + 1] = nw;
          prop_out[r * 3 + 2] = nf;
        }
        /* denominator q(z'|z) (kernel.py:238-251) */
        const float dq_l = tn_logprob_f(nh, mh_, sl, rsl, lbh, ubh) +
                           tn_logprob_f(nw, mw_, sl, rsl, lbw, ubw);
        const float dq_f = tn_logprob_f(nf, mf_, sf, rsf, lbf, ubf);
        h[j] = nh;
        w[j] = nw;
        f[j] = nf;
        const double nll = loglik(m, x, h, w, f, S, rate_p, lgx);
        const double nlp = log_prior_var(pr, h, w, f, S, cnt);
        const float nlt = (float)(nlp + tk * nll);
        double gp[3];
        mala_grad(m, pr, x, rate_p, h[j], w[j], f[j], active, tk, gp);
        /* numerator q(z|z') (kernel.py:199-224) */
        const float rh = nh + cl * (float)gp[0], rw = nw + cl * (float)gp[1];
        const float rf = nf + cf * (float)gp[2];
        const float nq_l = tn_logprob_f(oh, rh, sl, rsl, lbh, ubh) +
                           tn_logprob_f(ow, rw, sl, rsl, lbw, ubw);
        const float nq_f = tn_logprob_f(of, rf, sf, rsf, lbf, ubf);
        const float num = (nlt + nq_l) + nq_f;
        const float den = (lt + dq_l) + dq_f;
        float alpha = expf(num - den);
        if (alpha > 1.0f) alpha = 1.0f;
        acc = ua <= alpha; /* nan -> reject */
        if (acc) {
          ll = nll;
          double* tmp = rate;
          rate = rate_p;
          rate_p = tmp;
        } else {
          h[j] = oh;
          w[j] = ow;
          f[j] = of;
        }
      }
      for (int s = 0; s < S; ++s) {
        locs[(pid * S + s) * 2 + 0] = (float)h[s];
        locs[(pid * S + s) * 2 + 1] = (float)w[s];
        fluxes[pid * S + s] = (float)f[s];
      }
      if (acc_last) acc_last[pid] = (uint8_t)acc;
    }
    free(h);
    free(rate < rate_p ? rate : rate_p);
  }
  return 0;
}
