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
#ifndef OM_F32 /* float64 build only */
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
#endif


/*
 * One MH sweep over T*N particles.  image [T,H,W], counts [T,N], locs
 * [T,N,S,2] and fluxes [T,N,S] updated in place; tau [T].  Draws come from
 * the replay arrays (comp [K,T,N], uloc [K,T,N,2], uflux/uacc [K,T,N]) when
 * non-null, else from splitmix64 seeded by (seed, particle).  acc_last [T,N]
 * receives the accept flag of the last iteration (2: the particle was frozen
 * by an upper-edge proposal, a rejection).  Returns 0.
 */
#ifndef OM_F32 /* float64 build only */
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
#endif


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
#ifndef OM_F32 /* float64 build only */
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
#endif


/* ------------------------------------------------------------------------
 * The MH sweep again, with cached per-source PSF windows, in `real`
 * arithmetic (the oracle's statistics runs, tests/golden/make_oracle_stats.py).
 *
 * A proposal moves one source, so only its new window is evaluated; the rate
 * of every pixel in the bounding box of the old and new windows is re-summed
 * from the cached contributions in source order, and the log-likelihood is
 * re-summed over all pixels in pixel order from cached per-pixel terms.
 * Every value is therefore the one the full re-render of mh_oracle_sweep
 * computes, with the same operations in the same order: in the float64 build
 * the two sweeps are bit-identical (tests/test_oracle_cached.py), at ~1/4 of
 * the cost.
 *
 * Built twice (oracle/Makefile):
 *   libmh_oracle.so      real = double, the float64 oracle above;
 *   libmh_oracle_f32.so  real = float (-DOM_F32): the reference's float32
 *     arithmetic class -- PSF from r = |p + 0.5 - loc| and r**2
 *     (images.py:45, :137-145), rate = sum_s psf * (adu * f) + B
 *     (:162-167), torch's Normal.log_prob form (var = scale**2, log scale)
 *     summed in float32 (:169-175), float32 proposals and Hastings terms
 *     (distributions.py:40-52) and log target = log prior + tau * loglik with
 *     log numerator / denominator composed as kernel.py:64-116 does.
 * ---------------------------------------------------------------------- */
#ifdef OM_F32
typedef float real;
#define R_EXP expf
#define R_LOG logf
#define R_POW powf
#define R_SQRT sqrtf
#define R_FLOOR floorf
#else
typedef double real;
#define R_EXP exp
#define R_LOG log
#define R_POW pow
#define R_SQRT sqrt
#define R_FLOOR floor
#endif

typedef struct {
  int fh, fw;         /* window anchor floor(loc) */
  int r0, r1, c0, c1; /* window clipped to the tile (r0 > r1: empty) */
} om_win_t;

static void win_of(const om_model_t* m, real h, real w, om_win_t* d) {
  const int R = m->R;
  d->fh = (int)R_FLOOR(h);
  d->fw = (int)R_FLOOR(w);
  d->r0 = d->fh - R < 0 ? 0 : d->fh - R;
  d->r1 = d->fh + R > m->H - 1 ? m->H - 1 : d->fh + R;
  d->c0 = d->fw - R < 0 ? 0 : d->fw - R;
  d->c1 = d->fw + R > m->W - 1 ? m->W - 1 : d->fw + R;
}

static inline int win_has(const om_win_t* d, int ph, int pw) {
  return ph >= d->r0 && ph <= d->r1 && pw >= d->c0 && pw <= d->c1;
}

/* psf(pixel) * (adu * f) of one source over its clipped window, into
 * c[(ph - fh + R) * (2R + 1) + (pw - fw + R)] */
static void contrib(const om_model_t* m, real h, real w, real f, const om_win_t* d, real* c) {
  const int R = m->R, D = 2 * R + 1;
#ifdef OM_F32
  const real gf = (real)m->g * f;
#endif
  for (int ph = d->r0; ph <= d->r1; ++ph)
    for (int pw = d->c0; pw <= d->c1; ++pw) {
      real v;
#ifdef OM_F32
      /* images.py:31-45: pixel = floor(loc) + offset; r = |pixel + 0.5 - loc| */
      const real dh = ((real)ph + 0.5f) - h, dw = ((real)pw + 0.5f) - w;
      const real r = R_SQRT(dh * dh + dw * dw), r2 = r * r;
      if (m->model == 1) {
        const real t1 = R_EXP(-r2 / (real)(2 * m->s1));
        const real t2 = (real)m->b * R_EXP(-r2 / (real)(2 * m->s2));
        const real t3 = (real)m->p0 * R_POW(1 + r2 / (real)(m->beta * m->sp), (real)(-m->beta / 2));
        v = ((t1 + t2) + t3) / (real)(1 + m->b + m->p0) / (real)m->norm;
      } else {
        const real s = (real)m->psf_stdev;
        v = R_EXP(-r2 / (2 * s * s) - R_LOG(s) - (real)(0.5 * log(2 * M_PI)));
      }
      v = v * gf;
#else
      const double dh = ph + 0.5 - h, dw = pw + 0.5 - w;
      v = psf_value(m, dh * dh + dw * dw) * (m->g * f);
#endif
      c[(ph - d->fh + R) * D + (pw - d->fw + R)] = v;
    }
}

/* one pixel's log-likelihood term at rate (without background) `rate` */
static inline real pix_term(const om_model_t* m, real xp, real rate, real lgx) {
  const real lam = rate + (real)m->bg;
#ifdef OM_F32
  if (m->model == 1) {
    /* Normal(lam, sqrt(s0 + eta lam)).log_prob(x): torch's operation order */
    const real scale = R_SQRT((real)m->s0sq + (real)m->eta * lam);
    const real var = scale * scale;
    const real d = xp - lam;
    return -(d * d) / (2 * var) - R_LOG(scale) - (real)0.91893853320467274178;
  } else if (lam > 50000.0f) {
    const real scale = R_SQRT(lam), var = scale * scale, d = xp - lam;
    return -(d * d) / (2 * var) - R_LOG(scale) - (real)0.91893853320467274178;
  }
  return (xp == 0 ? 0.0f : xp * R_LOG(lam)) - lam - lgx;
#else
  if (m->model == 1) {
    const double v = m->s0sq + m->eta * lam;
    return -(xp - lam) * (xp - lam) / (2 * v) - 0.5 * log(v) - 0.5 * log(2 * M_PI);
  } else if (lam > 50000.0) {
    return -(xp - lam) * (xp - lam) / (2 * lam) - 0.5 * log(lam) - 0.5 * log(2 * M_PI);
  }
  return (xp == 0 ? 0.0 : xp * log(lam)) - lam - lgx;
#endif
}

typedef struct {
  int S, HW, D2;
  real *h, *w, *f;
  om_win_t* win;
  real* cv;   /* [S][D2] cached contributions */
  real* cnew; /* [D2] */
  real* term; /* [HW] */
  real* tb;   /* [HW] bounding-box terms */
  real* lgx;  /* [HW] */
} om_ws_t;

static void ws_alloc(om_ws_t* s, const om_model_t* m, int S) {
  const int D = 2 * m->R + 1;
  s->S = S;
  s->HW = m->H * m->W;
  s->D2 = D * D;
  s->h = malloc(sizeof(real) * 3 * S);
  s->w = s->h + S;
  s->f = s->w + S;
  s->win = malloc(sizeof(om_win_t) * S);
  s->cv = malloc(sizeof(real) * ((size_t)S + 1) * s->D2);
  s->cnew = s->cv + (size_t)S * s->D2;
  s->term = malloc(sizeof(real) * 3 * s->HW);
  s->tb = s->term + s->HW;
  s->lgx = s->tb + s->HW;
}

static void ws_free(om_ws_t* s) {
  free(s->h);
  free(s->win);
  free(s->cv);
  free(s->term);
}

/* rate (without background) at pixel (ph, pw): the cached contributions of
 * the sources whose window holds it, summed in source order; source j's
 * from cj / wj instead of the cache when cj != NULL */
static inline real rate_at(const om_model_t* m, const om_ws_t* s, int ph, int pw, int j,
                           const real* cj, const om_win_t* wj) {
  const int R = m->R, D = 2 * R + 1;
  real r = 0;
  for (int k = 0; k < s->S; ++k) {
    const om_win_t* d = (k == j && cj) ? wj : &s->win[k];
    if (!win_has(d, ph, pw)) continue;
    const real* c = (k == j && cj) ? cj : s->cv + (size_t)k * s->D2;
    r += c[(ph - d->fh + R) * D + (pw - d->fw + R)];
  }
  return r;
}

/* render every source into the cache and the per-pixel terms; returns the
 * log-likelihood (the sum of the terms in pixel order, as loglik()) */
static real ws_render(const om_model_t* m, om_ws_t* s, const float* x) {
  for (int k = 0; k < s->S; ++k) {
    win_of(m, s->h[k], s->w[k], &s->win[k]);
    contrib(m, s->h[k], s->w[k], s->f[k], &s->win[k], s->cv + (size_t)k * s->D2);
  }
  real ll = 0;
  for (int ph = 0; ph < m->H; ++ph)
    for (int pw = 0; pw < m->W; ++pw) {
      const int p = ph * m->W + pw;
      s->term[p] = pix_term(m, x[p], rate_at(m, s, ph, pw, -1, NULL, NULL), s->lgx[p]);
      ll += s->term[p];
    }
  return ll;
}

/* log-likelihood with source j moved to (h, w, f) (the caller has set
 * s->h/w/f[j]); its window and contributions into *wj / s->cnew, the terms
 * of the bounding box [b0..b1] x [b2..b3] of its old and new windows into
 * s->tb (row-major over the box) */
static real ws_propose(const om_model_t* m, om_ws_t* s, const float* x, int j, om_win_t* wj,
                       int* bb) {
  win_of(m, s->h[j], s->w[j], wj);
  contrib(m, s->h[j], s->w[j], s->f[j], wj, s->cnew);
  const om_win_t* o = &s->win[j];
  const int oe = o->r0 > o->r1 || o->c0 > o->c1, ne = wj->r0 > wj->r1 || wj->c0 > wj->c1;
  int b0, b1, b2, b3;
  if (oe && ne) {
    b0 = 0, b1 = -1, b2 = 0, b3 = -1;
  } else if (oe) {
    b0 = wj->r0, b1 = wj->r1, b2 = wj->c0, b3 = wj->c1;
  } else if (ne) {
    b0 = o->r0, b1 = o->r1, b2 = o->c0, b3 = o->c1;
  } else {
    b0 = o->r0 < wj->r0 ? o->r0 : wj->r0;
    b1 = o->r1 > wj->r1 ? o->r1 : wj->r1;
    b2 = o->c0 < wj->c0 ? o->c0 : wj->c0;
    b3 = o->c1 > wj->c1 ? o->c1 : wj->c1;
  }
  bb[0] = b0, bb[1] = b1, bb[2] = b2, bb[3] = b3;
  const int bw = b3 - b2 + 1;
  for (int ph = b0; ph <= b1; ++ph)
    for (int pw = b2; pw <= b3; ++pw) {
      const int p = ph * m->W + pw;
      s->tb[(ph - b0) * bw + (pw - b2)] =
          pix_term(m, x[p], rate_at(m, s, ph, pw, j, s->cnew, wj), s->lgx[p]);
    }
  real ll = 0;
  for (int ph = 0; ph < m->H; ++ph) {
    const int inr = ph >= b0 && ph <= b1;
    for (int pw = 0; pw < m->W; ++pw)
      ll += (inr && pw >= b2 && pw <= b3) ? s->tb[(ph - b0) * bw + (pw - b2)]
                                          : s->term[ph * m->W + pw];
  }
  return ll;
}

static void ws_accept(const om_model_t* m, om_ws_t* s, int j, const om_win_t* wj, const int* bb) {
  s->win[j] = *wj;
  memcpy(s->cv + (size_t)j * s->D2, s->cnew, sizeof(real) * s->D2);
  const int bw = bb[3] - bb[2] + 1;
  for (int ph = bb[0]; ph <= bb[1]; ++ph)
    for (int pw = bb[2]; pw <= bb[3]; ++pw)
      s->term[ph * m->W + pw] = s->tb[(ph - bb[0]) * bw + (pw - bb[2])];
}

#ifdef OM_F32
/* the state-dependent log prior in float32 (prior.py:67-75 + :220-226 /
 * :183-189): per active source 2 x log(1 / (high - low)) + the flux term
 * log_norm - (alpha + 1) log f, masked-summed over sources in order */
static float log_prior_f(const om_prior_t* pr, const float* f, int S, double cnt, float lu_h,
                         float lu_w, float lnorm) {
  float lp = 0.0f;
  for (int s = 0; s < S; ++s) {
    const float act = s < cnt ? 1.0f : 0.0f;
    lp += (lu_h + lu_w) * act;
  }
  for (int s = 0; s < S; ++s) {
    const float act = s < cnt ? 1.0f : 0.0f;
    const float fv = f[s] == 0 ? (float)pr->lower : f[s];
    lp += (lnorm - ((float)pr->alpha + 1.0f) * logf(fv)) * act;
  }
  return lp;
}
#endif

/*
 * mh_oracle_sweep with the cached re-render; same arguments and results (and
 * the same seeded stream).  `upper` is the flux prior's upper bound (used by
 * the float32 build's log-prior constant only).
 */
int mh_oracle_sweep_cached(const om_model_t* m, const om_prior_t* pr, const om_mh_t* mh,
                           const float* image, const float* counts, float* locs, float* fluxes,
                           const float* tau, int T, int N, int S, const int32_t* comp,
                           const float* uloc, const float* uflux, const float* uacc,
                           uint64_t seed, int threads, uint8_t* acc_last, double upper) {
  const int HW = m->H * m->W;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#ifdef OM_F32
  const float sl = (float)mh->sl, sf = (float)mh->sf;
  const float rsl = 1.0f / sl, rsf = 1.0f / sf;
  const float lbh = (float)mh->lb_h, lbw = (float)mh->lb_w, ubh = (float)mh->ub_h;
  const float ubw = (float)mh->ub_w, lbf = (float)mh->lb_f, ubf = (float)mh->ub_f;
  const float lu_h = -logf((float)pr->loc_high_h - (float)pr->loc_low);
  const float lu_w = -logf((float)pr->loc_high_w - (float)pr->loc_low);
  const float a = (float)pr->alpha, L = (float)pr->lower, U = (float)upper;
  const float lnorm = logf(a) + a * logf(L) + a * logf(U) - logf(powf(U, a) - powf(L, a));
#else
  (void)upper;
#endif
#pragma omp parallel
  {
    om_ws_t ws;
    ws_alloc(&ws, m, S);
#pragma omp for schedule(dynamic, 4)
    for (long pid = 0; pid < (long)T * N; ++pid) {
      const int t = (int)(pid / N);
      const float* x = image + (size_t)t * HW;
      for (int p = 0; p < HW; ++p) ws.lgx[p] = (real)lgamma((double)x[p] + 1.0);
      for (int s = 0; s < S; ++s) {
        ws.h[s] = locs[(pid * S + s) * 2 + 0];
        ws.w[s] = locs[(pid * S + s) * 2 + 1];
        ws.f[s] = fluxes[pid * S + s];
      }
      const double cnt = counts[pid];
      uint64_t st = seed ^ (0xA5A5A5A5ull * (uint64_t)(pid + 1));
      real ll = ws_render(m, &ws, x);
#ifdef OM_F32
      float lt = log_prior_f(pr, ws.f, S, cnt, lu_h, lu_w, lnorm) + tau[t] * ll;
#endif
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
        const real oh = ws.h[j], ow = ws.w[j], of = ws.f[j];
#ifdef OM_F32
        const float nh = tn_sample_f(oh, sl, rsl, lbh, ubh, (float)uh);
        const float nw = tn_sample_f(ow, sl, rsl, lbw, ubw, (float)uw);
        const float nf = tn_sample_f(of, sf, rsf, lbf, ubf, (float)uf);
#else
        const double nh = (float)tn_sample(oh, mh->sl, mh->lb_h, mh->ub_h, uh);
        const double nw = (float)tn_sample(ow, mh->sl, mh->lb_w, mh->ub_w, uw);
        const double nf = (float)tn_sample(of, mh->sf, mh->lb_f, mh->ub_f, uf);
#endif
        if (nh >= pr->loc_high_h || nw >= pr->loc_high_w) {
          acc = 2; /* upper-edge proposal: rejected and frozen (see mh_oracle_sweep) */
          break;
        }
        ws.h[j] = nh;
        ws.w[j] = nw;
        ws.f[j] = nf;
        om_win_t wj;
        int bb[4];
        const real nll = ws_propose(m, &ws, x, j, &wj, bb);
#ifdef OM_F32
        /* kernel.py:64-116: TruncatedDiagonalMVN(proposed).log_prob(prev) etc. */
        const float nq_l = tn_logprob_f(oh, nh, sl, rsl, lbh, ubh) +
                           tn_logprob_f(ow, nw, sl, rsl, lbw, ubw);
        const float nq_f = tn_logprob_f(of, nf, sf, rsf, lbf, ubf);
        const float dq_l = tn_logprob_f(nh, oh, sl, rsl, lbh, ubh) +
                           tn_logprob_f(nw, ow, sl, rsl, lbw, ubw);
        const float dq_f = tn_logprob_f(nf, of, sf, rsf, lbf, ubf);
        const float lt_p = log_prior_f(pr, ws.f, S, cnt, lu_h, lu_w, lnorm) + tau[t] * nll;
        const float num = (lt_p + nq_l) + nq_f;
        const float den = (lt + dq_l) + dq_f;
        float alpha = expf(num - den);
        if (alpha > 1.0f) alpha = 1.0f;
        acc = (float)ua <= alpha;
        if (acc) lt = lt_p;
#else
        const double hast = tn_logZ(oh, mh->sl, mh->lb_h, mh->ub_h) -
                            tn_logZ(nh, mh->sl, mh->lb_h, mh->ub_h) +
                            tn_logZ(ow, mh->sl, mh->lb_w, mh->ub_w) -
                            tn_logZ(nw, mh->sl, mh->lb_w, mh->ub_w) +
                            tn_logZ(of, mh->sf, mh->lb_f, mh->ub_f) -
                            tn_logZ(nf, mh->sf, mh->lb_f, mh->ub_f);
        const double dprior = (j < cnt) ? -(pr->alpha + 1) * (log(nf) - log(of)) : 0.0;
        const double loga = dprior + tau[t] * (nll - ll) + hast;
        const double e = exp(loga);
        const double alpha = e > 1.0 ? 1.0 : e;
        acc = ua <= alpha;
#endif
        if (acc) {
          ll = nll;
          ws_accept(m, &ws, j, &wj, bb);
        } else {
          ws.h[j] = oh;
          ws.w[j] = ow;
          ws.f[j] = of;
        }
      }
      for (int s = 0; s < S; ++s) {
        locs[(pid * S + s) * 2 + 0] = (float)ws.h[s];
        locs[(pid * S + s) * 2 + 1] = (float)ws.w[s];
        fluxes[pid * S + s] = (float)ws.f[s];
      }
      if (acc_last) acc_last[pid] = (uint8_t)acc;
    }
    ws_free(&ws);
  }
  return 0;
}

/* image log-likelihoods of T*N particles in `real` arithmetic (float64
 * build: = mh_oracle_loglik bit for bit) */
int mh_oracle_loglik_cached(const om_model_t* m, const float* image, const float* locs,
                            const float* fluxes, int T, int N, int S, int threads, double* out) {
  const int HW = m->H * m->W;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
  {
    om_ws_t ws;
    ws_alloc(&ws, m, S);
#pragma omp for schedule(static)
    for (long pid = 0; pid < (long)T * N; ++pid) {
      const float* x = image + (size_t)(pid / N) * HW;
      for (int p = 0; p < HW; ++p) ws.lgx[p] = (real)lgamma((double)x[p] + 1.0);
      for (int s = 0; s < S; ++s) {
        ws.h[s] = locs[(pid * S + s) * 2 + 0];
        ws.w[s] = locs[(pid * S + s) * 2 + 1];
        ws.f[s] = fluxes[pid * S + s];
      }
      out[pid] = ws_render(m, &ws, x);
    }
    ws_free(&ws);
  }
  return 0;
}
