/*
 * mh_oracle.c — CPU ORACLE / CPU BASELINE (test infrastructure only).
 *
 * Plain-C float64 restatement of the reference's MH sweep with the reference's
 * arithmetic: every proposal re-renders every source and re-evaluates every
 * pixel (smcdet/kernel.py:26-130 -> sampler.py:87-91 -> images.py:28-76 +
 * :159-175 / :85-102, prior.py:67-75/:183-189/:220-226,
 * distributions.py:22-58).  Particles are independent and run in parallel
 * with OpenMP.  Used (a) by tests, checked against the reference's recorded
 * MH draws, and (b) as bench.py's `cpu_baseline` ("port") on the GPU box's
 * host cores.  Never linked into the product library.
 */
#define _GNU_SOURCE
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
 * One MH sweep over T*N particles.  image [T,H,W], counts [T,N], locs
 * [T,N,S,2] and fluxes [T,N,S] updated in place; tau [T].  Draws come from
 * the replay arrays (comp [K,T,N], uloc [K,T,N,2], uflux/uacc [K,T,N]) when
 * non-null, else from splitmix64 seeded by (seed, particle).  acc_last [T,N]
 * receives the accept flag of the last iteration.  Returns 0.
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
        const double nh = tn_sample(oh, mh->sl, mh->lb_h, mh->ub_h, uh);
        const double nw = tn_sample(ow, mh->sl, mh->lb_w, mh->ub_w, uw);
        const double nf = tn_sample(of, mh->sf, mh->lb_f, mh->ub_f, uf);
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
