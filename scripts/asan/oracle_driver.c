/*
 * Host sanitizer driver for the C oracle (oracle/mh_oracle.c): built with
 * -fsanitize=address,undefined by `make asan` and run by
 * tests/test_sanitizers.py (test infrastructure; SURVEY.md §5 "race
 * detection / sanitizers").  Runs the MH and MALA sweeps (M71 and Poisson
 * models, Philox-free splitmix draws and replayed draws, edge-of-box
 * locations, tiles whose windows are clipped) and checks the outputs are
 * finite and inside the prior box.
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/mh_oracle.c"

static int check(const float* locs, const float* fl, int n, double lo, double hi) {
  for (int i = 0; i < n; ++i) {
    if (!isfinite(fl[i]) || fl[i] < 0) return 1;
    if (!(locs[2 * i] >= lo && locs[2 * i] <= hi)) return 2;
    if (!(locs[2 * i + 1] >= lo && locs[2 * i + 1] <= hi)) return 3;
  }
  return 0;
}

int main(void) {
  const int T = 2, N = 7, S = 5, K = 23;
  int bad = 0;
  for (int model = 1; model <= 2; ++model)
    for (int H = 8; H <= 20; H += 12) {
      om_model_t m;
      memset(&m, 0, sizeof m);
      m.model = model;
      m.H = m.W = H;
      m.R = 8;
      m.bg = model == 1 ? 104.1 : 200.0;
      m.g = model == 1 ? 241.0 : 1.0;
      m.s1 = 1.107; m.s2 = 2.08; m.sp = 2.325; m.beta = 5.24; m.b = 0.73; m.p0 = 0.51;
      m.norm = 12.75;
      m.psf_stdev = 0.93;
      m.s0sq = 1e-10; m.eta = 1.936;
      om_prior_t p = {model, 0.214, model == 1 ? 0.0629 : 345.8, -4.0, H + 4.0, H + 4.0};
      om_mh_t mh = {K, 0.1, model == 1 ? 2.5 : 100.0, -4.0, -4.0, H + 4.0, H + 4.0,
                    p.lower, model == 1 ? 1804.7 : 1e6};
      const size_t TN = (size_t)T * N;
      float* img = malloc(sizeof(float) * T * H * H);
      float* counts = malloc(sizeof(float) * TN);
      float* locs = malloc(sizeof(float) * TN * S * 2);
      float* fl = malloc(sizeof(float) * TN * S);
      float tau[2] = {0.3f, 1.0f};
      uint8_t* acc = malloc(TN);
      int32_t* comp = malloc(sizeof(int32_t) * K * TN);
      float* ul = malloc(sizeof(float) * K * TN * 2);
      float* uf = malloc(sizeof(float) * K * TN);
      float* ua = malloc(sizeof(float) * K * TN);
      float* grad = malloc(sizeof(float) * K * TN * 3);
      float* prop = malloc(sizeof(float) * K * TN * 3);
      uint64_t z = 12345;
      for (int i = 0; i < T * H * H; ++i) img[i] = (float)(m.bg + (i % 7) * 3.0);
      for (size_t i = 0; i < TN; ++i) counts[i] = (float)S;
      for (size_t i = 0; i < TN * S; ++i) {
        z = z * 6364136223846793005ull + 1442695040888963407ull;
        const double u = (double)(z >> 11) / 9007199254740992.0;
        locs[2 * i] = (float)(-4.0 + u * (H + 8.0));
        locs[2 * i + 1] = (float)(H + 4.0 - 0.01 - u * 0.5);  /* near the upper edge */
        fl[i] = (float)(p.lower + 10.0 * u);
      }
      for (size_t i = 0; i < K * TN; ++i) {
        z = z * 6364136223846793005ull + 1442695040888963407ull;
        comp[i] = (int32_t)((z >> 33) % S);
        ul[2 * i] = (float)((z >> 20) & 0xffff) / 65536.0f;
        ul[2 * i + 1] = 0.9999999f;  /* proposals clamped onto the edge */
        uf[i] = (float)((z >> 4) & 0xffff) / 65536.0f;
        ua[i] = (float)((z >> 36) & 0xffff) / 65536.0f;
      }
      for (int replay = 0; replay < 2; ++replay) {
        mh_oracle_sweep(&m, &p, &mh, img, counts, locs, fl, tau, T, N, S,
                        replay ? comp : NULL, replay ? ul : NULL, replay ? uf : NULL,
                        replay ? ua : NULL, 7, 2, acc);
        bad |= check(locs, fl, (int)(TN * S), -4.0, H + 4.0);
        mala_oracle_sweep(&m, &p, &mh, img, counts, locs, fl, tau, T, N, S,
                          replay ? comp : NULL, replay ? ul : NULL, replay ? uf : NULL,
                          replay ? ua : NULL, 8, 2, acc, grad, prop);
        bad |= check(locs, fl, (int)(TN * S), -4.0, H + 4.0);
      }
      free(img); free(counts); free(locs); free(fl); free(acc); free(comp); free(ul);
      free(uf); free(ua); free(grad); free(prop);
    }
  printf("oracle sanitizer driver: %s\n", bad ? "FAILED" : "ok");
  return bad;
}
