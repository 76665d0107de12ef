// Tile-pass tempering probe: cycles of the Brent root search (tile.h
// block_brentq) split into its f evaluations (the workgroup ESS reduction)
// and its control logic, one 512- or 256-thread workgroup, N = 4096
// log-likelihoods at three spreads.  Modes:
//   0  f(top) + brentq with the scalar objective
//   1  16 evaluations of the scalar objective
//   2  the select-form brentq on a closed-form f (no reduction: the control
//      logic alone)
//   3  16 evaluations of tile.h's (packed) block_ess_objective
//   4  f(top) + the select-form brentq with the packed objective
//   5  4 phase-stamped evaluations of the candidate
//   6  f(top) + tile.h's (branchy) brentq with the packed objective (mode 4's
//      root, bit for bit)
//   7  tile.h's brentq on the closed-form f
// (modes 0 and 1: the scalar objective as the tile pass had it before)
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I smcdet_amd/csrc
//        scripts/probe/brent_probe.hip -o scripts/probe/brent_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "tile.h"

using namespace smcdet;

// tile.h's scalar objective before the packed form (A/B reference)
template <int NT, int PER>
__device__ __forceinline__ double objective_scalar(const TileLL<NT, PER>& ll, int N, float lmax,
                                                      double delta, double thr, TileRed* red,
                                                      int& parity) {
#pragma clang fp contract(off)
  constexpr int VPT = VLayout<NT>::VPT;
  const float df = (float)delta;
  const float m = df * lmax;  // = max_i fl(df*l_i): rounding is monotone
  float s1[VPT], s2[VPT];
#pragma unroll
  for (int h = 0; h < VPT; ++h) {
    float e1[PER], e2[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const float e = ll.valid(h, j, N) ? fast_exp2((df * ll.l[h][j] - m) * kLog2e) : 0.f;
      e1[j] = e;
      e2[j] = e * e;
    }
    s1[h] = tree_sum(e1);
    s2[h] = tree_sum(e2);
  }
  float S1, S2;
  vblock_sum2f<NT>(s1, s2, S1, S2, red, parity);
  const double d1 = (double)S1;
  return ddiv(d1 * d1, (double)S2) - thr;
}


// the select form of brentq (measured in round 4, not adopted): the bracket
// update, the swap and the step choice as v_cndmask, both candidate steps
// computed every iteration
template <class F>
__device__ double brentq_select(F&& f, double xa, double xb, double fa, double fb) {
#pragma clang fp contract(off)
  const double xtol = 1e-6, rtol = 1e-6;
  double xpre = xa, xcur = xb, xblk = 0., fpre = fa, fcur = fb, fblk = 0., spre = 0., scur = 0.;
  if (fpre == 0.0) return xpre;
  if (fcur == 0.0) return xcur;
  for (int it = 0; it < 100; ++it) {
    const bool flip = fpre != 0 && fcur != 0 && (signbit(fpre) != signbit(fcur));
    const double s0 = xcur - xpre;
    xblk = flip ? xpre : xblk;
    fblk = flip ? fpre : fblk;
    spre = flip ? s0 : spre;
    scur = flip ? s0 : scur;
    const bool sw = fabs(fblk) < fabs(fcur);
    const double xc = sw ? xblk : xcur, fc = sw ? fblk : fcur;
    xblk = sw ? xcur : xblk;
    fblk = sw ? fcur : fblk;
    xpre = sw ? xcur : xpre;
    fpre = sw ? fcur : fpre;
    xcur = xc;
    fcur = fc;
    const double delta = (xtol + rtol * fabs(xcur)) / 2;
    const double sbis = (xblk - xcur) / 2;
    if (fcur == 0 || fabs(sbis) < delta) return xcur;
    const double si = ddiv(-fcur * (xcur - xpre), fcur - fpre);
    const double dpre = ddiv(fpre - fcur, xpre - xcur);
    const double dblk = ddiv(fblk - fcur, xblk - xcur);
    const double se = ddiv(-fcur * (fblk * dblk - fpre * dpre), dblk * dpre * (fblk - fpre));
    const double stry = xpre == xblk ? si : se;
    const bool interp = fabs(spre) > delta && fabs(fcur) < fabs(fpre);
    const bool take = interp && 2 * fabs(stry) < fmin(fabs(spre), 3 * fabs(sbis) - delta);
    spre = take ? scur : sbis;
    scur = take ? stry : sbis;
    xpre = xcur;
    fpre = fcur;
    xcur += fabs(scur) > delta ? scur : (sbis > 0 ? delta : -delta);
    fcur = f(xcur);
  }
  return xcur;
}



struct Out {
  double x;
  int n;
  long long cycles;
  long long ph[6];
};

// one f evaluation of block_ess_objective_pk, stamped: element work, wave
// DPP sums, LDS slot write + barrier, partial combine, double ratio
template <int NT, int PER>
__device__ double stamped_f(const TileLL<NT, PER>& ll, int N, float lm, double delta, double thr,
                            TileRed* red, int& parity, long long* ph) {
#pragma clang fp contract(off)
  constexpr int VPT = VLayout<NT>::VPT;
  const int lane = threadIdx.x & 63;
  ph[0] = clock64();
  const float df = (float)delta;
  const float m = df * lm;
  float s1[VPT], s2[VPT];
#pragma unroll
  for (int h = 0; h < VPT; ++h) {
    f2 E[PER / 2], Q[PER / 2];
#pragma unroll
    for (int k = 0; k < PER / 2; ++k) {
      f2 v = f2{ll.l[h][2 * k], ll.l[h][2 * k + 1]} * df;
      v = (v - m) * kLog2e;
      const f2 e = exp2_2(v);
      E[k] = e;
      Q[k] = e * e;
    }
    const f2 se = tree_sum(E), sq = tree_sum(Q);
    s1[h] = se.x + se.y;
    s2[h] = sq.x + sq.y;
  }
  __builtin_amdgcn_s_waitcnt(0);
  asm volatile("" ::"v"(s1[0]), "v"(s2[0]));
  ph[1] = clock64();
  const int k = parity;
  parity ^= 1;
#pragma unroll
  for (int h = 0; h < VPT; ++h) {
    float x = s1[h], y = s2[h];
    wave_sum2(x, y);
    asm volatile("" ::"v"(x), "v"(y));
    if (h == 0) ph[2] = clock64();
    if (lane == 0) {
      red->f2[k][vwave<NT>(h)][0] = x;
      red->f2[k][vwave<NT>(h)][1] = y;
    }
  }
  __syncthreads();
  ph[3] = clock64();
  float S1, S2;
  slot_tree2(red->f2[k][lane & 7][(lane >> 3) & 1], S1, S2);
  asm volatile("" ::"v"(S1), "v"(S2));
  ph[4] = clock64();
  const double d1 = (double)S1;
  const double r = ddiv(d1 * d1, (double)S2) - thr;
  asm volatile("" ::"v"(r));
  ph[5] = clock64();
  return r;
}

template <int NT, int MODE>
__global__ __launch_bounds__(NT) void brent_probe(const float* __restrict__ llg, int N, double thr,
                                                  double sig2, Out* out) {
  constexpr int PER = 8;
  constexpr int VPT = VLayout<NT>::VPT;
  __shared__ TileRed red;
  int parity = 0;
  TileLL<NT, PER> ll;
#pragma unroll
  for (int h = 0; h < VPT; ++h)
#pragma unroll
    for (int j = 0; j < PER; ++j) ll.l[h][j] = ll.valid(h, j, N) ? llg[vthread<NT>(h) + j * kTB] : 0.f;
  float lmv[VPT];
#pragma unroll
  for (int h = 0; h < VPT; ++h) {
    lmv[h] = -INFINITY;
#pragma unroll
    for (int j = 0; j < PER; ++j)
      if (ll.valid(h, j, N)) lmv[h] = fmaxf(lmv[h], ll.l[h][j]);
  }
  const float lm = vblock_max<NT>(lmv, &red, parity);
  int n = 0;
  auto f = [&](double x) -> double {
    ++n;
    if constexpr (MODE == 0 || MODE == 1) {
      return objective_scalar(ll, N, lm, x, thr, &red, parity);
    } else if constexpr (MODE == 3 || MODE == 4 || MODE == 6) {
      return block_ess_objective(ll, N, lm, x, thr, &red, parity);
    } else {  // ESS of log-normal weights, N exp(-x^2 sigma^2)
      return (double)N * (double)__expf((float)(-x * x * sig2)) - thr;
    }
  };
  __syncthreads();
  const long long t0 = clock64();
  double r = 0.0;
  long long ph[6] = {0, 0, 0, 0, 0, 0};
  if constexpr (MODE == 5) {
    for (int k = 0; k < 4; ++k) r += stamped_f(ll, N, lm, ldexp(1.0, -k), thr, &red, parity, ph);
  } else if constexpr (MODE == 1 || MODE == 3) {
    for (int k = 0; k < 16; ++k) r += f(ldexp(1.0, -k));
  } else {
    const double ftop = f(1.0);
    r = 1.0;
    if (ftop < 0.0) {
      if constexpr (MODE == 0 || MODE == 6 || MODE == 7)
        r = block_brentq(f, 0.0, 1.0, (double)N - thr, ftop);
      else
        r = brentq_select(f, 0.0, 1.0, (double)N - thr, ftop);
    }
  }
  const long long t1 = clock64();
  if (threadIdx.x == 0) {
    *out = Out{r, n, t1 - t0, {}};
    for (int i = 0; i < 6; ++i) out->ph[i] = ph[i] - ph[0];
  }
}

template <int NT, int MODE>
static Out run(const float* d_ll, int N, double sig2, Out* d_out) {
  Out best{0, 0, 1ll << 60};
  for (int rep = 0; rep < 5; ++rep) {
    brent_probe<NT, MODE><<<1, NT>>>(d_ll, N, 0.5 * N, sig2, d_out);
    Out o;
    hipMemcpy(&o, d_out, sizeof(Out), hipMemcpyDeviceToHost);
    if (o.cycles < best.cycles) best = o;
  }
  return best;
}

template <int NT>
static void sweep(const float* d_ll, int N, double sig2, Out* d_out) {
  const Out a = run<NT, 0>(d_ll, N, sig2, d_out);
  const Out b = run<NT, 1>(d_ll, N, sig2, d_out);
  const Out c = run<NT, 2>(d_ll, N, sig2, d_out);
  const Out d = run<NT, 3>(d_ll, N, sig2, d_out);
  const Out e = run<NT, 4>(d_ll, N, sig2, d_out);
  const Out p = run<NT, 5>(d_ll, N, sig2, d_out);
  printf("  NT %d stamped f (wave 0): elements %lld, DPP %lld, slot+barrier %lld, combine %lld, "
         "ratio %lld (total %lld)\n", NT, p.ph[1], p.ph[2] - p.ph[1], p.ph[3] - p.ph[2],
         p.ph[4] - p.ph[3], p.ph[5] - p.ph[4], p.ph[5]);
  const Out g = run<NT, 6>(d_ll, N, sig2, d_out);
  const Out h = run<NT, 7>(d_ll, N, sig2, d_out);
  printf("  NT %d: select-form logic %.0f cyc/iter vs branchy %.0f | pk objective: select-form brent "
         "%lld cyc vs branchy %lld (roots %s)\n", NT, (double)c.cycles / c.n,
         (double)h.cycles / h.n, e.cycles, g.cycles, e.x == g.x && e.n == g.n ? "identical" : "DIFFER");
  printf("  NT %d: brent %lld cyc / %d f (root %.9g) | f %.0f cyc | logic-only brent %.0f cyc/iter"
         " (%d f) | f_pk %.0f cyc | brent_pk %lld cyc / %d f (root %.9g, %s)\n",
         NT, a.cycles, a.n, a.x, b.cycles / 16.0, (double)c.cycles / c.n, c.n, d.cycles / 16.0,
         e.cycles, e.n, e.x, e.x == a.x ? "same" : "DIFFERS");
}

int main() {
  const int N = 4096;
  float* d_ll;
  Out* d_out;
  hipMalloc(&d_ll, N * sizeof(float));
  hipMalloc(&d_out, sizeof(Out));
  for (double sc : {3000.0, 300.0, 30.0}) {
    std::mt19937 g(7);
    std::normal_distribution<float> nd(-5000.f, (float)sc);
    std::vector<float> h(N);
    for (auto& v : h) v = nd(g);
    hipMemcpy(d_ll, h.data(), N * sizeof(float), hipMemcpyHostToDevice);
    printf("loglik spread %.0f nats\n", sc);
    sweep<512>(d_ll, N, sc * sc, d_out);
    sweep<256>(d_ll, N, sc * sc, d_out);
  }
  hipDeviceSynchronize();
  return 0;
}
