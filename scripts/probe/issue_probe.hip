// Multi-wave VALU issue probe (gfx950): SIMD cycles per wave-instruction for
// the instruction classes of the MH sweep, at W = 1, 2, 4, 7, 8 waves per SIMD.
// Each wave runs `iters` loop trips of 16 independent chains of one class (or
// an interleaved mix), stamps s_memtime (shader cycles) before and after and
// records its SIMD (HW_ID: SE, SH, CU, SIMD; XCC_ID).  Per SIMD: cycles per
// wave-instruction = (last wave's end - first wave's start) / (waves on that
// SIMD x instructions per wave); the table prints the median over SIMDs, and
// the waves per SIMD actually seen (min..max), which must equal W.  The grid
// is 256 CUs x W workgroups of 256 threads.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probe/issue_probe scripts/probe/issue_probe.hip
//   ./scripts/probe/issue_probe > profiles/r06/issue_probe.txt
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

#define FMA(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c))
#define MUL(x) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(b))
#define EXP(x) asm volatile("v_exp_f32 %0, %0" : "+v"(x))
#define LOG(x) asm volatile("v_log_f32 %0, %0" : "+v"(x))
#define RCP(x) asm volatile("v_rcp_f32 %0, %0" : "+v"(x))
#define PK(x) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(bb), "v"(cc))
#define PKM(x) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x) : "v"(bb))
#define DPP(x) asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 bound_ctrl:0" : "+v"(x))
#define RDL(x) asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(sx) : "v"(x))

// classes: instructions per loop trip (per wave) and their issue order
enum {
  kFma, kMul, kExp, kLog, kRcp, kPk, kPkMul, kFma3Exp1, kFma6Exp1, kPk1Fma1, kPkExp, kDpp,
  kReadlane, kNum
};
static const char* kNames[kNum] = {
    "v_fma_f32", "v_mul_f32", "v_exp_f32", "v_log_f32", "v_rcp_f32", "v_pk_fma_f32",
    "v_pk_mul_f32", "3 fma : 1 exp", "6 fma : 1 exp (C2 mix)", "1 pk_fma : 1 fma",
    "3 pk_fma : 1 exp", "v_mov_b32_dpp row_shr", "v_readlane_b32"};
static const int kInsts[kNum] = {16, 16, 16, 16, 16, 8, 8, 16, 14, 16, 16, 16, 16};

template <int OP>
__global__ __launch_bounds__(256) void probe(long long* cyc, float* out, int iters) {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // XCC_ID
  float a[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * 1e-3f + i;
  f2 p[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) p[i] = f2{a[2 * i], a[2 * i + 1]};
  const float b = 0.999f, c = 1e-4f;
  const f2 bb = {b, b}, cc = {c, c};
  int sx = 0;
  (void)sx;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if constexpr (OP == kFma) {
#pragma unroll
      for (int i = 0; i < 16; ++i) FMA(a[i]);
    } else if constexpr (OP == kMul) {
#pragma unroll
      for (int i = 0; i < 16; ++i) MUL(a[i]);
    } else if constexpr (OP == kExp) {
#pragma unroll
      for (int i = 0; i < 16; ++i) EXP(a[i]);
    } else if constexpr (OP == kLog) {
#pragma unroll
      for (int i = 0; i < 16; ++i) LOG(a[i]);
    } else if constexpr (OP == kRcp) {
#pragma unroll
      for (int i = 0; i < 16; ++i) RCP(a[i]);
    } else if constexpr (OP == kPk) {
#pragma unroll
      for (int i = 0; i < 8; ++i) PK(p[i]);
    } else if constexpr (OP == kPkMul) {
#pragma unroll
      for (int i = 0; i < 8; ++i) PKM(p[i]);
    } else if constexpr (OP == kFma3Exp1) {
#pragma unroll
      for (int i = 0; i < 16; i += 4) {
        EXP(a[i]);
        FMA(a[i + 1]);
        FMA(a[i + 2]);
        FMA(a[i + 3]);
      }
    } else if constexpr (OP == kFma6Exp1) {
#pragma unroll
      for (int i = 0; i < 14; i += 7) {
        EXP(a[i]);
        FMA(a[i + 1]);
        FMA(a[i + 2]);
        FMA(a[i + 3]);
        FMA(a[i + 4]);
        FMA(a[i + 5]);
        FMA(a[i + 6]);
      }
    } else if constexpr (OP == kPk1Fma1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        PK(p[i]);
        FMA(a[i]);
      }
    } else if constexpr (OP == kPkExp) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        EXP(a[i]);
        PK(p[2 * i]);
        PK(p[2 * i + 1]);
        PK(p[(2 * i + 4) & 7]);
      }
    } else if constexpr (OP == kDpp) {
#pragma unroll
      for (int i = 0; i < 16; ++i) DPP(a[i]);
    } else if constexpr (OP == kReadlane) {
#pragma unroll
      for (int i = 0; i < 16; ++i) RDL(a[i]);
    }
  }
  const long long t1 = clock64();
  float s = sx;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += a[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) s += p[i].x + p[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) {
    long long* r = cyc + 3 * (blockIdx.x * 4 + (threadIdx.x >> 6));
    r[0] = t0;
    r[1] = t1;
    // SIMD key: XCC, SE (14:13), SH (12), CU (11:8), SIMD (5:4)
    r[2] = (long long)((xcc & 15u) << 16 | ((hw >> 8) & 0x7fu) << 2 | ((hw >> 4) & 3u));
  }
}

typedef void (*Kern)(long long*, float*, int);
template <int... I>
static void table(Kern* k, std::integer_sequence<int, I...>) {
  ((k[I] = probe<I>), ...);
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  Kern k[kNum];
  table(k, std::make_integer_sequence<int, kNum>{});
  const int iters = 4000;
  const int waves[] = {1, 2, 4, 7, 8};
  long long* cyc;
  float* out;
  (void)hipMalloc(&cyc, (size_t)cus * 8 * 4 * 3 * sizeof(long long));
  (void)hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(float));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  printf("SIMD cycles per wave-instruction: median over SIMDs of (last end - first start) / "
         "(waves x instructions per wave), s_memtime; [min waves per SIMD seen, + if uneven]; "
         "%d CUs, %d loop trips\n", cus, iters);
  printf("%-26s", "class \\ waves per SIMD");
  for (int w : waves) printf(" %9d", w);
  printf("   ticks/ns (W=4)\n");
  // warm the clock
  for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k[0], dim3(cus * 4), dim3(256), 0, 0, cyc, out, iters);
  (void)hipDeviceSynchronize();
  for (int op = 0; op < kNum; ++op) {
    printf("%-26s", kNames[op]);
    double ghz = 0;
    for (int w : waves) {
      const int blocks = cus * w;
      std::vector<long long> h((size_t)blocks * 4 * 3);
      float ms = 0;
      for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k[op], dim3(blocks), dim3(256), 0, 0, cyc, out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
      }
      (void)hipMemcpy(h.data(), cyc, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
      struct Span { long long lo = 0, hi = 0; int n = 0; };
      std::map<long long, Span> simd;
      long long span_max = 0;
      for (size_t i = 0; i < (size_t)blocks * 4; ++i) {
        Span& sp = simd[h[3 * i + 2]];
        if (sp.n == 0 || h[3 * i] < sp.lo) sp.lo = h[3 * i];
        if (sp.n == 0 || h[3 * i + 1] > sp.hi) sp.hi = h[3 * i + 1];
        ++sp.n;
      }
      std::vector<double> per;
      int wmin = 1 << 30, wmax = 0;
      for (auto& kv : simd) {
        per.push_back((double)(kv.second.hi - kv.second.lo) / ((double)kv.second.n * iters * kInsts[op]));
        wmin = std::min(wmin, kv.second.n);
        wmax = std::max(wmax, kv.second.n);
        span_max = std::max(span_max, kv.second.hi - kv.second.lo);
      }
      std::sort(per.begin(), per.end());
      printf(" %5.2f[%d%s]", per[per.size() / 2], wmin, wmin == wmax ? "" : "+");
      if (w == 4) ghz = (double)span_max / (ms * 1e6);
    }
    printf("   %.2f\n", ghz);
  }
  return 0;
}
