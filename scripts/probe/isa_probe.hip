// Issue-cost probe: v_fma_f32 vs v_pk_fma_f32 vs v_exp_f32 vs v_pk_mul_f32,
// 8 independent chains per wave, 4 waves per SIMD (16 per CU).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ __launch_bounds__(256) void probe(float* out, int iters) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
        a6 = a0 + 6, a7 = a0 + 7;
  const float b = 0.999f, c = 1e-4f;
  for (int i = 0; i < iters; ++i) {
#define FMA1(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c))
#define EXP1(x) asm volatile("v_exp_f32 %0, %0" : "+v"(x))
#define PK1(X, Y)                                                                      \
  {                                                                                    \
    typedef float f2 __attribute__((ext_vector_type(2)));                             \
    f2 v = {X, Y};                                                                     \
    f2 bb = {b, b}, cc = {c, c};                                                       \
    asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(v) : "v"(bb), "v"(cc));          \
    X = v.x;                                                                           \
    Y = v.y;                                                                           \
  }
    if constexpr (OP == 0) {  // 8 scalar fma
      FMA1(a0); FMA1(a1); FMA1(a2); FMA1(a3); FMA1(a4); FMA1(a5); FMA1(a6); FMA1(a7);
    } else if constexpr (OP == 1) {  // 4 packed fma = 8 lanes-ops
      PK1(a0, a1); PK1(a2, a3); PK1(a4, a5); PK1(a6, a7);
    } else if constexpr (OP == 2) {  // 8 exp
      EXP1(a0); EXP1(a1); EXP1(a2); EXP1(a3); EXP1(a4); EXP1(a5); EXP1(a6); EXP1(a7);
    } else if constexpr (OP == 3) {  // 4 exp + 4 fma interleaved
      EXP1(a0); FMA1(a1); EXP1(a2); FMA1(a3); EXP1(a4); FMA1(a5); EXP1(a6); FMA1(a7);
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int blocks = cus * 4;  // 16 waves per CU
  float* out;
  hipMalloc(&out, blocks * 256 * sizeof(float));
  const int iters = 20000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"8x v_fma_f32", "4x v_pk_fma_f32", "8x v_exp_f32", "4 exp + 4 fma"};
  for (int rep = 0; rep < 2; ++rep)
    for (int op = 0; op < 4; ++op) {
      hipEventRecord(e0);
      switch (op) {
        case 0: probe<0><<<blocks, 256>>>(out, iters); break;
        case 1: probe<1><<<blocks, 256>>>(out, iters); break;
        case 2: probe<2><<<blocks, 256>>>(out, iters); break;
        case 3: probe<3><<<blocks, 256>>>(out, iters); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      // per SIMD: 4 waves x iters x 8 instructions (op 1: 4)
      const double ninst = 4.0 * iters * (op == 1 ? 4 : 8);
      if (rep) printf("%-18s %.3f ms  %.2f ns per wave-instruction per SIMD\n", names[op], ms,
                      ms * 1e6 / ninst);
    }
  return 0;
}
