// Dependent-chain latency of v_add_f32 / v_mul_f32 against v_pk_add_f32 / v_pk_mul_f32 on
// gfx950: one wave per SIMD, each lane runs ONE chain of N dependent ops (or 2 / 4 chains
// interleaved), cycles per op from s_memtime around the loop.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/pk_lat.hip -o tools/_bin/pk_lat
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int N = 4096;

template <int OP, int CH>   // OP 0 add, 1 mul, 2 pk_add, 3 pk_mul
__global__ __launch_bounds__(64) void k_lat(float *out, unsigned long long *cyc, float a) {
  float x[CH];
  f2 y[CH];
  const f2 av = {a, a};
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    x[c] = threadIdx.x * 1e-3f + c;
    y[c] = f2{x[c], x[c] + 0.5f};
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < N; ++t) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if (OP == 0) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[c]) : "v"(a));
      if (OP == 1) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[c]) : "v"(a));
      if (OP == 2) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(y[c]) : "v"(av));
      if (OP == 3) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(y[c]) : "v"(av));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += x[c] + y[c].x + y[c].y;
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int OP, int CH>
static double run(float *out, unsigned long long *cyc) {
  hipLaunchKernelGGL((k_lat<OP, CH>), dim3(1), dim3(64), 0, 0, out, cyc, 1.0000001f);
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL((k_lat<OP, CH>), dim3(1), dim3(64), 0, 0, out, cyc, 1.0000001f);
  unsigned long long c;
  (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  return (double)c / (N * CH);   // s_memtime cycles per op
}

int main() {
  float *out;
  unsigned long long *cyc;
  if (hipMalloc(&out, 4096) != hipSuccess || hipMalloc(&cyc, 8) != hipSuccess) return 1;
  printf("s_memtime cycles per op, one wave (chains interleaved per lane)\n");
  printf("chains 1: add %.2f mul %.2f pk_add %.2f pk_mul %.2f\n", run<0, 1>(out, cyc),
         run<1, 1>(out, cyc), run<2, 1>(out, cyc), run<3, 1>(out, cyc));
  printf("chains 2: add %.2f mul %.2f pk_add %.2f pk_mul %.2f\n", run<0, 2>(out, cyc),
         run<1, 2>(out, cyc), run<2, 2>(out, cyc), run<3, 2>(out, cyc));
  printf("chains 4: add %.2f mul %.2f pk_add %.2f pk_mul %.2f\n", run<0, 4>(out, cyc),
         run<1, 4>(out, cyc), run<2, 4>(out, cyc), run<3, 4>(out, cyc));
  printf("chains 8: add %.2f mul %.2f pk_add %.2f pk_mul %.2f\n", run<0, 8>(out, cyc),
         run<1, 8>(out, cyc), run<2, 8>(out, cyc), run<3, 8>(out, cyc));
  return 0;
}
