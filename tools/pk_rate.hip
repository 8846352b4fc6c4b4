// Issue rate of packed f32 VALU ops (v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32) against
// their scalar forms on gfx950: every lane runs CH independent chains for ITER trips, the
// same lane-op count in both forms (a packed op counts two).  Reports lane-ops/s and the
// packed/scalar time ratio (1.0 = a packed op issues in the time of a scalar one).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/pk_rate.hip -o tools/pk_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int CH = 8, ITER = 4096;

template <int OP>   // 0 mul, 1 add, 2 fma
__global__ __launch_bounds__(256) void k_scalar(float *out, float a, float b) {
  float x[2 * CH];
#pragma unroll
  for (int i = 0; i < 2 * CH; ++i) x[i] = threadIdx.x * 1e-3f + i;
  for (int t = 0; t < ITER; ++t) {
#pragma unroll
    for (int i = 0; i < 2 * CH; ++i) {
      if (OP == 0) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
      if (OP == 1) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
      if (OP == 2) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 2 * CH; ++i) s += x[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
__global__ __launch_bounds__(256) void k_packed(float *out, float a, float b) {
  f2 x[CH];
  f2 av = {a, a}, bv = {b, b};
#pragma unroll
  for (int i = 0; i < CH; ++i) x[i] = f2{threadIdx.x * 1e-3f + 2 * i, threadIdx.x * 1e-3f + 2 * i + 1};
  for (int t = 0; t < ITER; ++t) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (OP == 0) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(av));
      if (OP == 1) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x[i]) : "v"(av));
      if (OP == 2) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(av), "v"(bv));
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < CH; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class K>
static float time_it(K k, int blocks, float *out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1.0000001f, 1e-7f);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1.0000001f, 1e-7f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  float *out;
  const int maxb = 256 * 8 * 4;
  if (hipMalloc(&out, sizeof(float) * 256 * maxb) != hipSuccess) return 1;
  const char *names[3] = {"mul", "add", "fma"};
  // blocks of 4 waves: 256 blocks = 1 wave/SIMD, x2, x4, x8 waves/SIMD
  for (int wps : {1, 2, 4, 8}) {
    const int blocks = 256 * wps;
    const double lane_ops = (double)blocks * 256 * ITER * 2 * CH;
    for (int op = 0; op < 3; ++op) {
      float ts = op == 0 ? time_it(k_scalar<0>, blocks, out)
                         : op == 1 ? time_it(k_scalar<1>, blocks, out) : time_it(k_scalar<2>, blocks, out);
      float tp = op == 0 ? time_it(k_packed<0>, blocks, out)
                         : op == 1 ? time_it(k_packed<1>, blocks, out) : time_it(k_packed<2>, blocks, out);
      printf("waves/SIMD %d %s: scalar %.3f ms (%.1f T lane-op/s)  packed %.3f ms (%.1f T lane-op/s)  packed/scalar time %.3f\n",
             wps, names[op], ts, lane_ops / ts * 1e-9, tp, lane_ops / tp * 1e-9, tp / ts);
    }
  }
  (void)hipFree(out);
  return 0;
}
