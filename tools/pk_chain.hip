// Dependent-chain form of tools/pk_rate.hip: each lane updates 2 px (the rolling passes'
// PX = 2) through a chain of IEEE mul/add (no contraction) with one v_sqrt_f32 and one
// v_rcp_f32 per px per step, scalar (two chains) or with the mul/adds packed (one v_pk_*
// per pair of px; sqrt / rcp stay scalar on each half).  Lane-ops/s and time ratio per
// occupancy (waves per SIMD, launch of 4-wave blocks).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/pk_chain.hip -o tools/pk_chain
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 2048;

// chain step per px: t = a*b; a = t + c; s = sqrt(a); a = a*d; a = a + s; r = rcp(a);
//                    a = a*e; a = a + r; a = a*f; a = a + g   (8 mul/add, 1 sqrt, 1 rcp)
__global__ __launch_bounds__(256) void k_scalar(float *out, float b, float c, float d, float e,
                                                float f, float g) {
  float a0 = 1.0f + threadIdx.x * 1e-6f, a1 = 1.5f + threadIdx.x * 1e-6f;
  for (int t = 0; t < ITER; ++t) {
    float s0, s1, r0, r1;
    asm volatile(
        "v_mul_f32 %0, %0, %6\n v_mul_f32 %1, %1, %6\n"
        "v_add_f32 %0, %0, %7\n v_add_f32 %1, %1, %7\n"
        "v_sqrt_f32 %2, %0\n v_sqrt_f32 %3, %1\n"
        "v_mul_f32 %0, %0, %8\n v_mul_f32 %1, %1, %8\n"
        "v_add_f32 %0, %0, %2\n v_add_f32 %1, %1, %3\n"
        "v_rcp_f32 %4, %0\n v_rcp_f32 %5, %1\n"
        "v_mul_f32 %0, %0, %9\n v_mul_f32 %1, %1, %9\n"
        "v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %5\n"
        "v_mul_f32 %0, %0, %10\n v_mul_f32 %1, %1, %10\n"
        "v_add_f32 %0, %0, %11\n v_add_f32 %1, %1, %11\n"
        : "+v"(a0), "+v"(a1), "=&v"(s0), "=&v"(s1), "=&v"(r0), "=&v"(r1)
        : "v"(b), "v"(c), "v"(d), "v"(e), "v"(f), "v"(g));
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1;
}

__global__ __launch_bounds__(256) void k_packed(float *out, float b, float c, float d, float e,
                                                float f, float g) {
  f2 a = {1.0f + threadIdx.x * 1e-6f, 1.5f + threadIdx.x * 1e-6f};
  const f2 B = {b, b}, C = {c, c}, D = {d, d}, E = {e, e}, F = {f, f}, G = {g, g};
  for (int t = 0; t < ITER; ++t) {
    f2 s, r;
    asm volatile("v_pk_mul_f32 %0, %0, %1\n v_pk_add_f32 %0, %0, %2" : "+v"(a) : "v"(B), "v"(C));
    s.x = __builtin_amdgcn_sqrtf(a.x);
    s.y = __builtin_amdgcn_sqrtf(a.y);
    asm volatile("v_pk_mul_f32 %0, %0, %2\n v_pk_add_f32 %0, %0, %1" : "+v"(a) : "v"(s), "v"(D));
    r.x = __builtin_amdgcn_rcpf(a.x);
    r.y = __builtin_amdgcn_rcpf(a.y);
    asm volatile(
        "v_pk_mul_f32 %0, %0, %2\n v_pk_add_f32 %0, %0, %1\n"
        "v_pk_mul_f32 %0, %0, %3\n v_pk_add_f32 %0, %0, %4"
        : "+v"(a)
        : "v"(r), "v"(E), "v"(F), "v"(G));
  }
  out[blockIdx.x * 256 + threadIdx.x] = a.x + a.y;
}

template <class K>
static float time_it(K k, int blocks, float *out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.5f, 1.001f, 0.7f, 1.2f, 0.1f);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.5f, 1.001f, 0.7f, 1.2f, 0.1f);
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
  if (hipMalloc(&out, sizeof(float) * 256 * 256 * 8) != hipSuccess) return 1;
  for (int wps : {1, 2, 3, 4, 8}) {
    const int blocks = 256 * wps;
    const double px_steps = (double)blocks * 256 * ITER * 2;
    const float ts = time_it(k_scalar, blocks, out), tp = time_it(k_packed, blocks, out);
    printf("waves/SIMD %d: scalar %.3f ms (%.1f G px-steps/s)  packed %.3f ms (%.1f G px-steps/s)  packed/scalar time %.3f\n",
           wps, ts, px_steps / ts * 1e-6, tp, px_steps / tp * 1e-6, tp / ts);
  }
  (void)hipFree(out);
  return 0;
}
