// Exhaustive check of correctly rounded square-root sequences built from v_rsq_f32 and fma
// (full-rate instructions, where sqrt_rn_core's neighbour tests cost two half-rate compares
// and two half-rate selects: DESIGN 4.7, 10), against RN(sqrt(x)) = (float)sqrt((double)x),
// over every float x >= 2^-96 (the unscaled range of sqrt_nn), +0, and every x in (0, 2^-96)
// through sqrt_nn's scaled form (core(x * 2^32) * 2^-16).  The rsq input is x + 2^-126:
// equal to x from 2^-96 up, finite at x = +0, whose products then use x itself (g0 = x * y0 =
// +0, so the sequence returns +0 with no select).
//   C1: Markstein: y0 = rsq, g0 = x y0, h0 = y0 / 2, r = 1/2 - g0 h0, g1 = g0 + g0 r,
//       h1 = h0 + h0 r, d = x - g1^2, g = g1 + d h1
//   C2: C1 without refining h (g = g1 + d h0)
//   C3: no refinement (d = x - g0^2, g = g0 + d h0)
// Also: for every x in (0, 2^-96), C3 unscaled (what sqrt_nn returns when IterArgs::taut_small
// lets it skip the scaled form) stays below 1.5 * 2^-48 and leaves the projection's
// ng = 1 + taut*g and fma(taut, g, 1) at exactly 1 for taut = +-2^20 (the largest |taut| the
// host calls small), as the correctly rounded root does.
// Build: hipcc -O3 --offload-arch=gfx950 tools/sqrt_fma_check.hip -o tools/_bin/sqrt_fma_check
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ unsigned long long bad[3][2];   // [candidate][unscaled range, scaled range]
__device__ unsigned long long bad_skip;     // tiny x whose unscaled C3 could change ng

template <int C>
__device__ __forceinline__ float core(float x) {
  const float y0 = __builtin_amdgcn_rsqf(x + 0x1p-126f);
  const float g0 = x * y0;
  const float h0 = 0.5f * y0;
  if (C == 3) {
    const float d = __builtin_fmaf(-g0, g0, x);
    return __builtin_fmaf(d, h0, g0);
  }
  const float r = __builtin_fmaf(-g0, h0, 0.5f);
  const float g1 = __builtin_fmaf(g0, r, g0);
  const float d = __builtin_fmaf(-g1, g1, x);
  if (C == 2) return __builtin_fmaf(d, h0, g1);
  const float h1 = __builtin_fmaf(h0, r, h0);
  return __builtin_fmaf(d, h1, g1);
}

template <int C>
__device__ __forceinline__ void one(float x, uint32_t rb, int range) {
  const float s = range == 0 ? core<C>(x) : core<C>(x * 0x1p32f) * 0x1p-16f;
  if (__float_as_uint(s) != rb) atomicAdd(&bad[C - 1][range], 1ull);
}

__global__ void check(uint32_t base) {
  const uint32_t bits = base + blockIdx.x * blockDim.x + threadIdx.x;
  if (bits >= 0x7F800000u) return;   // +0 .. the largest finite float
  const float x = __uint_as_float(bits);
  const uint32_t rb = __float_as_uint((float)__builtin_sqrt((double)x));
  const int range = (x >= 0x1p-96f || bits == 0) ? 0 : 1;
  one<1>(x, rb, range);
  one<2>(x, rb, range);
  one<3>(x, rb, range);
  if (range == 1) {
    const float g = core<3>(x);
    bool ok = g >= 0.0f && g < 0x1.8p-48f;
    for (float t : {0x1p20f, -0x1p20f}) {
      const float tg = t * g;
      ok = ok && 1.0f + tg == 1.0f && __builtin_fmaf(t, g, 1.0f) == 1.0f;
    }
    if (!ok) atomicAdd(&bad_skip, 1ull);
  }
}

int main() {
  const uint32_t per = 1u << 24;
  for (uint64_t b = 0; b < 0x7F800000ull; b += per) check<<<per / 256, 256>>>((uint32_t)b);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("HIP error\n");
    return 2;
  }
  unsigned long long c[3][2];
  if (hipMemcpyFromSymbol(c, HIP_SYMBOL(bad), sizeof(c)) != hipSuccess) return 2;
  unsigned long long skip = 0;
  if (hipMemcpyFromSymbol(&skip, HIP_SYMBOL(bad_skip), sizeof(skip)) != hipSuccess) return 2;
  for (int k = 0; k < 3; ++k)
    printf("C%d: wrong for %llu inputs in [2^-96, max] and +0, %llu in (0, 2^-96) scaled\n", k + 1,
           c[k][0], c[k][1]);
  printf("C3 unscaled in (0, 2^-96): %llu inputs could change ng at |taut| = 2^20\n", skip);
  return 0;
}
