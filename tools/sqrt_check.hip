// Exhaustive check of v_sqrt_f32 (__builtin_amdgcn_sqrtf) on gfx950 against the correctly
// rounded square root, over every positive finite float (2^31 - 2^23 inputs):
//   up   = v_sqrt(x) is one ulp BELOW RN(sqrt(x)) (needs the +1 ulp correction),
//   down = v_sqrt(x) is one ulp ABOVE RN(sqrt(x)) (needs the -1 ulp correction),
//   far  = anything else wrong.
// Counts are reported for x >= 2^-96 (where tvl1_kernels.hpp sqrt_rn_core runs unscaled) and
// below.  RN(sqrt(x)) is computed on the device as (float)sqrt((double)x), which is correctly
// rounded for every float x (sqrt of a 24-bit significand never lands on a float midpoint).
// It also checks the one-sided correction candidates against RN for the same range.
// Build: hipcc -O3 --offload-arch=gfx950 tools/sqrt_check.hip -o tools/_sqrt_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ unsigned long long cnt[2][4];   // [range: >= 2^-96, below][ok, up, down, far]
__device__ unsigned long long one_sided_bad[2];   // "up-only" fix wrong / "down-only" fix wrong

__global__ void check(uint32_t base) {
  const uint32_t bits = base + blockIdx.x * blockDim.x + threadIdx.x;
  if (bits >= 0x7F800000u || bits == 0) return;   // positive finite, nonzero
  const float x = __uint_as_float(bits);
  const float s = __builtin_amdgcn_sqrtf(x);
  const float rn = (float)__builtin_sqrt((double)x);
  const int range = x >= 0x1p-96f ? 0 : 1;
  const uint32_t sb = __float_as_uint(s), rb = __float_as_uint(rn);
  int k = sb == rb ? 0 : (sb + 1 == rb ? 1 : (sb == rb + 1 ? 2 : 3));
  atomicAdd(&cnt[range][k], 1ull);
  if (range == 0) {
    // up-only: s, or s + 1 ulp when x - (s + ulp) * s > 0
    const float sp = __uint_as_float(sb + 1u);
    const float up_only = __builtin_fmaf(-sp, s, x) > 0.0f ? sp : s;
    // down-only: s, or s - 1 ulp when x - (s - ulp) * s <= 0
    const float sm = __uint_as_float(sb - 1u);
    const float down_only = __builtin_fmaf(-sm, s, x) <= 0.0f ? sm : s;
    if (__float_as_uint(up_only) != rb) atomicAdd(&one_sided_bad[0], 1ull);
    if (__float_as_uint(down_only) != rb) atomicAdd(&one_sided_bad[1], 1ull);
  }
}

int main() {
  const uint32_t per = 1u << 24;
  for (uint64_t b = 0; b < 0x7F800000ull; b += per) check<<<per / 256, 256>>>((uint32_t)b);
  if (hipDeviceSynchronize() != hipSuccess) { printf("HIP error\n"); return 2; }
  unsigned long long c[2][4], o[2];
  hipMemcpyFromSymbol(c, HIP_SYMBOL(cnt), sizeof(c));
  hipMemcpyFromSymbol(o, HIP_SYMBOL(one_sided_bad), sizeof(o));
  const char *rn[2] = {"x >= 2^-96", "x <  2^-96"};
  for (int r = 0; r < 2; ++r)
    printf("%s: correctly rounded %llu, one ulp low %llu, one ulp high %llu, worse %llu\n", rn[r],
           c[r][0], c[r][1], c[r][2], c[r][3]);
  printf("x >= 2^-96: up-only correction wrong %llu, down-only correction wrong %llu\n", o[0], o[1]);
  return 0;
}
