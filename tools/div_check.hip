// Checks the short correctly-rounded division a / d = div_fixup(q0 + r0*y) with
// y = one Newton step from v_rcp_f32 (Markstein: y == RN(1/d) makes q1 == RN(a/d) when
// nothing underflows) against IEEE a / d on gfx950:
//   A. y == RN(1/d) for every significand of the listed binades (exhaustive);
//   B. random quotients with d >= 1 (the projection's ng) and |a| <= d;
//   C. random quotients with d in [FLT_EPSILON, 2^24) (the TH step's grad) and any a;
//   D. edge numerators: +-0, +-d, +-2^-k d, all-ones-significand denominators.
// Build: hipcc -O3 -ffp-contract=off --offload-arch=gfx950 tools/div_check.hip -o tools/_div_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float recip(float d) {
  const float r = __builtin_amdgcn_rcpf(d);
  const float e = __builtin_fmaf(-d, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}
#ifndef QV
#define QV 0
#endif
__device__ __forceinline__ float qdiv(float a, float d, float y) {
  if (QV == 1) {   // 5 ops: numerator scaled by div_scale, one Markstein step inside div_fmas
    bool sc;
    const float n = __builtin_amdgcn_div_scalef(a, d, true, &sc);
    const float q0 = n * y;
    const float r0 = __builtin_fmaf(-d, q0, n);
    const float q = __builtin_amdgcn_div_fmasf(r0, y, q0, sc);
    return __builtin_amdgcn_div_fixupf(q, d, a);
  }
  const float q0 = a * y;
  const float r0 = __builtin_fmaf(-d, q0, a);
  const float q1 = __builtin_fmaf(r0, y, q0);
  if (QV == 2) return q1;   // tvl1_kernels.hpp div_short: no fixup (zero / tiny numerators are
                            // guarded to the full sequence by the callers)
  return __builtin_amdgcn_div_fixupf(q1, d, a);
}
__device__ unsigned long long bad[5];
__device__ unsigned maxeb_bad, minqe_bad = 1000;   // E: largest biased exponent of a, smallest of
                                                   // the quotient, among mismatches
__device__ unsigned long long ex[5][3];   // one example per test: d bits, a bits, got bits

__device__ void report(int t, float d, float a, float got) {
  if (atomicAdd(&bad[t], 1ull) == 0) {
    ex[t][0] = __float_as_uint(d);
    ex[t][1] = __float_as_uint(a);
    ex[t][2] = __float_as_uint(got);
  }
}

__global__ void testA(int e0) {   // d = 2^e0 * (1 + m 2^-23), all m
  const unsigned m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= (1u << 23)) return;
  const float d = __uint_as_float(((unsigned)(e0 + 127) << 23) | m);
  const float y = recip(d);
  const float ref = 1.0f / d;
  if (__float_as_uint(y) != __float_as_uint(ref)) report(0, d, 1.0f, y);
}

__global__ void testB(uint64_t seed, int maxexp) {
  const uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int it = 0; it < 64; ++it) {
    const uint64_t h = mix(seed ^ (id * 64 + it));
    const int ed = (int)((h >> 40) % (unsigned)(maxexp + 1));
    const float d = __uint_as_float(((unsigned)(ed + 127) << 23) | (unsigned)(h & 0x7FFFFF));
    const int ea = (int)((h >> 48) % 96);   // |a| from d down to d * 2^-95
    const float frac = __uint_as_float((127u << 23) | (unsigned)((h >> 23) & 0x7FFFFF));   // [1, 2)
    float a = d * 0.5f * frac * __uint_as_float((unsigned)(127 - ea) << 23);
    if (h >> 63) a = -a;
    if (!(a == a) || fabsf(a) > d) continue;
    const float got = qdiv(a, d, recip(d));
    const float ref = a / d;
    if (__float_as_uint(got) != __float_as_uint(ref)) report(1, d, a, got);
  }
}

__global__ void testC(uint64_t seed) {
  const uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int it = 0; it < 64; ++it) {
    const uint64_t h = mix(seed ^ (id * 64 + it) ^ 0x5555);
    const int ed = -23 + (int)((h >> 40) % 47);   // [2^-23, 2^24)
    float d = __uint_as_float(((unsigned)(ed + 127) << 23) | (unsigned)(h & 0x7FFFFF));
    if (d < 1.1920928955078125e-07f) continue;
    const int ea = -80 + (int)((h >> 48) % 110);   // a in [2^-80, 2^30)
    float a = __uint_as_float(((unsigned)(ea + 127) << 23) | (unsigned)((h >> 20) & 0x7FFFFF));
    if (h >> 63) a = -a;
    const float got = qdiv(a, d, recip(d));
    const float ref = a / d;
    if (__float_as_uint(got) != __float_as_uint(ref)) report(2, d, a, got);
  }
}

__global__ void testD() {
  const unsigned m = blockIdx.x * blockDim.x + threadIdx.x;   // significand of d
  if (m >= (1u << 23)) return;
  const float ds[3] = {__uint_as_float((127u << 23) | m), __uint_as_float((127u << 23) | 0x7FFFFFu),
                       __uint_as_float((140u << 23) | m)};
  for (int i = 0; i < 3; ++i) {
    const float d = ds[i], y = recip(d);
    const float as[8] = {0.0f, -0.0f, d, -d, d * 0.5f, -d * 0x1p-20f,
                         __uint_as_float(0x3F800000u | (m ^ 0x2AAAAAu)), -__uint_as_float(0x3F000000u | m)};
    for (int k = 0; k < 8; ++k) {
      const float a = as[k];
      if (fabsf(a) > d) continue;
      if (QV == 2 && a == 0.0f) continue;   // zeros take the full sequence (guarded)
      const float got = qdiv(a, d, y);
      const float ref = a / d;
      if (__float_as_uint(got) != __float_as_uint(ref)) report(3, d, a, got);
    }
  }
}

// E. tiny numerators (denormal a and/or subnormal quotients): a in [2^-149, 2^-60),
// d in [2^-23, 2^40)
__global__ void testE(uint64_t seed) {
  const uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int it = 0; it < 64; ++it) {
    const uint64_t h = mix(seed ^ (id * 64 + it) ^ 0x777);
    const int ed = -23 + (int)((h >> 40) % 63);
    const float d = __uint_as_float(((unsigned)(ed + 127) << 23) | (unsigned)(h & 0x7FFFFF));
    const unsigned eb = (unsigned)((h >> 48) % 68);   // biased exponent 0 (denormal) .. 67
    float a = __uint_as_float((eb << 23) | (unsigned)((h >> 20) & 0x7FFFFF));
    if (h >> 63) a = -a;
    const float got = qdiv(a, d, recip(d));
    const float ref = a / d;
    if (__float_as_uint(got) != __float_as_uint(ref)) {
      report(4, d, a, got);
      atomicMax(&maxeb_bad, eb);
      atomicMin(&minqe_bad, (__float_as_uint(ref) >> 23) & 0xFF);
    }
  }
}

int main() {
  // every binade the kernels divide by: TH grad in [FLT_EPSILON, 2^15], projection ng >= 1
  for (int e = -23; e <= 40; ++e) testA<<<(1 << 23) / 256, 256>>>(e);
  const int exps[] = {50, 99, 100, 120, 125};
  for (int e : exps) testA<<<(1 << 23) / 256, 256>>>(e);
  for (int s = 0; s < 16; ++s) testB<<<16384, 256>>>(0x1234567ull + s * 7919ull, 100);
  for (int s = 0; s < 16; ++s) testC<<<16384, 256>>>(0xABCDEFull + s * 104729ull);
  testD<<<(1 << 23) / 256, 256>>>();
  for (int s = 0; s < 16; ++s) testE<<<16384, 256>>>(0x31415ull + s * 3571ull);
  if (hipDeviceSynchronize() != hipSuccess) { printf("HIP error\n"); return 2; }
  unsigned long long b[5], e[5][3];
  hipMemcpyFromSymbol(b, HIP_SYMBOL(bad), sizeof(b));
  hipMemcpyFromSymbol(e, HIP_SYMBOL(ex), sizeof(e));
  const char *names[5] = {"A reciprocal (69 binades, exhaustive)", "B ng quotients (2^32 random)",
                          "C TH quotients (2^32 random)", "D edge numerators (2^23 x 3 x 8)",
                          "E tiny numerators (2^32 random)"};
  int rc = 0;
  for (int t = 0; t < 5; ++t) {
    printf("%-40s mismatches %llu", names[t], b[t]);
    if (b[t]) {
      printf("  e.g. d=%08llx a=%08llx got=%08llx", e[t][0], e[t][1], e[t][2]);
      rc = 1;
    }
    printf("\n");
  }
  unsigned mb = 0, mq = 0;
  hipMemcpyFromSymbol(&mb, HIP_SYMBOL(maxeb_bad), sizeof(mb));
  hipMemcpyFromSymbol(&mq, HIP_SYMBOL(minqe_bad), sizeof(mq));
  printf("E: largest biased exponent of a among mismatches %u; quotient biased exponents >= %u\n", mb, mq);
  unsigned long long nq = 0;
  return rc;
}
