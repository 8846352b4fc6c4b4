// Issue cost of the vector-instruction classes the TV-L1 kernels use, measured on gfx950:
// cycles per wave-instruction at 1, 2, 4 and 8 wavefronts per SIMD.  Every lane runs 8
// independent chains of one instruction (inline asm, so the compiler neither fuses nor
// reorders them) for ITER trips; each wavefront stamps s_memtime (shader cycles) and
// s_memrealtime (100 MHz) around its loop, so the clock of the run is printed too.
// "per wave" = cycles / instructions of one wave (its own issue cadence); "per SIMD" = the
// launch's event time in cycles / the wave-instructions one SIMD issued (the SIMD's
// throughput cost, launch overhead included, so an upper bound at short launches).  These are
// the prices tools/issue_model.py charges each instruction class.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/issue_rate.hip -o tools/_bin/issue_rate
//   tools/_bin/issue_rate
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int ITER = 4096, CH = 8;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

// OP: 0 v_add_f32, 1 v_mul_f32, 2 v_fma_f32, 3 v_rcp_f32, 4 v_sqrt_f32, 5 v_rsq_f32,
// 6 v_add_f64, 7 v_fma_f64, 8 v_cvt_f64_f32, 9 v_mov_b32_dpp wave_shr:1, 10 v_cndmask_b32,
// 11 v_add_u32, 12 4 x v_add_f32 + 1 v_rcp_f32 (counted as 5), 13 v_add_f32_dpp wave_shr:1,
// 14 ds_read_b32 x 8 then lgkmcnt(0) (counted as 8; consecutive dwords across lanes: no bank
// conflict), 15 v_mul_f64, 16 v_cmp_gt_f32 (to an SGPR pair), 17 v_mov_b32, 18 v_pk_add_f32,
// 19 v_readfirstlane_b32, 20 s_add_u32, 21 ds_read_b32 dependent chain (the address is the
// value read: latency), 22 ds_write_b32 x 8 then lgkmcnt(0) (counted as 8), 23 v_floor_f32,
// 24 v_cvt_i32_f32, 25 v_med3_f32, 26 s_barrier alone (4-wave block), 27 v_fma_f32 on one chain
// per lane (dependent: latency), 28 v_cndmask_b32_e32 (vcc), 29 v_sub_f32, 30 v_max_f32,
// 31 v_cmp_gt_f32_e32 (vcc), 32 v_and_b32, 33 v_lshl_add_u32, 34 v_mad_u32_u24,
// 35 v_cvt_f32_i32, 36 v_mul_f32_e64 with a neg modifier, 37 v_mov_b64, 38 v_fmac_f32,
// 39 v_min_f32_e64 with abs, 40 v_ldexp_f32, 41 v_lshlrev_b32
template <int OP>
__global__ __launch_bounds__(256) void k_rate(float *out, unsigned long long *cyc, float a, float b) {
  __shared__ float lds[256 * CH + 64];
  float x[CH];
  double d[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    x[i] = 1.0f + threadIdx.x * 1e-3f + i;
    d[i] = x[i];
    lds[i * 256 + threadIdx.x] = OP == 21 ? __int_as_float(4 * (int)((threadIdx.x + 1) & 255)) : x[i];
  }
  __syncthreads();
  const unsigned long long mask = __builtin_amdgcn_read_exec();
  unsigned la = 4u * threadIdx.x;   // plane i at 1 KiB * i: lanes on consecutive dwords
  unsigned sacc = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < ITER; ++t) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if constexpr (OP == 0) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
      if constexpr (OP == 1) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
      if constexpr (OP == 2) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
      if constexpr (OP == 3) asm volatile("v_rcp_f32 %0, %0" : "+v"(x[i]));
      if constexpr (OP == 4) asm volatile("v_sqrt_f32 %0, %0" : "+v"(x[i]));
      if constexpr (OP == 5) asm volatile("v_rsq_f32 %0, %0" : "+v"(x[i]));
      if constexpr (OP == 6) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"((double)a));
      if constexpr (OP == 7)
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[i]) : "v"((double)a), "v"((double)b));
      if constexpr (OP == 8) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d[i]) : "v"(x[i]));
      if constexpr (OP == 9)
        asm volatile("v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
                     : "+v"(x[i]));
      if constexpr (OP == 10)
        asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "s"(mask));
      if constexpr (OP == 11) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
      if constexpr (OP == 12) {
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[(i + 1) % CH]) : "v"(a));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[(i + 2) % CH]) : "v"(a));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[(i + 3) % CH]) : "v"(a));
        asm volatile("v_rcp_f32 %0, %0" : "+v"(x[(i + 4) % CH]));
      }
      if constexpr (OP == 13)
        asm volatile("v_add_f32_dpp %0, %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
                     : "+v"(x[i]) : "v"(a));
      if constexpr (OP == 15) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"((double)a));
      if constexpr (OP == 16) {
        unsigned long long m;
        asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x[i]), "v"(a));
        asm volatile("" ::"s"(m));
      }
      if constexpr (OP == 17) asm volatile("v_mov_b32 %0, %1" : "=v"(x[i]) : "v"(x[(i + 1) % CH]));
      if constexpr (OP == 18) {
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 v = {x[i], x[(i + 1) % CH]};
        asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(v) : "v"(f2{a, b}));
        x[i] = v.x;
      }
      if constexpr (OP == 19) {
        unsigned s_;
        asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(s_) : "v"(x[i]));
        asm volatile("" ::"s"(s_));
      }
      if constexpr (OP == 20) asm volatile("s_add_u32 %0, %0, 3" : "+s"(sacc));
      if constexpr (OP == 23) asm volatile("v_floor_f32 %0, %0" : "+v"(x[i]));
      if constexpr (OP == 24) {
        int q;
        asm volatile("v_cvt_i32_f32 %0, %1" : "=v"(q) : "v"(x[i]));
        asm volatile("" ::"v"(q));
      }
      if constexpr (OP == 25) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
      if constexpr (OP == 26) {
        if (i == 0) asm volatile("s_barrier" ::: "memory");
      }
      if constexpr (OP == 28)
        asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(a) : "vcc");
      if constexpr (OP == 29) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
      if constexpr (OP == 30) asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
      if constexpr (OP == 31) asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1" ::"v"(x[i]), "v"(a) : "vcc");
      if constexpr (OP == 32) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
      if constexpr (OP == 33) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(x[i]) : "v"(a));
      if constexpr (OP == 34) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
      if constexpr (OP == 35) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(x[i]));
      if constexpr (OP == 36) asm volatile("v_mul_f32_e64 %0, %0, -%1" : "+v"(x[i]) : "v"(a));
      if constexpr (OP == 37) asm volatile("v_mov_b64 %0, %1" : "=v"(d[i]) : "v"(d[(i + 1) % CH]));
      if constexpr (OP == 38) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
      if constexpr (OP == 39) asm volatile("v_min_f32_e64 %0, |%0|, %1" : "+v"(x[i]) : "v"(a));
      if constexpr (OP == 40) asm volatile("v_ldexp_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
      if constexpr (OP == 41) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(x[i]));
      if constexpr (OP == 27) {
        if (i == 0)
          for (int k = 0; k < CH; ++k) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[0]) : "v"(a), "v"(b));
      }
    }
    if constexpr (OP == 21) {   // one dependent chain: 8 reads, each address the previous value
#pragma unroll
      for (int k = 0; k < CH; ++k)
        asm volatile("ds_read_b32 %0, %0\n s_waitcnt lgkmcnt(0)" : "+v"(la));
    }
    if constexpr (OP == 22) {
      asm volatile(
          "ds_write_b32 %0, %1\n ds_write_b32 %0, %1 offset:1024\n ds_write_b32 %0, %1 offset:2048\n"
          "ds_write_b32 %0, %1 offset:3072\n ds_write_b32 %0, %1 offset:4096\n"
          "ds_write_b32 %0, %1 offset:5120\n ds_write_b32 %0, %1 offset:6144\n"
          "ds_write_b32 %0, %1 offset:7168\n s_waitcnt lgkmcnt(0)" ::"v"(la), "v"(x[0]) : "memory");
    }
    if constexpr (OP == 14) {
      asm volatile(
          "ds_read_b32 %0, %8\n ds_read_b32 %1, %8 offset:1024\n ds_read_b32 %2, %8 offset:2048\n"
          "ds_read_b32 %3, %8 offset:3072\n ds_read_b32 %4, %8 offset:4096\n"
          "ds_read_b32 %5, %8 offset:5120\n ds_read_b32 %6, %8 offset:6144\n"
          "ds_read_b32 %7, %8 offset:7168\n s_waitcnt lgkmcnt(0)"
          : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]),
            "=&v"(x[6]), "=&v"(x[7])
          : "v"(la));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = (float)sacc + (float)la;
#pragma unroll
  for (int i = 0; i < CH; ++i) s += x[i] + (float)d[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) {
    cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = t1 - t0;
    cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 1] = r1 - r0;
  }
}

template <int OP>
static int run(const char *name, int per_iter, int cus, float *out, unsigned long long *cyc) {
  // per wave: median of the waves' own s_memtime spans; per SIMD: the launch's HIP-event time
  // x the clock of the run (s_memtime / s_memrealtime) x 4 SIMDs per CU / wave-instructions
  // issued on the CU (every wave of a launch counted, whether or not they overlapped)
  printf("%-40s", name);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w : {1, 2, 4, 8}) {
    const int blocks = cus * w;   // 4 waves per block, one per SIMD: w waves per SIMD
    for (int rep = 0; rep < 3; ++rep)   // the first launches warm the clock
      hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, cyc, 1.0001f, 0.5f);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, cyc, 1.0001f, 0.5f);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.0f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> c(blocks * 8);
    CK(hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost));
    std::vector<unsigned long long> cy, rt;
    for (size_t k = 0; k < c.size(); k += 2) {
      cy.push_back(c[k]);
      rt.push_back(c[k + 1]);
    }
    std::sort(cy.begin(), cy.end());
    std::sort(rt.begin(), rt.end());
    const double insts = (double)ITER * per_iter;
    const double per_wave = (double)cy[cy.size() / 2] / insts;
    const double mhz = 100.0 * (double)cy[cy.size() / 2] / (double)std::max(1ull, rt[rt.size() / 2]);
    const double simd = (double)ms * 1e3 * mhz / (w * insts);   // cycles per wave-instr per SIMD
    printf("  %d/SIMD: %6.2f /wave %6.2f /SIMD", w, per_wave, simd);
  }
  printf("\n");
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return 0;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float *out;
  unsigned long long *cyc;
  CK(hipMalloc(&out, sizeof(float) * 256 * cus * 8));
  CK(hipMalloc(&cyc, 8 * 2 * 4 * cus * 8));
  printf("# cycles (s_memtime) per wave-instruction, median wave; %d CUs, %d chains x %d trips\n",
         cus, CH, ITER);
  run<0>("v_add_f32", CH, cus, out, cyc);
  run<1>("v_mul_f32", CH, cus, out, cyc);
  run<2>("v_fma_f32", CH, cus, out, cyc);
  run<11>("v_add_u32", CH, cus, out, cyc);
  run<10>("v_cndmask_b32", CH, cus, out, cyc);
  run<9>("v_mov_b32_dpp wave_shr:1", CH, cus, out, cyc);
  run<13>("v_add_f32_dpp wave_shr:1", CH, cus, out, cyc);
  run<3>("v_rcp_f32", CH, cus, out, cyc);
  run<4>("v_sqrt_f32", CH, cus, out, cyc);
  run<5>("v_rsq_f32", CH, cus, out, cyc);
  run<12>("4 v_add_f32 + 1 v_rcp_f32 (per op)", 5 * CH, cus, out, cyc);
  run<6>("v_add_f64", CH, cus, out, cyc);
  run<15>("v_mul_f64", CH, cus, out, cyc);
  run<7>("v_fma_f64", CH, cus, out, cyc);
  run<8>("v_cvt_f64_f32", CH, cus, out, cyc);
  run<14>("ds_read_b32 x8 + lgkmcnt(0) (per read)", 8, cus, out, cyc);
  run<21>("ds_read_b32 dependent chain (per read)", 8, cus, out, cyc);
  run<22>("ds_write_b32 x8 + lgkmcnt(0) (per write)", 8, cus, out, cyc);
  run<16>("v_cmp_gt_f32_e64", CH, cus, out, cyc);
  run<17>("v_mov_b32", CH, cus, out, cyc);
  run<18>("v_pk_add_f32", CH, cus, out, cyc);
  run<19>("v_readfirstlane_b32", CH, cus, out, cyc);
  run<23>("v_floor_f32", CH, cus, out, cyc);
  run<24>("v_cvt_i32_f32", CH, cus, out, cyc);
  run<25>("v_med3_f32", CH, cus, out, cyc);
  run<20>("s_add_u32", CH, cus, out, cyc);
  run<26>("s_barrier (4-wave block, per barrier)", 1, cus, out, cyc);
  run<27>("v_fma_f32 dependent chain (per fma)", CH, cus, out, cyc);
  run<28>("v_cndmask_b32_e32", CH, cus, out, cyc);
  run<29>("v_sub_f32", CH, cus, out, cyc);
  run<30>("v_max_f32", CH, cus, out, cyc);
  run<31>("v_cmp_gt_f32_e32", CH, cus, out, cyc);
  run<32>("v_and_b32", CH, cus, out, cyc);
  run<33>("v_lshl_add_u32", CH, cus, out, cyc);
  run<34>("v_mad_u32_u24", CH, cus, out, cyc);
  run<35>("v_cvt_f32_i32", CH, cus, out, cyc);
  run<36>("v_mul_f32_e64 (neg)", CH, cus, out, cyc);
  run<37>("v_mov_b64", CH, cus, out, cyc);
  run<38>("v_fmac_f32", CH, cus, out, cyc);
  run<39>("v_min_f32_e64 (abs)", CH, cus, out, cyc);
  run<40>("v_ldexp_f32", CH, cus, out, cyc);
  run<41>("v_lshlrev_b32", CH, cus, out, cyc);
  return 0;
}
