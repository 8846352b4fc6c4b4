// Wave-to-SIMD placement probe: which SIMD of its CU each wavefront of a block lands on
// (HW_ID register), for 4-wave (k_warp_iter NC = 2) and 3-wave (NC = 1) blocks at the
// occupancy those kernels run (LDS sized so 4 / 5 blocks share a CU).  Prints, per wave
// index in the block, how often it sat on SIMD 0..3, and how many distinct SIMDs the
// waves of one block covered.
// Build: hipcc -O3 --offload-arch=gfx950 tools/simd_probe.hip -o tools/_simd_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int NW, int LDSB>
__global__ __launch_bounds__(64 * NW) void probe(unsigned *out, int spin) {
  __shared__ float pad[LDSB / 4];
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID
  float acc = (float)threadIdx.x;
  for (int i = 0; i < spin; ++i) acc = __builtin_fmaf(acc, 1.0001f, 0.5f);
  pad[threadIdx.x] = acc;
  __syncthreads();
  if ((threadIdx.x & 63) == 0)
    out[blockIdx.x * NW + (threadIdx.x >> 6)] = pad[(threadIdx.x + 64) % (64 * NW)] == -1.0f ? 0u : hw;
}

template <int NW, int LDSB>
void run(int blocks) {
  unsigned *d;
  hipMalloc(&d, sizeof(unsigned) * blocks * NW);
  hipLaunchKernelGGL((probe<NW, LDSB>), dim3(blocks), dim3(64 * NW), 0, 0, d, 20000);
  hipDeviceSynchronize();
  std::vector<unsigned> h(blocks * NW);
  hipMemcpy(h.data(), d, sizeof(unsigned) * h.size(), hipMemcpyDeviceToHost);
  hipFree(d);
  int hist[4][4] = {};
  int cover[5] = {};
  for (int b = 0; b < blocks; ++b) {
    int mask = 0;
    for (int w = 0; w < NW; ++w) {
      const int simd = (h[b * NW + w] >> 4) & 3;
      hist[w][simd]++;
      mask |= 1 << simd;
    }
    cover[__builtin_popcount(mask)]++;
  }
  printf("%d-wave blocks, %d B LDS, %d blocks\n", NW, LDSB, blocks);
  for (int w = 0; w < NW; ++w)
    printf("  wave %d: simd0 %d simd1 %d simd2 %d simd3 %d\n", w, hist[w][0], hist[w][1], hist[w][2],
           hist[w][3]);
  printf("  distinct SIMDs per block: 1:%d 2:%d 3:%d 4:%d\n", cover[1], cover[2], cover[3], cover[4]);
}

int main() {
  run<4, 40192>(4096);
  run<3, 32000>(4096);
  return 0;
}
