// Calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the
// engine uses (MI355X_MICROARCH.md: only 16-B-per-lane streams are calibrated there).
// Each kernel streams a known byte count (1 GiB, past the 256 MiB Infinity Cache) with
// raw buffer loads or stores of 4, 8 or 16 B per lane, coalesced, one pass.
// Build: hipcc -O3 --offload-arch=gfx950 tools/calib_fetch.hip -o tools/_calib_fetch
// Run:   rocprofv3 --pmc FETCH_SIZE -d <dir> -o run -- tools/_calib_fetch   (then WRITE_SIZE)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void *p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)bytes, 0x00020000);
}

// every block streams `chunk` bytes; `sink` keeps loads alive (one dword per block)
template <int B>
__global__ void rd(float *base, unsigned bytes, unsigned chunk, float *sink) {
  const auto r = rsrc(base, bytes);
  float acc = 0.0f;
  const unsigned beg = blockIdx.x * chunk;
  for (unsigned o = beg + threadIdx.x * B; o < beg + chunk; o += 256 * B) {
    if constexpr (B == 4) acc += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)o, 0, 0));
    if constexpr (B == 8) {
      auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)o, 0, 0);
      float f[2];
      __builtin_memcpy(f, &v, 8);
      acc += f[0] + f[1];
    }
    if constexpr (B == 16) {
      auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)o, 0, 0);
      float f[4];
      __builtin_memcpy(f, &v, 16);
      acc += f[0] + f[1] + f[2] + f[3];
    }
  }
  if (acc == 12345.678f) sink[blockIdx.x] = acc;   // never true for zeroed memory
}

template <int B>
__global__ void wr(float *base, unsigned bytes, unsigned chunk) {
  const auto r = rsrc(base, bytes);
  const unsigned beg = blockIdx.x * chunk;
  for (unsigned o = beg + threadIdx.x * B; o < beg + chunk; o += 256 * B) {
    if constexpr (B == 4) __builtin_amdgcn_raw_buffer_store_b32(0u, r, (int)o, 0, 0);
    if constexpr (B == 8) {
      auto v = __builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0);   // type only
      v = decltype(v){};
      __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)o, 0, 0);
    }
    if constexpr (B == 16) {
      auto v = __builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 0);
      v = decltype(v){};
      __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)o, 0, 0);
    }
  }
}

int main() {
  const unsigned bytes = 1u << 30, chunk = 1u << 20, blocks = bytes / chunk;
  float *buf = nullptr, *sink = nullptr;
  if (hipMalloc((void **)&buf, bytes) != hipSuccess || hipMalloc((void **)&sink, 4 * blocks) != hipSuccess) {
    fprintf(stderr, "hipMalloc failed\n");
    return 1;
  }
  (void)hipMemset(buf, 0, bytes);
  (void)hipDeviceSynchronize();
  // order: rd4, rd8, rd16, wr4, wr8, wr16 (each dispatch moves exactly `bytes`)
  hipLaunchKernelGGL(rd<4>, dim3(blocks), dim3(256), 0, 0, buf, bytes, chunk, sink);
  hipLaunchKernelGGL(rd<8>, dim3(blocks), dim3(256), 0, 0, buf, bytes, chunk, sink);
  hipLaunchKernelGGL(rd<16>, dim3(blocks), dim3(256), 0, 0, buf, bytes, chunk, sink);
  hipLaunchKernelGGL(wr<4>, dim3(blocks), dim3(256), 0, 0, buf, bytes, chunk);
  hipLaunchKernelGGL(wr<8>, dim3(blocks), dim3(256), 0, 0, buf, bytes, chunk);
  hipLaunchKernelGGL(wr<16>, dim3(blocks), dim3(256), 0, 0, buf, bytes, chunk);
  if (hipDeviceSynchronize() != hipSuccess) {
    fprintf(stderr, "kernel failed\n");
    return 1;
  }
  printf("calib: 6 dispatches x %u bytes (rd4 rd8 rd16 wr4 wr8 wr16)\n", bytes);
  (void)hipFree(buf);
  (void)hipFree(sink);
  return 0;
}
