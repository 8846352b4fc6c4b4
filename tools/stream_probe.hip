// Memory-pattern probe for k_iterate_roll (no arithmetic): each wavefront walks down a
// 128-px column band (2 px per lane, 8-byte buffer loads/stores, bands overlapping by a
// 4-px halo), loading 9 planes per row two rows ahead and storing 6 planes per row, at
// C2 level-0 size (6144 x 4096).  Variant W16: the same bytes with 16-B accesses (planes
// paired AoS, 4 px... as 2 px x 2 planes per lane).  Prints GB/s for each.
// Build: hipcc -O3 --offload-arch=gfx950 tools/stream_probe.hip -o tools/_stream_probe
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int W = 6144, H = 4096, P = 6144;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs(const float *p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p), 0, (int)(4u * P * H), 0x00020000);
}

struct Planes { const float *in[9]; float *out[6]; };

template <int B> struct Vec;
template <> struct Vec<8> { typedef unsigned long long T; };
template <> struct Vec<16> { typedef unsigned int T __attribute__((ext_vector_type(4))); };

// B bytes per lane per plane (PX = B/4 px per lane), NIN planes loaded two rows ahead and
// NOUT planes stored per row; bands of 64*PX px overlapping by 4 px.
template <int B, int NIN, int NOUT>
__global__ __launch_bounds__(256) void probe(Planes pl, int bands, int seg) {
  constexpr int PX = B / 4, BW = 64 * PX, OUT = BW - 4;
  typedef typename Vec<B>::T V;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int band = wid % bands, sg = wid / bands;
  const int X = band * OUT - 4 + PX * lane;
  const unsigned vo = 4u * (unsigned)min(max(X, 0), P - PX);
  const int y0 = sg * seg, y1 = min(y0 + seg + 4, H);
  V a[NIN], b[NIN], c[NIN];
  auto ld = [&](V (&d)[NIN], int y) {
#pragma unroll
    for (int k = 0; k < NIN; ++k) {
      if constexpr (B == 8)
        d[k] = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b64(rs(pl.in[k]), (int)vo, (int)(4u * P * min(y, H - 1)), 0));
      else
        d[k] = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(rs(pl.in[k]), (int)vo, (int)(4u * P * min(y, H - 1)), 0));
    }
  };
  auto st = [&](const V (&d)[NIN], int y) {
    const bool ok = PX * lane >= 4 && PX * lane < BW - 4 && y < y1;
#pragma unroll
    for (int k = 0; k < NOUT; ++k) {
      V v = d[k] ^ d[(k + 3) % NIN];
      const int o = ok ? (int)(vo + 4u * P * y) : 0x7ffffff0;
      if constexpr (B == 8) {
        using T = decltype(__builtin_amdgcn_raw_buffer_load_b64(rs(pl.in[0]), 0, 0, 0));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(T, v), rs(pl.out[k]), o, 0, 0);
      } else {
        using T = decltype(__builtin_amdgcn_raw_buffer_load_b128(rs(pl.in[0]), 0, 0, 0));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(T, v), rs(pl.out[k]), o, 0, 0);
      }
    }
  };
  ld(a, y0);
  ld(b, y0 + 1);
  for (int y = y0; y < y1; y += 3) {
    ld(c, y + 2); __builtin_amdgcn_sched_barrier(0); st(a, y);
    ld(a, y + 3); __builtin_amdgcn_sched_barrier(0); st(b, y + 1);
    ld(b, y + 4); __builtin_amdgcn_sched_barrier(0); st(c, y + 2);
  }
}

// Same bytes, but R rows are loaded, then R rows stored (stores in bursts per wave).
template <int R>
__global__ __launch_bounds__(256) void probe_burst(Planes pl, int bands, int seg) {
  constexpr int NIN = 9, NOUT = 6;
  typedef unsigned long long V;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int band = wid % bands, sg = wid / bands;
  const int X = band * 124 - 4 + 2 * lane;
  const unsigned vo = 4u * (unsigned)min(max(X, 0), P - 2);
  const int y0 = sg * seg, y1 = min(y0 + seg + 4, H);
  V d[R][NIN];
  for (int y = y0; y < y1; y += R) {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int k = 0; k < NIN; ++k)
        d[r][k] = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b64(rs(pl.in[k]), (int)vo, (int)(4u * P * min(y + r, H - 1)), 0));
    __builtin_amdgcn_sched_barrier(0);
    const bool okl = 2 * lane >= 4 && 2 * lane < 124;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int k = 0; k < NOUT; ++k) {
        V v = d[r][k] ^ d[r][(k + 3) % NIN];
        using T = decltype(__builtin_amdgcn_raw_buffer_load_b64(rs(pl.in[0]), 0, 0, 0));
        const int o = okl && y + r < y1 ? (int)(vo + 4u * P * (y + r)) : 0x7ffffff0;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(T, v), rs(pl.out[k]), o, 0, 0);
      }
  }
}

template <int R>
void run_burst(const Planes &pl) {
  const int bands = (W + 123) / 124;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int seg : {64, 128}) {
    const int waves = bands * ((H + seg - 1) / seg);
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL((probe_burst<R>), dim3((waves + 3) / 4), dim3(256), 0, 0, pl, bands, seg);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep) best = ms < best ? ms : best;
    }
    const double rows = (double)bands * 128 * ((double)H + 4.0 * ((H + seg - 1) / seg));
    const double bytes = rows * 4 * 9 + (double)W * H * 4 * 6;
    printf("burst R=%d b64 9 in 6 out   seg %3d waves %5d: %7.1f us %6.0f GB/s\n", R, seg, waves,
           best * 1e3, bytes / (best * 1e-3) / 1e9);
  }
}

template <int B, int NIN, int NOUT>
void run(const Planes &pl, const char *name) {
  constexpr int PX = B / 4, OUT = 64 * PX - 4;
  const int bands = (W + OUT - 1) / OUT;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int seg : {32, 64, 128}) {
    const int waves = bands * ((H + seg - 1) / seg);
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL((probe<B, NIN, NOUT>), dim3((waves + 3) / 4), dim3(256), 0, 0, pl, bands, seg);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep) best = ms < best ? ms : best;
    }
    const double rows = (double)bands * 64 * PX * ((double)H + 4.0 * ((H + seg - 1) / seg));
    const double bytes = rows * B / PX * NIN + (double)W * H * B / PX * NOUT;
    printf("%-28s seg %3d waves %5d: %7.1f us %6.0f GB/s  (%.2f GB)\n", name, seg, waves, best * 1e3,
           bytes / (best * 1e-3) / 1e9, bytes / 1e9);
  }
}

int main() {
  Planes pl;
  const size_t plane = 4ull * P * H;
  for (int k = 0; k < 9; ++k) { float *p; (void)hipMalloc((void **)&p, plane); (void)hipMemset(p, 0, plane); pl.in[k] = p; }
  for (int k = 0; k < 6; ++k) { float *p; (void)hipMalloc((void **)&p, plane); pl.out[k] = p; }
  run<8, 9, 6>(pl, "2px b64 9 planes in, 6 out");
  run<16, 9, 6>(pl, "4px b128 9 planes in, 6 out");
  run<16, 5, 3>(pl, "2px-pairs b128 5 in, 3 out");
  run<8, 5, 3>(pl, "1px-pairs b64 5 in, 3 out");
  run_burst<1>(pl);
  run_burst<2>(pl);
  run_burst<4>(pl);
  run_burst<8>(pl);
  return 0;
}
