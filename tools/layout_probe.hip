// HBM layout probe for the 2-iteration pass pattern (no arithmetic): the k_iterate_roll
// access stream (128-px column bands, 2 px per lane, 8-byte buffer accesses, 9 planes
// loaded two rows ahead, 6 planes stored per row) at C2 level-0 size, with the 15 planes
// laid out three ways:
//   sep    : one plane after another (plane k at k * P*H), row stride P;
//   stagger: the same with plane k shifted by k * SHIFT bytes;
//   rows   : row-interleaved ([row][plane][col]), row stride 15 P, so one row of every
//            plane is one contiguous 15 * 24 KB span.
// Prints GB/s (algorithmic bytes / time) for each.
// Build: hipcc -O3 --offload-arch=gfx950 tools/layout_probe.hip -o tools/_layout_probe
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int W = 6144, H = 4096, P = 6144, NP = 15, NIN = 9, NOUT = 6;

struct Planes { const float *in[NIN]; float *out[NOUT]; unsigned nb_in[NIN], nb_out[NOUT]; };

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs(const float *p, unsigned nb) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p), 0, (int)nb, 0x00020000);
}

typedef unsigned long long V;

template <int AL, int AS>
__global__ __launch_bounds__(256) void probe(Planes pl, int bands, int seg, int S) {
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int band = wid % bands, sg = wid / bands;
  const int X = band * 124 - 4 + 2 * lane;
  const unsigned vo = 4u * (unsigned)min(max(X, 0), P - 2);
  const int y0 = sg * seg, y1 = min(y0 + seg + 4, H);
  V a[NIN], b[NIN], c[NIN];
  auto ld = [&](V (&d)[NIN], int y) {
#pragma unroll
    for (int k = 0; k < NIN; ++k)
      d[k] = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b64(rs(pl.in[k], pl.nb_in[k]), (int)vo,
                                                                        (int)(4u * S * min(y, H - 1)), AL));
  };
  auto st = [&](const V (&d)[NIN], int y) {
    const bool ok = 2 * lane >= 4 && 2 * lane < 124 && y < y1;
#pragma unroll
    for (int k = 0; k < NOUT; ++k) {
      V v = d[k] ^ d[(k + 3) % NIN];
      const int o = ok ? (int)(vo + 4u * S * y) : 0x7ffffff0;
      using T = decltype(__builtin_amdgcn_raw_buffer_load_b64(rs(pl.in[0], 0), 0, 0, 0));
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(T, v), rs(pl.out[k], pl.nb_out[k]), o, 0, AS);
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

static float *g_buf;
static size_t g_bytes;

// plane k starts at float offset base[k]; row stride S floats
template <int AL = 0, int AS = 0>
static void run(const char *name, const size_t (&base)[NP], int S) {
  Planes pl;
  for (int k = 0; k < NP; ++k) {
    float *p = g_buf + base[k];
    const unsigned nb = (unsigned)((g_bytes - 4 * base[k]) > 0x7ffffff0u ? 0x7ffffff0u : (g_bytes - 4 * base[k]));
    if (k < NIN) { pl.in[k] = p; pl.nb_in[k] = nb; }
    else { pl.out[k - NIN] = p; pl.nb_out[k - NIN] = nb; }
  }
  const int bands = (W + 123) / 124;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int seg : {64, 128}) {
    const int waves = bands * ((H + seg - 1) / seg);
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL((probe<AL, AS>), dim3((waves + 3) / 4), dim3(256), 0, 0, pl, bands, seg, S);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep) best = ms < best ? ms : best;
    }
    const double rows = (double)bands * 128 * ((double)H + 4.0 * ((H + seg - 1) / seg));
    const double bytes = rows * 4 * NIN + (double)W * H * 4 * NOUT;
    printf("%-34s seg %3d: %7.1f us %6.0f GB/s\n", name, seg, best * 1e3, bytes / (best * 1e-3) / 1e9);
  }
}

int main() {
  const size_t plane = (size_t)P * H;
  g_bytes = 4 * (NP * plane + NP * 8192);
  (void)hipMalloc((void **)&g_buf, g_bytes);
  (void)hipMemset(g_buf, 0, g_bytes);
  size_t base[NP];
  for (int k = 0; k < NP; ++k) base[k] = k * plane;
  run("sep (plane after plane)", base, P);
  run<2, 0>("sep, nt loads", base, P);
  run<0, 2>("sep, nt stores", base, P);
  run<2, 2>("sep, nt loads + stores", base, P);
  run<0, 16>("sep, sc1 stores", base, P);
  for (int shift : {256, 4096 + 256}) {
    for (int k = 0; k < NP; ++k) base[k] = k * plane + (size_t)k * shift / 4;
    char name[64];
    snprintf(name, sizeof name, "stagger %d B per plane", shift);
    run(name, base, P);
  }
  for (int k = 0; k < NP; ++k) base[k] = (size_t)k * P;
  run("rows ([row][plane][col])", base, NP * P);
  return 0;
}
