// k_warp_iter on one C2 level-0 geometry (6144 x 4096, synthetic inputs), alone: kernel
// time by HIP events, and per wavefront its start / end (s_memrealtime, 100 MHz) and
// hardware slot, to see how the one-round launch spends its time (start skew, wave
// lifetime spread, tail).
//   hipcc -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 \
//     -I include -I fibsem-optflow_amd/csrc tools/wi_probe.hip -o tools/_bin/wi_probe
//   tools/_bin/wi_probe [W H reps seg_rows]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#ifdef WI_BARRIER   // -DWI_BARRIER: also time each wave's barrier waits (perturbs the timing)
#define TVL1_BARRIER_PROBE
#endif
#include "tvl1_kernels.hpp"

using namespace tvl1k;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

#ifndef WI_BW
#define WI_BW 128
#endif
#ifndef WI_M
#define WI_M 6
#endif
#ifndef WI_NC
#define WI_NC 2
#endif
constexpr int M = WI_M, BW = WI_BW, NC = WI_NC, NWV = NC + BW / 64;   // waves per block

#ifdef WI_WPE
#define WI_ATTR __attribute__((amdgpu_waves_per_eu(WI_WPE)))
#else
#define WI_ATTR
#endif
template <int FM, int PRIO>
__global__ __launch_bounds__(64 * NC + BW) WI_ATTR void k_probe(WarpIterArgs w, unsigned long long *ts) {
  __shared__ float ring[wi_rows<M>() * ring_pitch(wi_ww<M, BW>())];
  __shared__ float cring[2 * 5 * BW];
  __shared__ float hring[NC == 2 ? 2 * kWiH * BW : 1];
  const int wid = __builtin_amdgcn_readfirstlane(xcd_chunk(blockIdx.x, gridDim.x));
  if (wid >= w.ra.waves) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  warp_iter_body<M, FM, BW, PRIO, NC>(w, wid, ring, cring, hring);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
#ifdef WI_BARRIER
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_fetch_add(tvl1_probe_bar + NWV * (size_t)gridDim.x + NWV * blockIdx.x + (threadIdx.x >> 6),
                           c1 - c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  (void)c0;
  (void)c1;
#endif
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // XCC_ID
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    unsigned long long *o = ts + 4 * (NWV * (size_t)blockIdx.x + wv);
    o[0] = t0;
    o[1] = t1;
    o[2] = hw;
    o[3] = xcc;
  }
}

static int roll_segment(int bands, int lh, int k, int slots) {
  int best = lh;
  long best_cost = -1;
  for (int R = 1; R <= 4; ++R) {
    const int segs = std::max(1, R * slots / bands);
    const int seg = std::max(8, (lh + segs - 1) / segs);
    const long waves = (long)bands * ((lh + seg - 1) / seg);
    const long rounds = (waves + slots - 1) / slots;
    const long cost = rounds * (seg + 2 * k);
    if (best_cost < 0 || cost < best_cost) {
      best_cost = cost;
      best = seg;
    }
  }
  return best;
}

int main(int argc, char **argv) {
  const int W = argc > 1 ? atoi(argv[1]) : 6144, H = argc > 2 ? atoi(argv[2]) : 4096;
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  const int seg_arg = argc > 4 ? atoi(argv[4]) : 0;
  // mode 1: the consumer's HBM accesses (p loads, u / p stores) out of range (dropped);
  // mode 2: every access out of range (P = 0): the launch without HBM traffic
  const int mode = argc > 5 ? atoi(argv[5]) : 0;
  const int P = (W + 63) / 64 * 64;
  const size_t plane = (size_t)P * H;
  const size_t pstride = plane * 4;
  // planes: I0, I1, C[3], U0[2], U1[2], P0[4], P1[4]
  std::vector<float> h(plane);
  float *base;
  CK(hipMalloc(&base, 17 * pstride));
  float *pl[17];
  for (int i = 0; i < 17; ++i) pl[i] = base + i * plane;
  auto fill = [&](float *d, auto f) {
    for (int y = 0; y < H; ++y)
      for (int x = 0; x < P; ++x) h[(size_t)y * P + x] = x < W ? f(x, y) : 0.0f;
    CK(hipMemcpy(d, h.data(), pstride, hipMemcpyHostToDevice));
  };
  auto tex = [](float x, float y) {
    return 127.5f + 60.0f * sinf(0.11f * x + 0.05f * y) * cosf(0.07f * y - 0.03f * x) +
           40.0f * sinf(0.031f * x * 0.7f + 0.023f * y);
  };
  fill(pl[0], [&](int x, int y) { return tex(x, y); });
  fill(pl[1], [&](int x, int y) { return tex(x + 1.3f * sinf(0.002f * y), y + 0.8f * cosf(0.003f * x)); });
  fill(pl[5], [&](int x, int y) { return 1.2f * sinf(0.002f * y); });
  fill(pl[6], [&](int x, int y) { return 0.7f * cosf(0.003f * x); });
  for (int i = 9; i < 13; ++i)
    fill(pl[i], [&](int x, int y) { return 0.3f * sinf(0.01f * x * (i - 7) + 0.013f * y); });
  double *partials;
  const int maxblk = 1 << 16;
  CK(hipMalloc(&partials, maxblk * sizeof(double)));

  WarpIterArgs w{};
  IterArgs &a = w.ra.it;
  a.W = W;
  a.H = H;
  a.P = P;
  a.l_t = 0.15f * 0.3f;
  a.theta = 0.3f;
  a.gamma = 0.0f;
  a.taut = 0.25f / 0.3f;
  a.calc_err = 1;
  a.p_zero = 0;
  a.partials = partials;
  a.I1wx = pl[2]; a.I1wy = pl[3]; a.rho = pl[4];
  a.u1s = pl[5]; a.u2s = pl[6]; a.u1d = pl[7]; a.u2d = pl[8];
  a.p11s = pl[9]; a.p12s = pl[10]; a.p21s = pl[11]; a.p22s = pl[12];
  a.p11d = pl[13]; a.p12d = pl[14]; a.p21d = pl[15]; a.p22d = pl[16];
  RollBufs &b = w.ra.b;
  b.c = pl[2]; b.us = pl[5]; b.ud = pl[7]; b.ps = pl[9]; b.pd = pl[13];
  b.pstride = (unsigned)pstride;
  b.cb = (unsigned)(2 * pstride + plane * 4);
  b.ub = (unsigned)(1 * pstride + plane * 4);
  b.pb = (unsigned)(3 * pstride + plane * 4);
  w.I0 = pl[0];
  w.I1 = pl[1];
  w.store_c = 0;
  if (mode >= 1) b.cb = b.ub = b.pb = 0;
  if (mode >= 2) a.P = 0;

  int per_cu = 0, cus = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)k_probe<0, 0>, 64 * NC + BW, 0));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int slots = per_cu * cus;
  w.ra.bands = (W + BW - 5) / (BW - 4);
  w.ra.seg_rows = seg_arg > 0 ? seg_arg : roll_segment(w.ra.bands, H, 2 + M, slots);
  w.ra.waves = w.ra.bands * ((H + w.ra.seg_rows - 1) / w.ra.seg_rows);
  printf("mode %d: ", mode);
  printf("W %d H %d bands %d seg_rows %d blocks %d slots %d (%d/CU)\n", W, H, w.ra.bands,
         w.ra.seg_rows, w.ra.waves, slots, per_cu);
  if (w.ra.waves > maxblk) return 1;
  unsigned long long *ts;
  CK(hipMalloc(&ts, (size_t)w.ra.waves * NWV * 4 * sizeof(unsigned long long)));
  unsigned long long *bar;
  const size_t nbar = (size_t)w.ra.waves * NWV * 2;
  CK(hipMalloc(&bar, nbar * 8));
#ifdef WI_BARRIER
  CK(hipMemcpyToSymbol(HIP_SYMBOL(tvl1_probe_bar), &bar, sizeof(bar)));
#endif
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int prio = 0;
  auto run = [&](bool probe) {
    float best = 1e30f, sum = 0.0f;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0));
      CK(hipMemset(bar, 0, nbar * 8));
      if (probe && prio)
        hipLaunchKernelGGL((k_probe<0, 1>), dim3(w.ra.waves), dim3(64 * NC + BW), 0, 0, w, ts);
      else if (probe)
        hipLaunchKernelGGL((k_probe<0, 0>), dim3(w.ra.waves), dim3(64 * NC + BW), 0, 0, w, ts);
      else
        hipLaunchKernelGGL((k_warp_iter<M, 0, BW, 1, NC>), dim3(w.ra.waves), dim3(64 * NC + BW), 0, 0, w);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
      if (r) sum += ms;
    }
    printf("%s: best %.1f us, mean %.1f us\n", probe ? (prio ? "probe+prio" : "probe") : "k_warp_iter (engine, prio)", 1e3f * best,
           1e3f * sum / (reps - 1));
  };
  run(false);
  for (prio = 0; prio < 2; ++prio) {
  run(true);
  std::vector<unsigned long long> t((size_t)w.ra.waves * 4 * NWV);
  CK(hipMemcpy(t.data(), ts, t.size() * 8, hipMemcpyDeviceToHost));
  int rate_khz = 0;
  CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
  const double us = 1e3 / rate_khz;
  unsigned long long t0 = ~0ull, t1 = 0;
  for (int i = 0; i < w.ra.waves * NWV; ++i) {
    t0 = std::min(t0, t[4 * i]);
    t1 = std::max(t1, t[4 * i + 1]);
  }
  printf("span %.1f us (clock %d kHz)\n", (t1 - t0) * us, rate_khz);
  std::vector<double> st, en, life;
  std::vector<double> xe(8, 0.0), xn(8, 0.0);
  for (int bl = 0; bl < w.ra.waves; ++bl) {
    const unsigned long long *o = &t[4 * NWV * bl];
    st.push_back((o[0] - t0) * us);
    unsigned long long e = 0;
    for (int v = 0; v < NWV; ++v) e = std::max(e, o[4 * v + 1]);
    en.push_back((e - t0) * us);
    life.push_back((o[1] - o[0]) * us);
    const int x = (int)(o[3] & 7);
    xe[x] += en.back();
    xn[x] += 1;
  }
  auto q = [](std::vector<double> v, double f) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(f * (v.size() - 1))];
  };
  printf("block start  us: min %.1f p50 %.1f p90 %.1f max %.1f\n", q(st, 0), q(st, .5), q(st, .9), q(st, 1));
  printf("block end    us: min %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f\n", q(en, 0), q(en, .1),
         q(en, .5), q(en, .9), q(en, 1));
  printf("block life   us: min %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f\n", q(life, 0), q(life, .1),
         q(life, .5), q(life, .9), q(life, 1));
  double busy = 0;
  for (double l : life) busy += l;
  printf("mean life / span: %.3f\n", busy / life.size() / ((t1 - t0) * us));
  for (int x = 0; x < 8; ++x)
    if (xn[x] > 0) printf("xcc %d: %4.0f blocks, mean end %.1f us\n", x, xn[x], xe[x] / xn[x]);
  // blocks per CU (se, cu) and the end time against the CU's block count
  std::vector<int> cnt(8 * 64 * 16, 0);
  auto cu_key = [&](const unsigned long long *o) {
    const unsigned hw = (unsigned)o[2];
    const int cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    return (((int)(o[3] & 7) * 8 + se) * 2 + sh) * 16 + cu;
  };
  for (int bl = 0; bl < w.ra.waves; ++bl) cnt[cu_key(&t[4 * NWV * bl])]++;
  std::vector<double> eb(8, 0.0), nb(8, 0.0);
  int used = 0;
  for (int c : cnt) used += c > 0;
  for (int bl = 0; bl < w.ra.waves; ++bl) {
    const int c = std::min(cnt[cu_key(&t[4 * NWV * bl])], 7);
    eb[c] += en[bl];
    nb[c] += 1;
  }
  printf("CUs used %d\n", used);
  for (int c = 1; c < 8; ++c)
    if (nb[c] > 0) printf("CU holding %d blocks: %5.0f blocks, mean end %.1f us\n", c, nb[c], eb[c] / nb[c]);
  // SIMD composition: waves (consumers / producers) on each SIMD, for the whole launch
  auto simd_key = [&](const unsigned long long *o) { return cu_key(o) * 4 + (int)((o[2] >> 4) & 3); };
  std::vector<int> scons(8 * 64 * 16 * 4, 0), sprod(8 * 64 * 16 * 4, 0);
  for (int bl = 0; bl < w.ra.waves; ++bl)
    for (int v = 0; v < NWV; ++v) (v < NC ? scons : sprod)[simd_key(&t[4 * NWV * bl + 4 * v])]++;
  {
    double acc[8][8] = {}, n[8][8] = {};
    for (int bl = 0; bl < w.ra.waves; ++bl) {
      const int k = simd_key(&t[4 * NWV * bl]);
      const int c = std::min(scons[k], 7), pr = std::min(sprod[k], 7);
      acc[c][pr] += life[bl];
      n[c][pr] += 1;
    }
    printf("consumer's SIMD holds (consumers, producers): blocks, mean life\n");
    for (int c = 0; c < 8; ++c)
      for (int pr = 0; pr < 8; ++pr)
        if (n[c][pr] > 0) printf("  (%d, %d): %5.0f blocks, life %.1f us\n", c, pr, n[c][pr], acc[c][pr] / n[c][pr]);
    double accm[8] = {}, nm[8] = {};
    for (int bl = 0; bl < w.ra.waves; ++bl) {
      int mx = 0;
      for (int v = 0; v < NWV; ++v) {
        const int k = simd_key(&t[4 * NWV * bl + 4 * v]);
        mx = std::max(mx, 2 * scons[k] + sprod[k]);
      }
      mx = std::min(mx, 7);
      accm[mx] += life[bl];
      nm[mx] += 1;
    }
    printf("max over the block's SIMDs of (2 x consumers + producers): blocks, mean life\n");
    for (int m = 0; m < 8; ++m)
      if (nm[m] > 0) printf("  %d: %5.0f blocks, life %.1f us\n", m, nm[m], accm[m] / nm[m]);
  }
  {
    const int segs = (H + w.ra.seg_rows - 1) / w.ra.seg_rows;
    std::vector<double> sl(segs, 0.0), sn(segs, 0.0), bl_(w.ra.bands, 0.0), bn(w.ra.bands, 0.0);
    for (int bl = 0; bl < w.ra.waves; ++bl) {
      const int wid = [&] {
        const int n = w.ra.waves, q = n / 8, rem = n % 8, x = bl % 8, i = bl / 8;
        return x * q + std::min(x, rem) + i;
      }();
      sl[wid / w.ra.bands] += life[bl]; sn[wid / w.ra.bands] += 1;
      bl_[wid % w.ra.bands] += life[bl]; bn[wid % w.ra.bands] += 1;
    }
    printf("life by segment:");
    for (int i = 0; i < segs; ++i) printf(" %.0f", sl[i] / sn[i]);
    printf("\nlife by band:");
    for (int i = 0; i < w.ra.bands; ++i) printf(" %.0f", bl_[i] / bn[i]);
    printf("\n");
  }
  // simd placement of the three waves of each block
  std::vector<int> sim(4, 0);
  for (int i = 0; i < w.ra.waves * NWV; ++i) sim[(t[4 * i + 2] >> 4) & 3]++;
  printf("waves per simd id: %d %d %d %d\n", sim[0], sim[1], sim[2], sim[3]);
#ifdef WI_BARRIER
  {  // barrier wait share per role (shader cycles, last repetition)
    std::vector<unsigned long long> hb(nbar);
    CK(hipMemcpy(hb.data(), bar, nbar * 8, hipMemcpyDeviceToHost));
    double bw[NWV] = {}, lf[NWV] = {};
    for (int bl = 0; bl < w.ra.waves; ++bl)
      for (int v = 0; v < NWV; ++v) {
        bw[v] += hb[NWV * bl + v];
        lf[v] += hb[NWV * (size_t)w.ra.waves + NWV * bl + v];
      }
    printf("barrier share of wave life (waves 0..%d, consumers first):", NWV - 1);
    for (int v = 0; v < NWV; ++v) printf(" %.3f", bw[v] / lf[v]);
    printf("\n");
  }
#endif
  {  // life by dispatch ordinal on the CU (blocks of one CU in blockIdx order)
    std::vector<int> seen(8 * 64 * 16, 0);
    double acc[8] = {}, n[8] = {};
    for (int bl = 0; bl < w.ra.waves; ++bl) {
      const int o = std::min(seen[cu_key(&t[4 * NWV * bl])]++, 7);
      acc[o] += life[bl];
      n[o] += 1;
    }
    printf("life by dispatch ordinal on the CU:");
    for (int o = 0; o < 8; ++o)
      if (n[o] > 0) printf(" %d: %.1f (%.0f)", o, acc[o] / n[o], n[o]);
    printf("\n");
  }
  }
  return 0;
}
