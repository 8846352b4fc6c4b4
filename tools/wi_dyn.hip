// k_warp_iter's launch tail: the shipped one-round static launch
// (k_warp_iter, one block per (band, segment), 1000 blocks on 1024 slots at C2 level 0)
// against persistent blocks that pull (band, row range) items from a per-XCD queue
// (one global atomic counter per XCD, vector atomics).  Items are cut per XCD from its
// contiguous row range over all bands: a first round of S1-row items, one per block, then
// the rest in S2-row items, so the last round is short.  Same per-px arithmetic; the
// residual partials go to one slot per item.  Prints best / mean HIP-event time per
// launch for each schedule, and the spread of per-block end times (s_memrealtime).
//   hipcc -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 \
//     -I include -I fibsem-optflow_amd/csrc tools/wi_dyn.hip -o tools/_bin/wi_dyn
//   tools/_bin/wi_dyn [W H reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "tvl1_kernels.hpp"

using namespace tvl1k;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

constexpr int M = 6, BW = 128, NC = 2, NWV = NC + BW / 64;

struct Item {
  int band, ys, ye, slot;
};

// persistent blocks: block b serves XCD queue b % 8 (the dispatcher's round-robin)
__global__ __launch_bounds__(64 * NC + BW) void k_dyn(WarpIterArgs w, const Item *__restrict__ items,
                                                       const int *__restrict__ qbase,
                                                       const int *__restrict__ qcount, int *heads,
                                                       unsigned long long *ts) {
  __shared__ float ring[wi_rows<M>() * ring_pitch(wi_ww<M, BW>())];
  __shared__ float cring[2 * 5 * BW];
  __shared__ float hring[2 * kWiH * BW];
  __shared__ int s_it;
  const int x = blockIdx.x % kXcds;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const int n = qcount[x], base = qbase[x];
  for (;;) {
    if (threadIdx.x == 0)
      s_it = __hip_atomic_fetch_add(heads + x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();   // also: every wave is done with the previous item's LDS rings
    const int it = __builtin_amdgcn_readfirstlane(s_it);
    if (it >= n) break;
    const Item I = items[base + it];
    warp_iter_seg<M, 0, BW, 1, NC>(w, __builtin_amdgcn_readfirstlane(I.band),
                                   __builtin_amdgcn_readfirstlane(I.ys),
                                   __builtin_amdgcn_readfirstlane(I.ye),
                                   __builtin_amdgcn_readfirstlane(I.slot), ring, cring, hring);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    ts[2 * blockIdx.x] = t0;
    ts[2 * blockIdx.x + 1] = t1;
  }
}

static int roll_segment(int bands, int lh, int k, int slots) {   // the engine's rule
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

// per XCD x: rows [x H / 8, (x+1) H / 8) of every band; the first nblk items S1 rows (bands
// round-robin), then what is left of each band in pieces of at most S2 rows, longest first
static void make_items(int H, int bands, int nblk, int S1, int S2, std::vector<Item> &items,
                       std::vector<int> &qbase, std::vector<int> &qcount) {
  items.clear();
  qbase.assign(kXcds, 0);
  qcount.assign(kXcds, 0);
  int slot = 0;
  for (int x = 0; x < kXcds; ++x) {
    const int r0 = (int)((long)H * x / kXcds), r1 = (int)((long)H * (x + 1) / kXcds);
    std::vector<int> next(bands, r0);
    qbase[x] = (int)items.size();
    for (int i = 0, b = 0; i < nblk; ++i, b = (b + 1) % bands) {
      int tries = 0;
      while (next[b] >= r1 && tries++ < bands) b = (b + 1) % bands;
      if (next[b] >= r1) break;
      const int ye = std::min(next[b] + S1, r1);
      items.push_back({b, next[b], ye, slot++});
      next[b] = ye;
    }
    std::vector<Item> rest;
    for (int b = 0; b < bands; ++b)
      for (int y = next[b]; y < r1; y += S2) rest.push_back({b, y, std::min(y + S2, r1), 0});
    std::stable_sort(rest.begin(), rest.end(),
                     [](const Item &p, const Item &q) { return p.ye - p.ys > q.ye - q.ys; });
    for (Item &it : rest) {
      it.slot = slot++;
      items.push_back(it);
    }
    qcount[x] = (int)items.size() - qbase[x];
  }
}

int main(int argc, char **argv) {
  const int W = argc > 1 ? atoi(argv[1]) : 6144, H = argc > 2 ? atoi(argv[2]) : 4096;
  const int reps = argc > 3 ? atoi(argv[3]) : 10;
  const int P = (W + 63) / 64 * 64;
  const size_t plane = (size_t)P * H;
  const size_t pstride = plane * 4;
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
  const int maxslots = 1 << 16;
  CK(hipMalloc(&partials, maxslots * sizeof(double)));

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

  int per_cu = 0, cus = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)k_dyn, 64 * NC + BW, 0));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int slots = per_cu * cus;
  w.ra.bands = (W + BW - 5) / (BW - 4);
  w.ra.seg_rows = roll_segment(w.ra.bands, H, 2 + M, slots);
  w.ra.waves = w.ra.bands * ((H + w.ra.seg_rows - 1) / w.ra.seg_rows);
  printf("W %d H %d bands %d: static seg_rows %d blocks %d; slots %d (%d/CU)\n", W, H,
         w.ra.bands, w.ra.seg_rows, w.ra.waves, slots, per_cu);

  int *heads, *dqb, *dqc;
  Item *ditems;
  unsigned long long *ts;
  CK(hipMalloc(&heads, kXcds * sizeof(int)));
  CK(hipMalloc(&dqb, kXcds * sizeof(int)));
  CK(hipMalloc(&dqc, kXcds * sizeof(int)));
  CK(hipMalloc(&ditems, maxslots * sizeof(Item)));
  CK(hipMalloc(&ts, 2 * slots * sizeof(unsigned long long)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int rate_khz = 0;
  CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));

  auto time_static = [&]() {
    float best = 1e30f, sum = 0.0f;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL((k_warp_iter<M, 0, BW, 1, NC>), dim3(w.ra.waves), dim3(64 * NC + BW), 0, 0, w);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
      if (r) sum += ms;
    }
    printf("static k_warp_iter          : best %6.1f us  mean %6.1f us\n", 1e3f * best,
           1e3f * sum / (reps - 1));
    return best;
  };
  auto time_dyn = [&](int S1, int S2, float ref) {
    std::vector<Item> items;
    std::vector<int> qb, qc;
    const int nblk = slots / kXcds;
    make_items(H, w.ra.bands, nblk, S1, S2, items, qb, qc);
    if ((int)items.size() > maxslots) return;
    long rows = 0;
    for (const Item &it : items) rows += it.ye - it.ys;
    if (rows != (long)H * w.ra.bands) {
      printf("item rows %ld != %ld\n", rows, (long)H * w.ra.bands);
      exit(1);
    }
    CK(hipMemcpy(ditems, items.data(), items.size() * sizeof(Item), hipMemcpyHostToDevice));
    CK(hipMemcpy(dqb, qb.data(), kXcds * sizeof(int), hipMemcpyHostToDevice));
    CK(hipMemcpy(dqc, qc.data(), kXcds * sizeof(int), hipMemcpyHostToDevice));
    float best = 1e30f, sum = 0.0f;
    for (int r = 0; r < reps; ++r) {
      CK(hipMemset(heads, 0, kXcds * sizeof(int)));
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_dyn, dim3(slots), dim3(64 * NC + BW), 0, 0, w, ditems, dqb, dqc, heads, ts);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
      if (r) sum += ms;
    }
    std::vector<unsigned long long> t(2 * slots);
    CK(hipMemcpy(t.data(), ts, t.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull, t1 = 0;
    std::vector<double> en;
    for (int i = 0; i < slots; ++i) t0 = std::min(t0, t[2 * i]);
    for (int i = 0; i < slots; ++i) {
      t1 = std::max(t1, t[2 * i + 1]);
      en.push_back((t[2 * i + 1] - t0) * 1e3 / rate_khz);
    }
    std::sort(en.begin(), en.end());
    printf("dynamic S1 %4d S2 %4d (%5zu items): best %6.1f us  mean %6.1f us  (%+5.1f %%)  "
           "block end p10 %.1f p50 %.1f max %.1f us\n",
           S1, S2, items.size(), 1e3f * best, 1e3f * sum / (reps - 1), 100.0 * (best / ref - 1.0),
           en[en.size() / 10], en[en.size() / 2], en.back());
  };
  // alternate static and dynamic schedules twice, so clock drift shows
  for (int round = 0; round < 2; ++round) {
    const float ref = time_static();
    const int per = (int)((long)H * w.ra.bands / kXcds / (slots / kXcds));   // rows per block
    time_dyn(w.ra.seg_rows, w.ra.seg_rows, ref);   // the static cut, handed out dynamically
    time_dyn(per / 2, per / 2, ref);
    time_dyn(per / 4, per / 4, ref);
    time_dyn(per * 8 / 10, std::max(8, per / 8), ref);
    time_dyn(per * 7 / 10, std::max(8, per / 6), ref);
    time_dyn(per * 9 / 10, std::max(8, per / 10), ref);
    time_dyn(per * 6 / 10, std::max(8, per / 4), ref);
  }
  return 0;
}
