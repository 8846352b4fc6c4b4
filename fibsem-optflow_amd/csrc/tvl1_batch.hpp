// tvl1_batch.hpp — batched kernels of the MI355X TV-L1 engine: one launch works on up to
// kBatchMax same-size pairs (tvl1_calc_batch).
//
// The production workload is not one 6144x4096 pair but two 3072x100 ROI strips per slice
// pair (gen_cross_file_list.py top/bottom ROIs at scale 0.5, nscales 10 -> 9
// levels, warps 5).  One such solve is ~400 launches of a few microseconds each on levels
// of 8.8 K - 307 K px: kernel dispatch, not the GPU, sets its pace.  These kernels give
// every launch a pair dimension (blockIdx.z or .y -> pair b) so a batch of strips shares
// each dispatch.  Per pair, plane X of level s lives at X + b * (pair stride of the plane)
// in a batch arena; which of the two u / p buffer sets is current, whether the pass ends
// in a residual check and whether p is still 0 are per-pair bits in the kernel arguments
// (BatchSel), because pairs leave a warp's iteration loop at different iterations.
//
// The arithmetic is the single-pair kernels' (warp_ring_body, warp_iter_body, roll_body,
// resize_px), so every pair's flow is bit-identical to oracle/.
#pragma once

#include <cfloat>

namespace tvl1k {

constexpr int kBatchMax = 256;

struct BatchMask {           // one bit per pair of a chunk
  uint64_t w[kBatchMax / 64];
  __host__ __device__ int test(int b) const { return (int)((w[b >> 6] >> (b & 63)) & 1u); }
  __host__ void set(int b) { w[b >> 6] |= 1ull << (b & 63); }
  __host__ void clear(int b) { w[b >> 6] &= ~(1ull << (b & 63)); }
  __host__ void flip(int b) { w[b >> 6] ^= 1ull << (b & 63); }
};

struct BatchSel {            // the pairs a launch works on, passed by value
  int n;                     // number of entries in idx
  uint8_t idx[kBatchMax];    // pair indices
  BatchMask ubit, pbit;      // per pair: current u set / p set (0 or 1)
  BatchMask cerr, pzero;     // per pair: the pass ends in a residual check / p == 0
  BatchMask storec;          // kb_warp_iter: per pair, store the warp constants to HBM
};

__device__ __forceinline__ int bsel_bit(const BatchMask &m, int b) { return m.test(b); }

// K1 convertTo for both frames of every pair: blockIdx.z = 2 * pair + frame.
TVL1_PLAIN __global__ void kb_convert(const uint8_t *__restrict__ I0, size_t p0, size_t s0,
                           const uint8_t *__restrict__ I1, size_t p1, size_t s1,
                           float *__restrict__ d0, float *__restrict__ d1, int W, int H, int P,
                           size_t ps) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= W || y >= H) return;
  const int b = blockIdx.z >> 1;
  if ((blockIdx.z & 1) == 0)
    d0[b * ps + (size_t)y * P + x] = (float)I0[b * s0 + (size_t)y * p0 + x];
  else
    d1[b * ps + (size_t)y * P + x] = (float)I1[b * s1 + (size_t)y * p1 + x];
}

// K2 pyramid step for both frames of every pair (blockIdx.z = 2 * pair + frame).
template <bool C>
__global__ void kb_resize_down2(const float *__restrict__ a0, const float *__restrict__ a1,
                                int sw, int sh, int sp, size_t sps, float *__restrict__ b0,
                                float *__restrict__ b1, int dw, int dh, int dp, size_t dps,
                                float fx, float fy) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= dw || y >= dh) return;
  const int b = blockIdx.z >> 1;
  const float *src = ((blockIdx.z & 1) == 0 ? a0 : a1) + b * sps;
  float *dst = ((blockIdx.z & 1) == 0 ? b0 : b1) + b * dps;
  dst[(size_t)y * dp + x] = resize_px<C>(src, sw, sh, sp, x, y, fx, fy);
}

// K5 as k_warp_ring's streaming gather (64-px bands, LDS window ring of I1 / I1x / I1y
// built from I1) on each selected pair (blockIdx.y = entry of sel).
struct BatchRing {
  WarpRingArgs wa;           // geometry (bands, seg_rows, waves per pair); pointers set per pair
  const float *I0, *I1;      // level s images of pair 0 (pair stride ips)
  const float *U[2][2];      // u sets (pair stride ps)
  float *C[3];
  size_t ips, ps;
  BatchSel sel;
};
template <int M, int NW, int FM>
__global__ __launch_bounds__(64 * NW) void kb_warp_ring(BatchRing br) {
  __shared__ float ring[warp_ring_rows<M, NW>() * ring_pitch(64 + 2 * ring_mx<M>())];
  const int b = __builtin_amdgcn_readfirstlane(br.sel.idx[blockIdx.y]);   // uniform: SGPR descriptors
  WarpRingArgs a = br.wa;
  const int us = bsel_bit(br.sel.ubit, b);
  a.I0 = br.I0 + b * br.ips;
  a.I1 = br.I1 + b * br.ips;
  a.u1 = br.U[us][0] + b * br.ps;
  a.u2 = br.U[us][1] + b * br.ps;
  a.I1wx = br.C[0] + b * br.ps;
  a.I1wy = br.C[1] + b * br.ps;
  a.rho = br.C[2] + b * br.ps;
  const int wid = __builtin_amdgcn_readfirstlane(xcd_chunk(blockIdx.x, gridDim.x));
  if (wid >= a.waves) return;
  warp_ring_body<M, NW, FM>(a, wid, ring);
}

// K5 + the warp's first pass (2 iterations ending in the first check) fused, as
// k_warp_iter (warp_iter_body; NC consumer wavefronts), on each selected pair (blockIdx.y =
// entry of sel).  The warp constants go to HBM only for the pairs in sel.storec -- those
// predicted to need later passes (a level's first warp, or a pair whose previous warp ran
// past its first check), as k_warp_iter's store_c; a pair that continues without them is
// re-gathered by kb_warp_ring after the check.
struct BatchWI {
  WarpIterArgs w;            // geometry and scalars; pointers set per pair
  const float *I0, *I1;      // level s images of pair 0 (pair stride ips)
  float *U[2][2];
  float *Pp[2][4];
  float *C[3];
  size_t ips, ps;
  double *partials;
  int nblk;
  BatchSel sel;
};
template <int M, int FM, int NC = 2>
__global__ __launch_bounds__(64 * NC + 128) void kb_warp_iter(BatchWI bw) {
  __shared__ float ring[wi_rows<M>() * ring_pitch(wi_ww<M, 128>())];
  __shared__ float cring[2 * 5 * 128];
  __shared__ float hring[NC == 2 ? 2 * kWiH * 128 : 1];
  const int b = __builtin_amdgcn_readfirstlane(bw.sel.idx[blockIdx.y]);   // uniform: SGPR descriptors
  WarpIterArgs w = bw.w;
  IterArgs &a = w.ra.it;
  {
    const size_t o = b * bw.ps;
    const int us = bsel_bit(bw.sel.ubit, b), qs = bsel_bit(bw.sel.pbit, b);
    a.u1s = bw.U[us][0] + o;
    a.u2s = bw.U[us][1] + o;
    a.u1d = bw.U[us ^ 1][0] + o;
    a.u2d = bw.U[us ^ 1][1] + o;
    a.p11s = bw.Pp[qs][0] + o;
    a.p12s = bw.Pp[qs][1] + o;
    a.p21s = bw.Pp[qs][2] + o;
    a.p22s = bw.Pp[qs][3] + o;
    a.p11d = bw.Pp[qs ^ 1][0] + o;
    a.p12d = bw.Pp[qs ^ 1][1] + o;
    a.p21d = bw.Pp[qs ^ 1][2] + o;
    a.p22d = bw.Pp[qs ^ 1][3] + o;
    a.I1wx = bw.C[0] + o;
    a.I1wy = bw.C[1] + o;
    a.rho = bw.C[2] + o;
    a.calc_err = 1;
    a.p_zero = bsel_bit(bw.sel.pzero, b);
    a.partials = bw.partials + (size_t)b * bw.nblk;
    w.I0 = bw.I0 + b * bw.ips;
    w.I1 = bw.I1 + b * bw.ips;
    w.store_c = bsel_bit(bw.sel.storec, b);
    RollBufs &B = w.ra.b;   // group geometry set by the host
    B.c = a.I1wx;
    B.us = a.u1s;
    B.ud = a.u1d;
    B.ps = a.p11s;
    B.pd = a.p11d;
  }
  const int wid = __builtin_amdgcn_readfirstlane(xcd_chunk(blockIdx.x, gridDim.x));
  if (wid >= w.ra.waves) return;
  warp_iter_body<M, FM, 128, 0, NC>(w, wid, ring, cring, hring);
}

// K6+K8(+K7 partials): one pass of K iterations as a k_iterate_roll<false, K, PX> wavefront
// pipeline on each selected pair (blockIdx.y = entry of sel, 4 wavefronts per block): for
// strips the column bands walk all rows of the level in one segment, so the halo recompute
// is 2K rows and 2 halo px per band (64x32 blocked regions recomputed 1.5-1.8x).  Residual partials of pair b at partials + b * nblk (one per wave).
struct BatchRoll {
  RollArgs ra;               // geometry, l_t, theta, taut (plane pointers set per pair)
  float *U[2][2];
  float *Pp[2][4];
  const float *C[3];
  size_t ps;
  double *partials;
  int nblk;
  BatchSel sel;
};
template <int K, int PX, int FM>
__global__ __launch_bounds__(256) void kb_iterate_roll(BatchRoll br) {
  constexpr bool LDSR = roll_lds_on<false, K, PX>();
  __shared__ float lds[LDSR ? 4 * kRollLdsWave : 1];
  const int b = br.sel.idx[blockIdx.y];
  RollArgs ra = br.ra;
  IterArgs &a = ra.it;
  {
    const size_t o = b * br.ps;
    const int us = bsel_bit(br.sel.ubit, b), qs = bsel_bit(br.sel.pbit, b);
    a.u1s = br.U[us][0] + o;
    a.u2s = br.U[us][1] + o;
    a.u1d = br.U[us ^ 1][0] + o;
    a.u2d = br.U[us ^ 1][1] + o;
    a.p11s = br.Pp[qs][0] + o;
    a.p12s = br.Pp[qs][1] + o;
    a.p21s = br.Pp[qs][2] + o;
    a.p22s = br.Pp[qs][3] + o;
    a.p11d = br.Pp[qs ^ 1][0] + o;
    a.p12d = br.Pp[qs ^ 1][1] + o;
    a.p21d = br.Pp[qs ^ 1][2] + o;
    a.p22d = br.Pp[qs ^ 1][3] + o;
    a.I1wx = br.C[0] + o;
    a.I1wy = br.C[1] + o;
    a.rho = br.C[2] + o;
    a.calc_err = bsel_bit(br.sel.cerr, b);
    a.p_zero = bsel_bit(br.sel.pzero, b);
    a.partials = br.partials + (size_t)b * br.nblk;
    RollBufs &B = ra.b;   // group geometry set by the host
    B.c = a.I1wx;
    B.us = a.u1s;
    B.ud = a.u1d;
    B.ps = a.p11s;
    B.pd = a.p11d;
  }
  const int wid =
      __builtin_amdgcn_readfirstlane(xcd_chunk(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6));
  if (wid >= ra.waves) return;
  roll_body<false, K, PX, FM, 0, kb_roll_ahead<K, PX>(), LDSR>(
      ra, wid, lds + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * (LDSR ? kRollLdsWave : 0));
}

// build-only median filter (k_median) of every selected pair's current u set into the
// other set (blockIdx.z = 2 * entry + component)
struct BatchMedian {
  float *U[2][2];
  size_t ps;
  int W, H, P, ksize;
  BatchSel sel;
};
TVL1_PLAIN __global__ void kb_median(BatchMedian w) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= w.W || y >= w.H) return;
  const int b = w.sel.idx[blockIdx.z >> 1], c = blockIdx.z & 1;
  const int us = bsel_bit(w.sel.ubit, b);
  const float *src = w.U[us][c] + b * w.ps;
  const int r = w.ksize / 2;
  float v[25];
  int n = 0;
  for (int dy = -r; dy <= r; ++dy)
    for (int dx = -r; dx <= r; ++dx)
      v[n++] = src[(size_t)imin(imax(y + dy, 0), w.H - 1) * w.P + imin(imax(x + dx, 0), w.W - 1)];
  for (int i = 1; i < n; ++i) {
    const float t = v[i];
    int j = i - 1;
    while (j >= 0 && v[j] > t) {
      v[j + 1] = v[j];
      --j;
    }
    v[j + 1] = t;
  }
  w.U[us ^ 1][c][b * w.ps + (size_t)y * w.P + x] = v[n / 2];
}

// ---- The coarsest level of a batch, one workgroup per pair, entirely on chip (r5).
// The production strip's coarsest level (515 x 17 px at nscales 10) is where a batch spends
// the most per px-iteration: its streaming passes are one wavefront's 21-step walk long,
// recompute 1.4x (8 of every 64 band columns, 4 drained rows of 17) and end in a host-read
// residual check every few iterations -- 89 launches and ~45 host round trips per batch, for
// 204 iterations per pair.  Here one workgroup holds a whole pair's level: lane x
// of the workgroup owns column x, its rows' u and p in registers, the warp constants and I1
// in LDS.  It runs procOneScale's loop for every warp of the level -- warpBackward, then the
// iterations with the residual summed by the workgroup and the stopping rule evaluated on
// chip -- with x-neighbours by DPP inside a wavefront and through LDS across wavefronts, and
// two barriers per iteration.  Nothing is recomputed, nothing goes to HBM between
// iterations, and the host waits once per level.  The arithmetic is warp_gather_fn (taps at
// clamped coordinates, centeredGradient per tap as k_warp_ring's global path),
// estimate_u_px and dual_px with their general border forms: the same operations as the
// streaming kernels, so the same bits.  The residual is summed in double per column (rows
// in order) and over the workgroup in a fixed order; the stopping decisions sit >= 1e-4
// (relative) from their thresholds on every input measured, and the parity
// tests compare every pair's flow and per-warp counts with the oracle bitwise.
constexpr int kSmallR = 17;         // rows per lane: the level's height, at most
constexpr int kSmallWaves = 9;      // 576 lanes, one column each: the level's width, at most
constexpr int kSmallPx = 9000;      // LDS planes of W * H floats: I1 and the three constants

struct BatchSmall {
  const float *I0, *I1;   // the level's images of pair 0 (pair stride ips)
  float *u1, *u2;         // u set written (pair stride ps); the level starts from u = 0
  size_t ips, ps;
  int W, H, P;            // level geometry; P = plane pitch in floats
  int warps, iterations, eps_pos;
  double thr;             // scaledEps = eps^2 * W * H
  IterArgs it;            // l_t, theta, taut (gamma = 0)
  int *warp_iters;        // [pair][warps] iterations each warp ran
  int *checks;            // [pair] residual checks
  BatchSel sel;
};

template <int FM>
__global__ __launch_bounds__(64 * kSmallWaves) void kb_small_level(BatchSmall a) {
  __shared__ float sI1[kSmallPx];
  __shared__ float sC[3][kSmallPx];
  __shared__ float xu[kSmallWaves][2][kSmallR];   // each wavefront's lane 0: u1, u2 (new)
  __shared__ float xp[kSmallWaves][2][kSmallR];   // each wavefront's lane 63: p11, p21
  __shared__ double red[kSmallWaves];
  constexpr int R = kSmallR;
  const int b = a.sel.idx[blockIdx.x];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  const int W = a.W, H = a.H, P = a.P;
  // the padded lanes must share lane W-1's wavefront (the gather is not followed by a
  // barrier): the launch geometry is 64 * ceil(W / 64) threads, nothing else
  if ((int)blockDim.x != 64 * ((W + 63) / 64)) return;
  const int x = threadIdx.x;
  const bool valid = x < W;
  const int xs = imin(x, W - 1);   // lanes past the level's width compute on column W - 1
  const float *I0 = a.I0 + b * a.ips;
  const float *I1 = a.I1 + b * a.ips;
  for (int i = threadIdx.x; i < W * H; i += blockDim.x) {
    const int yy = i / W;
    sI1[i] = I1[(size_t)yy * P + (i - yy * W)];
  }
  float u1[R], u2[R], p11[R], p12[R], p21[R], p22[R];
#pragma unroll
  for (int y = 0; y < R; ++y) u1[y] = u2[y] = p11[y] = p12[y] = p21[y] = p22[y] = 0.0f;
  if (lane == 63)
    for (int y = 0; y < R; ++y) xp[wv][0][y] = xp[wv][1][y] = 0.0f;
  __syncthreads();
  int checks = 0;
  for (int wp = 0; wp < a.warps; ++wp) {
    // K5 warpBackward of this lane's column (+ K3 centeredGradient per tap), constants to LDS.
    // One row per trip of a loop that is not unrolled (one gather's code): row y's u is
    // always u1[0] / u2[0] and the arrays rotate by one row per trip, R trips in all, so
    // they end where they began (register arrays take constant indices only)
    for (int y = 0; y < R; ++y) {
      const float cu1 = u1[0], cu2 = u2[0];
#pragma unroll
      for (int i = 0; i < R - 1; ++i) {
        u1[i] = u1[i + 1];
        u2[i] = u2[i + 1];
      }
      u1[R - 1] = cu1;
      u2[R - 1] = cu2;
      if (y >= H) continue;
      const float wx = (float)xs + cu1;
      const float wy = (float)y + cu2;
      const int fx = tap_floor(wx);
      const int fy = tap_floor(wy);
      float sum = 0.0f, sumx = 0.0f, sumy = 0.0f, wsum = 0.0f;
      warp_gather_fn<FM>(
          [&](int cy, int cx) {
            const int rx = imin(imax(cx, 0), W - 1), ry = imin(imax(cy, 0), H - 1);
            const float *row = sI1 + ry * W;
            const float gx = 0.5f * (row[imin(rx + 1, W - 1)] - row[imax(rx - 1, 0)]);
            const float gyv = 0.5f * (sI1[imin(ry + 1, H - 1) * W + rx] - sI1[imax(ry - 1, 0) * W + rx]);
            return Tap3{row[rx], gx, gyv};
          },
          wx, wy, fx, fy, sum, sumx, sumy, wsum);
      const float coeff = approx(FM) ? __builtin_amdgcn_rcpf(wsum) : recip_rn(wsum);
      const float I1wv = sum * coeff;
      const float I1wxv = sumx * coeff;
      const float I1wyv = sumy * coeff;
      if (valid) {
        sC[0][y * W + x] = I1wxv;
        sC[1][y * W + x] = I1wyv;
        sC[2][y * W + x] = rho_c<FM>(I1wv, I1wxv, I1wyv, cu1, cu2, I0[(size_t)y * P + x]);
      }
    }
    // procOneScale's iterations.  No barrier after the gather: a lane x < W reads only the
    // constants it wrote itself, and a padded lane (x >= W) reads column W-1, written by lane
    // W-1 -- which sits in the same wavefront, because the block is exactly 64 * ceil(W / 64)
    // threads (the launch; checked at kernel entry), and LDS accesses of one wavefront stay
    // in program order
    double error = DBL_MAX, prevError = 0.0;
    int n;
    for (n = 0; error > a.thr && n < a.iterations; ++n) {
      const bool calc = a.eps_pos && (n & 1) && prevError < a.thr;
      // estimateU: u^n = TH(u^{n-1}) + theta div p^{n-1}; p of the left column by DPP, and for
      // lane 0 from the left wavefront's lane 63 (published after the previous iteration)
      double acc = 0.0;
      // the lane's constants' LDS index, advanced by a row per row: opaque per iteration so
      // the compiler does not keep 17 row addresses live across the loop
      int ci = xs;
      asm volatile("" : "+v"(ci));
#pragma unroll
      for (int y = 0; y < R; ++y) {
        if (y >= H) continue;   // (a fixed trip count: fully unrolled)
        float l11 = from_left(p11[y]), l21 = from_left(p21[y]);
        if (lane == 0 && wv > 0) {
          l11 = xp[wv - 1][0][y];
          l21 = xp[wv - 1][1][y];
        }
        const float c0 = sC[0][ci], c1 = sC[1][ci], c2 = sC[2][ci];
        ci += W;
        float n1, n2, n3;
        const int yu = y > 0 ? y - 1 : 0;   // (never a negative register index)
        estimate_u_px<false, FM>(c0, c1, c2, u1[y], u2[y], 0.0f, p11[y], l11, p12[y],
                                 y > 0 ? p12[yu] : 0.0f, p21[y], l21, p22[y],
                                 y > 0 ? p22[yu] : 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, xs, y, a.it,
                                 n1, n2, n3);
        if (calc && valid) acc += (double)residual_px<FM>(u1[y] - n1, u2[y] - n2);
        u1[y] = n1;
        u2[y] = n2;
        __builtin_amdgcn_sched_barrier(0);   // rows one after another: no hoisting, low pressure
      }
      if (calc) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if (lane == 0) red[wv] = acc;
      }
      if (lane == 0) {
#pragma unroll
        for (int y = 0; y < R; ++y) {   // (register arrays: constant indices only)
          if (y >= H) continue;   // (a fixed trip count: fully unrolled)
          xu[wv][0][y] = u1[y];
          xu[wv][1][y] = u2[y];
        }
      }
      __syncthreads();
      if (calc) {   // cuda::sum and the stopping rule, the same double for every lane
        double e = 0.0;
        for (int w = 0; w < nw; ++w) e += red[w];
        error = e;
        prevError = e;
        ++checks;
      } else {
        error = DBL_MAX;
        prevError -= a.thr;
      }
      // estimateDualVariables: u^n of the right column by DPP, and for lane 63 from the right
      // wavefront's lane 0; p updated in place (each row reads only u)
#pragma unroll
      for (int y = 0; y < R; ++y) {
        if (y >= H) continue;   // (a fixed trip count: fully unrolled)
        float r1 = from_right(u1[y]), r2 = from_right(u2[y]);
        if (lane == 63 && wv + 1 < nw) {
          r1 = xu[wv + 1][0][y];
          r2 = xu[wv + 1][1][y];
        }
        const bool has_down = y + 1 < H;
        const float d1 = has_down ? u1[imin(y + 1, R - 1)] : u1[y];
        const float d2 = has_down ? u2[imin(y + 1, R - 1)] : u2[y];
        float q11, q12, q21, q22;
        dual_px<false, false, FM>(u1[y], r1, d1, xs + 1 < W, has_down, a.it.taut, p11[y], p12[y],
                                  q11, q12, a.it.taut_small);
        dual_px<false, false, FM>(u2[y], r2, d2, xs + 1 < W, has_down, a.it.taut, p21[y], p22[y],
                                  q21, q22, a.it.taut_small);
        p11[y] = q11; p12[y] = q12;
        p21[y] = q21; p22[y] = q22;
        __builtin_amdgcn_sched_barrier(0);
      }
      if (lane == 63) {
#pragma unroll
        for (int y = 0; y < R; ++y) {
          if (y >= H) continue;   // (a fixed trip count: fully unrolled)
          xp[wv][0][y] = p11[y];
          xp[wv][1][y] = p21[y];
        }
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) a.warp_iters[(size_t)b * a.warps + wp] = n;
  }
  if (valid) {
#pragma unroll
    for (int y = 0; y < R; ++y) {
      if (y >= H) continue;   // (a fixed trip count: fully unrolled)
      a.u1[b * a.ps + (size_t)y * P + x] = u1[y];
      a.u2[b * a.ps + (size_t)y * P + x] = u2[y];
    }
  }
  if (threadIdx.x == 0) a.checks[b] = checks;
}

// K7 for the selected pairs: fixed-order sum of pair b's n partials (at partials + b * stride)
// into out[b].
TVL1_PLAIN __global__ void kb_reduce(const double *__restrict__ partials, size_t stride, int n,
                                     BatchSel sel, double *__restrict__ out) {
  __shared__ double s[kBlock];
  const int b = sel.idx[blockIdx.x];
  const double *p = partials + (size_t)b * stride;
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += kBlock) acc += p[i];
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int o = kBlock / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[b] = s[0];
}

// K9 flow upsample (u1, u2 scaled by 1/scaleStep) of every pair from its current u set
// into the other one (blockIdx.z = 2 * entry + component).
struct BatchUp {
  float *U[2][2];
  size_t ps;
  int sw, sh, sp, dw, dh, dp;
  float fx, fy, mul;
  BatchSel sel;
};
template <bool C>
__global__ void kb_upsample(BatchUp w) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= w.dw || y >= w.dh) return;
  const int b = w.sel.idx[blockIdx.z >> 1], c = blockIdx.z & 1;
  const int us = bsel_bit(w.sel.ubit, b);
  const float *src = w.U[us][c] + b * w.ps;
  float *dst = w.U[us ^ 1][c] + b * w.ps;
  dst[(size_t)y * w.dp + x] = resize_px<C>(src, w.sw, w.sh, w.sp, x, y, w.fx, w.fy) * w.mul;
}

// K10: every pair's final u set to the caller's flow (pair b at u + b * fstride bytes).
struct BatchOut {
  const float *U[2][2];
  size_t ps;
  int W, H, P;
  float *u, *v;
  size_t fpitch, fstride;
  BatchSel sel;
};
TVL1_PLAIN __global__ void kb_output(BatchOut w) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= w.W || y >= w.H) return;
  const int b = w.sel.idx[blockIdx.z];
  const int us = bsel_bit(w.sel.ubit, b);
  const size_t i = b * w.ps + (size_t)y * w.P + x;
  char *ou = reinterpret_cast<char *>(w.u) + b * w.fstride + (size_t)y * w.fpitch;
  char *ov = reinterpret_cast<char *>(w.v) + b * w.fstride + (size_t)y * w.fpitch;
  reinterpret_cast<float *>(ou)[x] = w.U[us][0][i];
  reinterpret_cast<float *>(ov)[x] = w.U[us][1][i];
}

}  // namespace tvl1k
