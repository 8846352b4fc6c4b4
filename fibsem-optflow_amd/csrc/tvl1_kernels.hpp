// tvl1_kernels.hpp — device kernels of the MI355X TV-L1 engine (gfx950, wave64).
//
// Each kernel restates one stage of the solver the reference calls at
// /root/reference/src/optflow.cpp:518-519 (OpenCV 3.4.1 cv::cuda::OpticalFlowDual_TVL1,
// semantics in SURVEY.md Appendix A; kernel inventory SURVEY 2.1 K1..K12).  In the default
// arithmetic mode (kIEEE: float32, OpenCV's expression order, no FMA contraction -- the
// library is compiled with -ffp-contract=off) the results are identical to oracle/tvl1_oracle.c
// bit for bit.  The data layout and fusion are MI355X-first:
//
//   * every f32 plane is pitched to a multiple of 64 floats (256 B rows);
//   * estimateU (K6) and estimateDualVariables (K8) are fused, and up to 4 iterations run
//     in ONE HBM pass: k_iterate_roll is a wavefront pipeline down a 128- or 256-px column
//     band (x neighbours by DPP, y neighbours in registers, no LDS); k_iterate_tb runs
//     64 x 32 regions in LDS for long passes on small levels;
//   * warpBackward (K5) builds the (I1, I1x, I1y) window from I1 in an LDS ring
//     (k_warp_ring; centeredGradient, K3, per slot), and on large levels it is fused with
//     the warp's first 2-iteration pass (k_warp_iter: producer and consumer wavefronts);
//   * the state (u, p) ping-pongs between two buffer sets (Jacobi), so bands and regions
//     never race on their halos;
//   * grad = I1wx^2 + I1wy^2 is recomputed from I1wx, I1wy (same operations as K5) instead
//     of being stored and re-read every iteration;
//   * the residual sum (K7) is fused into the iteration as per-wavefront / per-block double
//     partials reduced by one tiny kernel in a fixed order (deterministic).
//   * k_iterate (one iteration per launch) and k_warp_img (tiled, 64-bit addressing) serve
//     the parameter sets and plane sizes the streaming kernels do not take (taut < 0,
//     profile 1, planes >= 2 GiB).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// The non-template kernels are defined once, in tvl1_engine.hip's translation unit.
// tvl1_passes.hip includes these headers for its template instantiations only: there they
// are declared as never-instantiated templates, so that unit emits no code for them.
#ifdef TVL1_PASSES_TU
#define TVL1_PLAIN template <int TVL1_PASSES_TU_UNUSED = 0>
#else
#define TVL1_PLAIN
#endif

namespace tvl1k {

constexpr int kWave = 64;
constexpr int kBlock = 256;                 // 4 waves
constexpr int kSegPx = (kWave - 2) * 4;     // 248 useful px per wave (lanes 1..62)
constexpr float kFltEps = 1.1920928955078125e-07f;  // numeric_limits<float>::epsilon()

__device__ __forceinline__ int imin(int a, int b) { return a < b ? a : b; }
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }

// RN(1/d): v_rcp_f32 (1 ulp) and one Newton step.  Equal to IEEE 1.0f / d for every
// significand of the binades 2^-23 .. 2^40 (and 2^50, 2^99, 2^100, 2^120, 2^125), checked
// exhaustively on gfx950 by tools/div_check.hip test A.  warpBackward's coeff = 1 / wsum has
// wsum ~ 1 (the Keys weights sum to 1), well inside.
__device__ __forceinline__ float recip_rn(float d) {
  const float r = __builtin_amdgcn_rcpf(d);
  const float e = __builtin_fmaf(-d, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}

// Arithmetic mode of the solver kernels (tvl1_params.fast_math; the FM template argument):
//   kIEEE (0)  IEEE float32, no contraction: bit-identical to oracle/ (the default);
//   kFast (1)  the reference build's CUDA_FAST_MATH (singularity/optflow.def:33-34): a*b + c
//              contracted as nvcc does, division and sqrt approximated (v_rcp_f32 /
//              v_sqrt_f32, 1 ulp);
//   kFma  (2)  nvcc's default -fmad=true contraction alone, IEEE division and sqrt:
//              bit-identical to oracle/'s fma mode.
// The contraction rule (NVPTX's DAG combine, which fuses aggressively): an add or subtract
// with a multiply operand becomes one fma, the LEFT operand's product when both are
// products (a*b + c*d -> fma(a, b, c*d)).  Each site below says which expression it fuses.
constexpr int kIEEE = 0, kFast = 1, kFma = 2;
__host__ __device__ constexpr bool contracts(int m) { return m != kIEEE; }
__host__ __device__ constexpr bool approx(int m) { return m == kFast; }

// XCD-aware tile order (speed only, never correctness).  The dispatcher deals
// workgroups round-robin over the 8 XCDs (MI355X_MICROARCH: blocks b and b+8 share an
// XCD), each with its own 4 MiB L2.  Give every XCD a contiguous run of tile slots and
// walk the slots in 8-tile-wide column bands, row by row, so a tile's x- and
// y-neighbours (which re-read its halo lines) run on the same XCD shortly after it.
constexpr int kXcds = 8, kBand = 8;
__device__ __forceinline__ void tile_of_block(int bid, int nblocks, int tiles_x, int tiles_y,
                                              int &bx, int &by) {
  const int q = nblocks / kXcds, rem = nblocks % kXcds;
  const int xcd = bid % kXcds, k = bid / kXcds;
  const int slot = xcd * q + imin(xcd, rem) + k;
  const int full = tiles_x / kBand;
  const int band = imin(slot / (kBand * tiles_y), full);
  const int width = band < full ? kBand : tiles_x - full * kBand;
  const int in_band = slot - band * kBand * tiles_y;
  by = in_band / width;
  bx = band * kBand + (in_band - by * width);
}

// XCD-contiguous block order: the blocks the hardware sends to one XCD (b % 8) get one
// contiguous run of logical indices, so neighbouring bands share that XCD's L2.
__device__ __forceinline__ int xcd_chunk(int b, int n) {
  const int q = n / kXcds, rem = n % kXcds;
  const int x = b % kXcds, i = b / kXcds;
  return x * q + imin(x, rem) + i;
}

// Buffer access to a plane: scalar descriptor (base, size in bytes), the row in the
// scalar offset, the lane's column as one 32-bit VGPR byte offset.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const float *p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p), 0, (int)bytes, 0x00020000);
}
constexpr unsigned kOOB = 0x7ffffff0u;   // byte offset beyond every plane: store dropped
#ifndef TVL1_STORE_AUX
#define TVL1_STORE_AUX 2
#endif
constexpr int kWarpStoreAux = TVL1_STORE_AUX;   // cache policy of warp constant stores (2 = nt)
template <int AUX = 0>
__device__ __forceinline__ void bstore(float *p, unsigned bytes, unsigned voff, unsigned soff, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), plane_rsrc(p, bytes), (int)voff, (int)soff, AUX);
}
// PX consecutive floats of a plane (4-, 8- or 16-byte store)
template <int PX>
__device__ __forceinline__ void bstorev(float *p, unsigned bytes, unsigned voff, const float (&v)[PX],
                                        unsigned soff = 0) {
  if constexpr (PX == 1) {
    bstore(p, bytes, voff, soff, v[0]);
  } else if constexpr (PX == 4) {
    using T = decltype(__builtin_amdgcn_raw_buffer_load_b128(plane_rsrc(p, bytes), 0, 0, 0));
    T t;
    __builtin_memcpy(&t, v, 16);
    __builtin_amdgcn_raw_buffer_store_b128(t, plane_rsrc(p, bytes), (int)voff, (int)soff, 0);
  } else {
    using T = decltype(__builtin_amdgcn_raw_buffer_load_b64(plane_rsrc(p, bytes), 0, 0, 0));
    T t;
    __builtin_memcpy(&t, v, 8);
    __builtin_amdgcn_raw_buffer_store_b64(t, plane_rsrc(p, bytes), (int)voff, (int)soff, 0);
  }
}
// PX consecutive floats of a plane (4-, 8- or 16-byte load)
template <int PX>
__device__ __forceinline__ void bload(float (&d)[PX], const float *p, unsigned bytes, unsigned voff,
                                      unsigned soff) {
  if constexpr (PX == 1) {
    d[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(plane_rsrc(p, bytes), (int)voff, (int)soff, 0));
  } else if constexpr (PX == 4) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(plane_rsrc(p, bytes), (int)voff, (int)soff, 0);
    static_assert(sizeof(v) == 16, "b128 load");
    __builtin_memcpy(d, &v, 16);
  } else {
    static_assert(PX == 2, "1, 2 or 4 px per lane");
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(plane_rsrc(p, bytes), (int)voff, (int)soff, 0);
    static_assert(sizeof(v) == 8, "b64 load");
    __builtin_memcpy(d, &v, 8);
  }
}

// ---------------------------------------------------------------- K1 convert
// GpuMat::convertTo(CV_32F, 1.0) for both frames (blockIdx.z selects the frame).
TVL1_PLAIN __global__ void k_convert_u8(const uint8_t *__restrict__ s0, size_t sp0,
                             const uint8_t *__restrict__ s1, size_t sp1,
                             float *__restrict__ d0, float *__restrict__ d1, int W, int H,
                             int P) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= W || y >= H) return;
  if (blockIdx.z == 0)
    d0[(size_t)y * P + x] = (float)s0[(size_t)y * sp0 + x];
  else
    d1[(size_t)y * P + x] = (float)s1[(size_t)y * sp1 + x];
}

// [A.1] for CV_32FC1 inputs: convertTo(CV_32F, 255.0) = src * 255 + 0 (nvcc contracts it
// to fma(255, src, 0): the same value, -0 becomes +0 either way).  Pitches in bytes.
TVL1_PLAIN __global__ void k_convert_f32(const float *__restrict__ s0, size_t sp0,
                              const float *__restrict__ s1, size_t sp1,
                              float *__restrict__ d0, float *__restrict__ d1, int W, int H,
                              int P) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= W || y >= H) return;
  const float *s = blockIdx.z == 0 ? (const float *)((const char *)s0 + (size_t)y * sp0)
                                   : (const float *)((const char *)s1 + (size_t)y * sp1);
  (blockIdx.z == 0 ? d0 : d1)[(size_t)y * P + x] = s[x] * 255.0f + 0.0f;
}

// ---------------------------------------------------------------- K2 / K9 resize
// cuda::resize INTER_LINEAR: corner-aligned, src = dst * f, +1 taps clamped.
// C (contracting modes): the tap weights' differences take the product src_x = dst_x * fx
// unrounded (x2 - src_x -> fma(-dst_x, fx, x2), src_x - x1 -> fma(dst_x, fx, -x1); the floor
// uses the rounded product) and out + src * w -> fma(src, w, out).
template <bool C = false>
__device__ __forceinline__ float resize_px(const float *__restrict__ src, int sw, int sh,
                                           int sp, int dx, int dy, float fx, float fy) {
  const float dxf = (float)dx, dyf = (float)dy;
  const float src_x = dxf * fx;
  const float src_y = dyf * fy;
  const int x1 = (int)floorf(src_x);
  const int y1 = (int)floorf(src_y);
  const int x2 = x1 + 1;
  const int y2 = y1 + 1;
  const int x2r = imin(x2, sw - 1);
  const int y2r = imin(y2, sh - 1);
  const float ax = C ? __builtin_fmaf(-dxf, fx, (float)x2) : (float)x2 - src_x;
  const float bx = C ? __builtin_fmaf(dxf, fx, -(float)x1) : src_x - (float)x1;
  const float ay = C ? __builtin_fmaf(-dyf, fy, (float)y2) : (float)y2 - src_y;
  const float by = C ? __builtin_fmaf(dyf, fy, -(float)y1) : src_y - (float)y1;
  const float t00 = src[(size_t)y1 * sp + x1], t01 = src[(size_t)y1 * sp + x2r];
  const float t10 = src[(size_t)y2r * sp + x1], t11 = src[(size_t)y2r * sp + x2r];
  float out = 0.0f;
  if (C) {
    out = __builtin_fmaf(t00, ax * ay, out);
    out = __builtin_fmaf(t01, bx * ay, out);
    out = __builtin_fmaf(t10, ax * by, out);
    out = __builtin_fmaf(t11, bx * by, out);
  } else {
    out = out + t00 * (ax * ay);
    out = out + t01 * (bx * ay);
    out = out + t10 * (ax * by);
    out = out + t11 * (bx * by);
  }
  return out;
}

// Pyramid step for both frames at once (blockIdx.z selects the frame).
template <bool C>
__global__ void k_resize_down2(const float *__restrict__ a0, const float *__restrict__ a1,
                               int sw, int sh, int sp, float *__restrict__ b0,
                               float *__restrict__ b1, int dw, int dh, int dp, float fx,
                               float fy) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= dw || y >= dh) return;
  const float *src = blockIdx.z == 0 ? a0 : a1;
  float *dst = blockIdx.z == 0 ? b0 : b1;
  dst[(size_t)y * dp + x] = resize_px<C>(src, sw, sh, sp, x, y, fx, fy);
}

// Flow upsample to the next finer level + cuda::multiply(1/scaleStep) on u1, u2
// (u3 is resized but not scaled, as in calcImpl).  blockIdx.z = component.
template <bool C>
__global__ void k_upsample(const float *__restrict__ s1, const float *__restrict__ s2,
                           const float *__restrict__ s3, int sw, int sh, int sp,
                           float *__restrict__ d1, float *__restrict__ d2,
                           float *__restrict__ d3, int dw, int dh, int dp, float fx, float fy,
                           float mul) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= dw || y >= dh) return;
  const int c = blockIdx.z;
  const float *src = c == 0 ? s1 : (c == 1 ? s2 : s3);
  float *dst = c == 0 ? d1 : (c == 1 ? d2 : d3);
  const float r = resize_px<C>(src, sw, sh, sp, x, y, fx, fy);
  dst[(size_t)y * dp + x] = c < 2 ? r * mul : r;
}

// ---------------------------------------------------------------- K3 gradient
// centeredGradient of I1, written interleaved (I1, I1x, I1y, 0) for the K5 gather.
TVL1_PLAIN __global__ void k_gradient(const float *__restrict__ I, int W, int H, int P,
                           float4 *__restrict__ G) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= W || y >= H) return;
  const float *row = I + (size_t)y * P;
  const float c = row[x];
  const float gx = 0.5f * (row[imin(x + 1, W - 1)] - row[imax(x - 1, 0)]);
  const float gy = 0.5f * (I[(size_t)imin(y + 1, H - 1) * P + x] - I[(size_t)imax(y - 1, 0) * P + x]);
  G[(size_t)y * P + x] = make_float4(c, gx, gy, 0.0f);
}

// ---------------------------------------------------------------- profile 1
// OpenCV's CPU cv::DualTVL1OpticalFlow schedule (tvl1_params.profile = 1; restated in
// oracle/tvl1_oracle_dualtvl1.c, whose file:line-free notes list what is recalled).
//
// cv::resize INTER_LINEAR on CV_32F: half-pixel source coordinate (double, cast to
// float), x clamped to the edge columns (f := 0, the last column a single tap), the two
// rows clamped but their weights kept; or the exact-2x INTER_AREA fast path.  Planes by
// blockIdx.z (< nmul of them are then multiplied by mul: cv::multiply(u, 1/scaleStep)).
TVL1_PLAIN __global__ void k_resize_hp(const float *__restrict__ s0, const float *__restrict__ s1,
                            const float *__restrict__ s2, int sw, int sh, int sp,
                            float *__restrict__ d0, float *__restrict__ d1,
                            float *__restrict__ d2, int dw, int dh, int dp, double scale_x,
                            double scale_y, int area_fast, int nmul, float mul) {
  const int dx = blockIdx.x * 64 + threadIdx.x;
  const int dy = blockIdx.y * 4 + threadIdx.y;
  if (dx >= dw || dy >= dh) return;
  const int c = blockIdx.z;
  const float *src = c == 0 ? s0 : (c == 1 ? s1 : s2);
  float *dst = c == 0 ? d0 : (c == 1 ? d1 : d2);
  float r;
  if (sw == dw && sh == dh) {
    r = src[(size_t)dy * sp + dx];
  } else if (area_fast) {
    const float *S = src + (size_t)(2 * dy) * sp + 2 * dx;
    r = (S[0] + S[1] + S[sp] + S[sp + 1]) * 0.25f;
  } else {
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    const float b0 = 1.f - fy, b1 = fy;
    const int r0 = imin(imax(sy, 0), sh - 1), r1 = imin(imax(sy + 1, 0), sh - 1);
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) fx = 0.f, sx = 0;
    const bool single = sx + 1 >= sw;
    if (sx >= sw - 1) fx = 0.f, sx = sw - 1;
    const float a0 = 1.f - fx, a1 = fx;
    const float *S0 = src + (size_t)r0 * sp, *S1 = src + (size_t)r1 * sp;
    const float t0 = single ? S0[sx] * 1.0f : S0[sx] * a0 + S0[sx + 1] * a1;
    const float t1 = single ? S1[sx] * 1.0f : S1[sx] * a0 + S1[sx + 1] * a1;
    r = t0 * b0 + t1 * b1;
  }
  dst[(size_t)dy * dp + dx] = c < nmul ? r * mul : r;
}

// remap(I1 / I1x / I1y, x + u1, y + u2, INTER_CUBIC, BORDER_CONSTANT 0) + calcGradRho:
// the map rounded to 1/32 px (cvRound), the Keys a = -0.75 weights of interpolateCubic at
// the two 1/32 fractions (the float table entries, recomputed with the same operations),
// 4x4 taps from G = (I1, I1x, I1y); a tap outside the image adds nothing.
__device__ __forceinline__ void cubic_tab_entry(int i, float (&t)[4]) {
  const float A = -0.75f;
  const float x = (float)i * (1.f / 32);
  t[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
  t[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
  t[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
  t[3] = 1.f - t[0] - t[1] - t[2];
}
__device__ __forceinline__ int round_map(float v) {
  if (!(v > -2147483648.f && v < 2147483648.f)) return (int)0x80000000u;
  return (int)rintf(v);
}
TVL1_PLAIN __global__ void k_remap_cubic(const float *__restrict__ I0, const float4 *__restrict__ G,
                              const float *__restrict__ u1, const float *__restrict__ u2,
                              int W, int H, int P, float *__restrict__ I1wx,
                              float *__restrict__ I1wy, float *__restrict__ rho) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= W || y >= H) return;
  const size_t i = (size_t)y * P + x;
  const float u1v = u1[i], u2v = u2[i];
  const float X = (float)x + u1v, Y = (float)y + u2v;
  const int ix = round_map(X * 32.f), iy = round_map(Y * 32.f);
  const int sx = imin(imax(ix >> 5, -32768), 32767) - 1;
  const int sy = imin(imax(iy >> 5, -32768), 32767) - 1;
  float ty[4], tx[4];
  cubic_tab_entry(iy & 31, ty);
  cubic_tab_entry(ix & 31, tx);
  float sum = 0.0f, sumx = 0.0f, sumy = 0.0f;
  if ((unsigned)sx < (unsigned)imax(W - 3, 0) && (unsigned)sy < (unsigned)imax(H - 3, 0)) {
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
      const float4 *r = G + (size_t)(sy + k1) * P + sx;
      const float w0 = ty[k1] * tx[0], w1 = ty[k1] * tx[1], w2 = ty[k1] * tx[2],
                  w3 = ty[k1] * tx[3];
      const float4 g0 = r[0], g1 = r[1], g2 = r[2], g3 = r[3];
      const float a = g0.x * w0 + g1.x * w1 + g2.x * w2 + g3.x * w3;
      const float b = g0.y * w0 + g1.y * w1 + g2.y * w2 + g3.y * w3;
      const float c = g0.z * w0 + g1.z * w1 + g2.z * w2 + g3.z * w3;
      if (k1 == 0) {
        sum = a; sumx = b; sumy = c;
      } else {
        sum += a; sumx += b; sumy += c;
      }
    }
  } else if (!(sx >= W || sx + 4 <= 0 || sy >= H || sy + 4 <= 0)) {
    sum = sumx = sumy = 0.0f * 1.0f;
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
      const int yi = sy + k1;
      if (yi < 0 || yi >= H) continue;
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) {
        const int xj = sx + k2;
        if (xj < 0 || xj >= W) continue;
        const float w = ty[k1] * tx[k2];
        const float4 g = G[(size_t)yi * P + xj];
        sum += (g.x - 0.0f) * w;
        sumx += (g.y - 0.0f) * w;
        sumy += (g.z - 0.0f) * w;
      }
    }
  }
  // calcGradRho (grad = I1wx^2 + I1wy^2 is recomputed by the iteration kernels)
  I1wx[i] = sumx;
  I1wy[i] = sumy;
  rho[i] = sum - sumx * u1v - sumy * u2v - I0[i];
}

// ---------------------------------------------------------------- K5 warp
// Window geometry of k_warp_img (the tiled, 64-bit-addressed warpBackward for planes the
// 32-bit buffer offsets of the streaming kernels cannot address): a 64 x 16 px tile and
// the (I1, I1x, I1y) window it can reach with |u| <= kWarpHalo - 2.
constexpr int kWarpTW = 64, kWarpTH = 16, kWarpHalo = 6;
constexpr int kWarpWW = kWarpTW + 2 * kWarpHalo, kWarpWH = kWarpTH + 2 * kWarpHalo;

// floor() of a tap coordinate as an int with no overflow: coordinates are clamped to
// +-2^24 first (every float beyond that is an integer and every tap of it clamps to
// the image border anyway), so fx - 1 .. fx + 2 never overflow.  NaN maps to 0.
__device__ __forceinline__ int tap_floor(float w) {
  const float c = fminf(fmaxf(w, -16777216.0f), 16777216.0f);
  return (int)floorf(c == c ? c : 0.0f);
}

// Keys kernel pieces: |t| <= 1 and 1 < |t| < 2 (OpenCV `cubic`).
__device__ __forceinline__ float cubic_in(float x) {
  x = fabsf(x);
  return x * x * (1.5f * x - 2.5f) + 1.0f;
}
__device__ __forceinline__ float cubic_out(float x) {
  x = fabsf(x);
  return x * (x * (-0.5f * x + 2.5f) - 4.0f) + 2.0f;
}

// Fixed 4x4 form of OpenCV's tap loop (cy in [ceil(wy-2), floor(wy+2)], cx likewise):
// every tap it visits outside cx in [floor(wx)-1, floor(wx)+2] has weight exactly 0
// (|t| = 2), and inside that range the tap distances are t0 in [1,2), t1 in [0,1),
// t2 in [-1,0), t3 in [-2,-1) -- so taps 1,2 always take the |t|<=1 piece and taps
// 0,3 the outer piece; at the two ends (t0 = 1, |t3| = 2) both pieces evaluate to
// exactly 0.0f.  Summation order (rows outer, columns inner, ascending) and the
// weight product cubic(wx-cx) * cubic(wy-cy) are unchanged, so the result is
// bit-identical to the reference loop while being branch-free and unrollable.
// The 4x4 taps: tap(cy, cx) -> (I1, I1x, I1y) at that (unclamped) tap coordinate.
struct Tap3 {
  float x, y, z;
};
// Contracting modes: cubic's polynomials (x*x*t + 1 -> fma(x*x, t, 1), t = 1.5x - 2.5 ->
// fma(1.5, x, -2.5); likewise the outer piece) and the accumulations sum + w*I -> fma.
__device__ __forceinline__ float cubic_in_fm(float x) {
  x = fabsf(x);
  return __builtin_fmaf(x * x, __builtin_fmaf(1.5f, x, -2.5f), 1.0f);
}
__device__ __forceinline__ float cubic_out_fm(float x) {
  x = fabsf(x);
  return __builtin_fmaf(x, __builtin_fmaf(x, __builtin_fmaf(-0.5f, x, 2.5f), -4.0f), 2.0f);
}
template <int FM = 0, class TapF>
__device__ __forceinline__ void warp_gather_fn(TapF tap, float wx, float wy, int fx, int fy,
                                               float &sum, float &sumx, float &sumy, float &wsum) {
  // (float)(fx + k) == (float)fx + k exactly: |fx| <= 2^24 (tap_floor), and both round
  // the same integer once
  const float fxf = (float)fx, fyf = (float)fy;
  float kx[4], ky[4];
  if (contracts(FM)) {
    kx[0] = cubic_out_fm(wx - (fxf - 1.0f));
    kx[1] = cubic_in_fm(wx - fxf);
    kx[2] = cubic_in_fm(wx - (fxf + 1.0f));
    kx[3] = cubic_out_fm(wx - (fxf + 2.0f));
    ky[0] = cubic_out_fm(wy - (fyf - 1.0f));
    ky[1] = cubic_in_fm(wy - fyf);
    ky[2] = cubic_in_fm(wy - (fyf + 1.0f));
    ky[3] = cubic_out_fm(wy - (fyf + 2.0f));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float w = kx[i] * ky[j];
        const Tap3 g = tap(fy - 1 + j, fx - 1 + i);
        sum = __builtin_fmaf(w, g.x, sum);
        sumx = __builtin_fmaf(w, g.y, sumx);
        sumy = __builtin_fmaf(w, g.z, sumy);
        wsum = wsum + w;
      }
    }
    return;
  }
  kx[0] = cubic_out(wx - (fxf - 1.0f));
  kx[1] = cubic_in(wx - fxf);
  kx[2] = cubic_in(wx - (fxf + 1.0f));
  kx[3] = cubic_out(wx - (fxf + 2.0f));
  ky[0] = cubic_out(wy - (fyf - 1.0f));
  ky[1] = cubic_in(wy - fyf);
  ky[2] = cubic_in(wy - (fyf + 1.0f));
  ky[3] = cubic_out(wy - (fyf + 2.0f));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float w = kx[i] * ky[j];
      const Tap3 g = tap(fy - 1 + j, fx - 1 + i);
      sum = sum + w * g.x;
      sumx = sumx + w * g.y;
      sumy = sumy + w * g.z;
      wsum = wsum + w;
    }
  }
}

// Streaming warpBackward (k_warp_ring, and the producers of k_warp_iter): a block of NW
// wavefronts owns a 64-px column band of a row segment and walks down it, NW output rows
// per step (one row per wavefront, one px per lane).  The block's LDS holds a ring of R rows
// of the (I1, I1x, I1y) window, (64 + 2M) columns wide (clamped coordinates, exactly the
// texture-clamp values; ring row = image row mod R): at step s the rows y0-M .. y0+NW-1+M
// are resident (y0 = first row of the step), so a px whose taps stay within M - 1 px of it
// gathers from LDS; any other px takes the global-memory path (same taps, same order).
// Each wavefront loads one new window row and its own u1 / u2 / I0 row kWarpAhead steps
// ahead into registers and writes the window row when its step comes, so loads are in
// flight while earlier rows compute.  One LDS-only barrier per step (NW > 1): rows written
// at step s+1 are >= 1 and < 2NW + 2M <= R rows past any row a slower wavefront still reads
// at step s, so they never land on a slot in use.  The register rings are unrolled
// (kWarpAhead + 1 steps per loop trip), so no register holding a load in flight is copied.
constexpr int kWarpAhead = 2;

template <int M, int NW>
constexpr int warp_ring_rows() { return 2 * NW + 2 * M <= 16 ? 16 : 32; }

// Column margin and row pitch of the window rings (r4).  The gathers'
// taps are ds_read_b32 / ds_read2_b32, banked (dword address mod 32) per 32-lane half.  A
// half's lanes read consecutive window columns, but where the flow's y-component crosses an
// integer inside the half its lanes read two ring rows: with the r3 row pitch 3WW = 420
// (k_warp_iter) / 228 (k_warp_ring) dwords = 4 (mod 32), 4 lanes of one row landed on the
// banks of 4 lanes of the other, a 2-way conflict on every tap read of that half (measured:
// SQ_LDS_BANK_CONFLICT 16 % of SQ_LDS_IDX_ACTIVE in k_warp_iter; a model of C2's level 0
// gives 26 % extra cycles on the gather).  A pitch = 0 (mod 32) maps a half's 32 consecutive
// columns to 32 distinct banks whichever rows they read.  Rows keep the margin M (the ring
// holds rows r-M .. r+M); columns take M - 1 (flow |u1| < 4 px inside the window instead of
// 5; beyond it the same global-memory path as ever), which makes 3WW fit a multiple of 32
// in less LDS than before: k_warp_iter 3 * 138 = 414 -> 416, k_warp_ring 3 * 74 = 222 -> 224.
template <int M>
constexpr int ring_mx() { return M == 6 ? 5 : M; }
constexpr int ring_pitch(int ww) { return (3 * ww + 31) & ~31; }

// warpBackward's rho_c = I1w - I1wx*u1 - I1wy*u2 - I0 (contracted: the two products
// fused into the running difference, fma(-I1wy, u2, fma(-I1wx, u1, I1w)) - I0).
template <int FM>
__device__ __forceinline__ float rho_c(float I1w, float I1wx, float I1wy, float u1, float u2,
                                       float i0) {
  return contracts(FM) ? __builtin_fmaf(-I1wy, u2, __builtin_fmaf(-I1wx, u1, I1w)) - i0
                       : I1w - I1wx * u1 - I1wy * u2 - i0;
}

// Issue priority falling with a block's progress through its segment (step trip h of n):
// at equal priority a SIMD's arbiter prefers its oldest wave, so in a one-round launch the
// blocks dispatched last to a CU finish last and leave the CU part idle meanwhile.  Measured
// on k_warp_iter at C2 level 0 (tools/wi_probe.hip, per-wave s_memrealtime): block lives of
// 266 / 296 / 333 / 332 / 414 us by dispatch order on the CU, launch 424 us; with this
// 327 / 329 / 350 / 356 / 386 us, launch 388 us.  (Progress against the XCD's other
// blocks, from a per-XCD atomic counter, was slower: 616 us.)
template <int PRIO>
__device__ __forceinline__ void progress_prio(int h, int n) {
  if (!PRIO) return;
  if (h == 0) __builtin_amdgcn_s_setprio(3);
  else if (h == n / 4) __builtin_amdgcn_s_setprio(2);
  else if (h == n / 2) __builtin_amdgcn_s_setprio(1);
  else if (h == 3 * n / 4) __builtin_amdgcn_s_setprio(0);
}

// LDS-only workgroup barrier: waits for this wave's LDS writes, not for its global loads
// in flight (a plain __syncthreads() would drain the prefetch).
#ifdef TVL1_BARRIER_PROBE
// tools/wi_probe.hip: shader cycles each wave spends in lds_barrier (one slot per wave)
__device__ unsigned long long *tvl1_probe_bar;
#endif
__device__ __forceinline__ void lds_barrier() {
#ifdef TVL1_BARRIER_PROBE
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#ifdef TVL1_BARRIER_PROBE
  const unsigned long long dt = __builtin_amdgcn_s_memtime() - t0;
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_fetch_add(tvl1_probe_bar + (blockDim.x >> 6) * blockIdx.x + (threadIdx.x >> 6), dt,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

// The window ring is filled from I1 and holds three float planes (I1, I1x, I1y) -- each window slot's
// centred gradient is computed when its row enters the ring with centeredGradient's
// exact formula at the clamped slot coordinate (the texture-clamp value of the gradient
// image), so there is no G plane: HBM per px and warp is I1 (4 B x 1 + 2M/64) + u1, u2,
// I0 + the three outputs, instead of 16 B of G.  Taps are 2-cycle ds_read_b32s.
// true when a speculative launch's prediction failed: every wave of the grid returns at once
__device__ __forceinline__ bool gated_off(const unsigned long long *gate, unsigned long long seq) {
  return gate != nullptr && *gate != seq;   // a uniform load at entry (written by an earlier launch)
}

struct WarpRingArgs {
  const float *I0, *I1;
  const float *u1, *u2;
  float *I1wx, *I1wy, *rho;
  int W, H, P;
  int bands, seg_rows, waves;   // waves = blocks (bands x segments)
};

struct WarpRowI {   // this lane's 2 window slots of one row (raw I1 stencils) + one flow row
  float c0, l0, r0, n0, s0;   // slot lane:      centre, x-1, x+1, y-1, y+1 (clamped)
  float c1, l1, r1, n1, s1;   // slot 64 + lane
  float u1, u2, i0;
};

// xs: byte offsets of the lane's 2 window slots: clamped column, its clamped x-1 and x+1.
// The row is a scalar offset, so the 10 loads need no per-lane address arithmetic.
__device__ __forceinline__ void warp_ring_load(WarpRowI &v, const WarpRingArgs &a, unsigned nb,
                                               unsigned rowb, int gy, const unsigned (&xs)[2][3]) {
  const int r = imin(imax(gy, 0), a.H - 1);
  const unsigned so = (unsigned)r * rowb, su = (unsigned)imax(r - 1, 0) * rowb,
                 sd = (unsigned)imin(r + 1, a.H - 1) * rowb;
  float t[1];
  bload<1>(t, a.I1, nb, xs[0][0], so); v.c0 = t[0];
  bload<1>(t, a.I1, nb, xs[0][1], so); v.l0 = t[0];
  bload<1>(t, a.I1, nb, xs[0][2], so); v.r0 = t[0];
  bload<1>(t, a.I1, nb, xs[0][0], su); v.n0 = t[0];
  bload<1>(t, a.I1, nb, xs[0][0], sd); v.s0 = t[0];
  // the second slot only exists for lanes < 2M; other lanes re-read slot 0's column
  bload<1>(t, a.I1, nb, xs[1][0], so); v.c1 = t[0];
  bload<1>(t, a.I1, nb, xs[1][1], so); v.l1 = t[0];
  bload<1>(t, a.I1, nb, xs[1][2], so); v.r1 = t[0];
  bload<1>(t, a.I1, nb, xs[1][0], su); v.n1 = t[0];
  bload<1>(t, a.I1, nb, xs[1][0], sd); v.s1 = t[0];
}

__device__ __forceinline__ void warp_flow_load(WarpRowI &v, const WarpRingArgs &a, unsigned nb,
                                               unsigned rowb, int fy, unsigned xcb) {
  const unsigned so = (unsigned)imin(fy, a.H - 1) * rowb;
  float t[1];
  bload<1>(t, a.u1, nb, xcb, so); v.u1 = t[0];
  bload<1>(t, a.u2, nb, xcb, so); v.u2 = t[0];
  bload<1>(t, a.I0, nb, xcb, so); v.i0 = t[0];
}

// Ring layout: [ring row][plane (I1, I1x, I1y)][WW], rows ring_pitch(WW) apart: one tap
// row's 12 values are within 3 * WW < 256 dwords of one base, so they load with
// ds_read2_b32 immediate offsets.
template <int M, int NW>
__device__ __forceinline__ void warp_ring_put(float *__restrict__ ring, const WarpRowI &v, int r,
                                              int lane) {
  constexpr int MX = ring_mx<M>(), WW = 64 + 2 * MX, R = warp_ring_rows<M, NW>();
  float *dst = ring + (r & (R - 1)) * ring_pitch(WW);
  dst[lane] = v.c0;
  dst[WW + lane] = 0.5f * (v.r0 - v.l0);
  dst[2 * WW + lane] = 0.5f * (v.s0 - v.n0);
  if (lane < 2 * MX) {
    dst[64 + lane] = v.c1;
    dst[WW + 64 + lane] = 0.5f * (v.r1 - v.l1);
    dst[2 * WW + 64 + lane] = 0.5f * (v.s1 - v.n1);
  }
}

template <int M, int NW, int FM>
__device__ __forceinline__ void warp_ring_step(float *__restrict__ ring, const WarpRowI &cur,
                                               WarpRowI &ahead, const WarpRingArgs &a, int y0,
                                               int ye, int w, int lane, int x0,
                                               const unsigned (&xs)[2][3], unsigned xcb,
                                               unsigned nb, unsigned rowb) {
  constexpr int MX = ring_mx<M>(), WW = 64 + 2 * MX, R = warp_ring_rows<M, NW>();
  constexpr int PITCH = ring_pitch(WW);
  // loads for step + A: window row y0 + NW*A + M + w, flow row y0 + NW*A + w
  warp_ring_load(ahead, a, nb, rowb, y0 + NW * kWarpAhead + M + w, xs);
  warp_flow_load(ahead, a, nb, rowb, y0 + NW * kWarpAhead + w, xcb);
  __builtin_amdgcn_sched_barrier(0);
  // window row y0 + M + w enters the ring: centeredGradient at each clamped slot
  warp_ring_put<M, NW>(ring, cur, y0 + M + w, lane);
  if (NW > 1) lds_barrier();   // (a wave's own LDS accesses execute in order)
  const int x = x0 + lane, y = y0 + w;
  const float wx = (float)x + cur.u1;
  const float wy = (float)y + cur.u2;
  const int fx = tap_floor(wx);
  const int fy = tap_floor(wy);
  float sum = 0.0f, sumx = 0.0f, sumy = 0.0f, wsum = 0.0f;
  const bool inwin = fx - 1 >= x0 - MX && fx + 2 < x0 + 64 + MX && fy - 1 >= y - M && fy + 2 <= y + M;
  if (inwin) {
    warp_gather_fn<FM>(
        [&](int cy, int cx) {
          const float *p = ring + (cy & (R - 1)) * PITCH + (cx - (x0 - MX));
          return Tap3{p[0], p[WW], p[2 * WW]};
        },
        wx, wy, fx, fy, sum, sumx, sumy, wsum);
  } else {
    warp_gather_fn<FM>(
        [&](int cy, int cx) {
          const int rx = imin(imax(cx, 0), a.W - 1), ry = imin(imax(cy, 0), a.H - 1);
          const float *row = a.I1 + (size_t)ry * a.P;
          const float gx = 0.5f * (row[imin(rx + 1, a.W - 1)] - row[imax(rx - 1, 0)]);
          const float gy = 0.5f * (a.I1[(size_t)imin(ry + 1, a.H - 1) * a.P + rx] -
                                   a.I1[(size_t)imax(ry - 1, 0) * a.P + rx]);
          return Tap3{row[rx], gx, gy};
        },
        wx, wy, fx, fy, sum, sumx, sumy, wsum);
  }
  const float coeff = approx(FM) ? __builtin_amdgcn_rcpf(wsum) : recip_rn(wsum);
  const float I1wv = sum * coeff;
  const float I1wxv = sumx * coeff;
  const float I1wyv = sumy * coeff;
  const unsigned vo = x < a.W && y < ye ? (unsigned)y * rowb + 4u * (unsigned)x : kOOB;
  bstore<kWarpStoreAux>(a.I1wx, nb, vo, 0, I1wxv);
  bstore<kWarpStoreAux>(a.I1wy, nb, vo, 0, I1wyv);
  bstore<kWarpStoreAux>(a.rho, nb, vo, 0, rho_c<FM>(I1wv, I1wxv, I1wyv, cur.u1, cur.u2, cur.i0));
}

template <int M, int NW, int FM>
__device__ __forceinline__ void warp_ring_body(const WarpRingArgs &a, int wid, float *__restrict__ ring) {
  constexpr int MX = ring_mx<M>(), WW = 64 + 2 * MX, R = warp_ring_rows<M, NW>();
  static_assert(3 * WW < 256, "one tap row within ds_read2_b32 offsets");
  static_assert(2 * NW + 2 * M <= R, "ring too small for the margin");
  static_assert(2 * MX <= 64, "second window slot per lane");
  static_assert(ring_pitch(WW) % 32 == 0, "row pitch: no bank conflicts between ring rows");
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int band = wid % a.bands, seg = wid / a.bands;
  const int x0 = band * 64;
  // the lane's two window slots: clamped column, its clamped x-1 and x+1 (byte offsets)
  unsigned xs[2][3];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int slot = k == 0 || lane < 2 * MX ? lane + 64 * k : lane;
    const int cc = imin(imax(x0 - MX + slot, 0), a.W - 1);
    xs[k][0] = 4u * cc;
    xs[k][1] = 4u * imax(cc - 1, 0);
    xs[k][2] = 4u * imin(cc + 1, a.W - 1);
  }
  const unsigned xcb = 4u * imin(x0 + lane, a.W - 1);
  const unsigned nb = 4u * (unsigned)a.P * (unsigned)a.H;   // plane bytes
  const unsigned rowb = 4u * (unsigned)a.P;
  const int ys = seg * a.seg_rows, ye = imin(ys + a.seg_rows, a.H);
  // ring prologue: window rows ys - M .. ys + M - 1, wave w taking rows w, w + NW, ...;
  // all loads are issued before the first write
  {
    constexpr int PR = (2 * M + NW - 1) / NW;
    WarpRowI t[PR];
#pragma unroll
    for (int i = 0; i < PR; ++i) warp_ring_load(t[i], a, nb, rowb, ys - M + w + NW * i, xs);
#pragma unroll
    for (int i = 0; i < PR; ++i) {
      const int r = ys - M + w + NW * i;
      if (r < ys + M) warp_ring_put<M, NW>(ring, t[i], r, lane);
    }
  }
  static_assert(kWarpAhead == 2, "the step loop below is unrolled for a 3-row ring");
  WarpRowI A, B, C;
  auto first = [&](WarpRowI &v, int step) {
    warp_ring_load(v, a, nb, rowb, ys + NW * step + M + w, xs);
    warp_flow_load(v, a, nb, rowb, ys + NW * step + w, xcb);
  };
  first(A, 0);
  first(B, 1);
  for (int y0 = ys; y0 < ye; y0 += 3 * NW) {
    warp_ring_step<M, NW, FM>(ring, A, C, a, y0, ye, w, lane, x0, xs, xcb, nb, rowb);
    warp_ring_step<M, NW, FM>(ring, B, A, a, y0 + NW, ye, w, lane, x0, xs, xcb, nb, rowb);
    warp_ring_step<M, NW, FM>(ring, C, B, a, y0 + 2 * NW, ye, w, lane, x0, xs, xcb, nb, rowb);
  }
}

template <int M, int NW, int FM = 0>
__global__ __launch_bounds__(64 * NW) void k_warp_ring(WarpRingArgs a) {
  __shared__ float ring[warp_ring_rows<M, NW>() * ring_pitch(64 + 2 * ring_mx<M>())];
  const int wid = __builtin_amdgcn_readfirstlane(xcd_chunk(blockIdx.x, gridDim.x));
  if (wid >= a.waves) return;   // whole blocks
  warp_ring_body<M, NW, FM>(a, wid, ring);
}

// warpBackward straight from the level image (no precomputed gradient plane): the
// tile stages I1 over its window + 1 px (clamped coordinates) in LDS, builds the
// (I1, I1x, I1y) window from it with centeredGradient's exact formula
//   I1x = 0.5f * (I1[y][min(x+1,W-1)] - I1[y][max(x-1,0)])   (likewise I1y)
// evaluated at the CLAMPED tap coordinate (texture clamp of the gradient images), and
// gathers every tap from LDS.  Every image coordinate that formula needs for a window cell
// lies in [ox-1, ox+WW] x [oy-1, oy+WH], so the extended I1 window covers it.  HBM per
// px: u1, u2, I0, I1 (16 B) + 12 B of outputs, instead of 16 B of gradient plane.
constexpr int kWarpEW = kWarpWW + 2, kWarpEH = kWarpWH + 2;

__device__ __forceinline__ float4 grad_cell(const float *__restrict__ ext, int ox, int oy, int W,
                                            int H, int cx, int cy) {
  const int rx = imin(imax(cx, 0), W - 1), ry = imin(imax(cy, 0), H - 1);
  auto E = [&](int x, int y) { return ext[(y - (oy - 1)) * kWarpEW + (x - (ox - 1))]; };
  const float c = E(rx, ry);
  const float gx = 0.5f * (E(imin(rx + 1, W - 1), ry) - E(imax(rx - 1, 0), ry));
  const float gy = 0.5f * (E(rx, imin(ry + 1, H - 1)) - E(rx, imax(ry - 1, 0)));
  return make_float4(c, gx, gy, 0.0f);
}

// Global-memory gather for pixels whose taps leave the window: the same taps, with the
// gradient of each (clamped) tap computed from I1 in global memory.
template <int FM>
__device__ __forceinline__ void warp_gather_img_global(const float *__restrict__ I1, int P, int W,
                                                       int H, float wx, float wy, int fx, int fy,
                                                       float &sum, float &sumx, float &sumy,
                                                       float &wsum) {
  warp_gather_fn<FM>(
      [&](int cy, int cx) {
        const int rx = imin(imax(cx, 0), W - 1), ry = imin(imax(cy, 0), H - 1);
        const float *row = I1 + (size_t)ry * P;
        const float gx = 0.5f * (row[imin(rx + 1, W - 1)] - row[imax(rx - 1, 0)]);
        const float gy = 0.5f * (I1[(size_t)imin(ry + 1, H - 1) * P + rx] -
                                 I1[(size_t)imax(ry - 1, 0) * P + rx]);
        return Tap3{row[rx], gx, gy};
      },
      wx, wy, fx, fy, sum, sumx, sumy, wsum);
}

template <int FM>
__global__ __launch_bounds__(256) void k_warp_img(const float *__restrict__ I0,
                                                  const float *__restrict__ I1,
                                                  const float *__restrict__ u1,
                                                  const float *__restrict__ u2, int W, int H,
                                                  int P, int tiles_x, float *__restrict__ I1wx,
                                                  float *__restrict__ I1wy,
                                                  float *__restrict__ rho) {
  __shared__ float4 win[kWarpWH * kWarpWW];
  __shared__ float ext[kWarpEH * kWarpEW];
  int bx, by;
  tile_of_block(blockIdx.x, gridDim.x, tiles_x, gridDim.x / tiles_x, bx, by);
  const int x0 = bx * kWarpTW, y0 = by * kWarpTH;
  const int ox = x0 - kWarpHalo, oy = y0 - kWarpHalo;   // window origin (unclamped coords)
  constexpr int R = kWarpTH / 4;
  const int x = x0 + (threadIdx.x & 63);
  const int xc = imin(x, W - 1);
  float u1v[R], u2v[R], i0v[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int y = imin(y0 + (threadIdx.x >> 6) + 4 * j, H - 1);
    const size_t i = (size_t)y * P + xc;
    u1v[j] = u1[i];
    u2v[j] = u2[i];
    i0v[j] = I0[i];
  }
  for (int i = threadIdx.x; i < kWarpEH * kWarpEW; i += 256) {
    const int ey = i / kWarpEW, ex = i - ey * kWarpEW;
    const int cx = imin(imax(ox - 1 + ex, 0), W - 1);
    const int cy = imin(imax(oy - 1 + ey, 0), H - 1);
    ext[i] = I1[(size_t)cy * P + cx];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kWarpWH * kWarpWW; i += 256) {
    const int wy = i / kWarpWW, wx = i - wy * kWarpWW;
    win[i] = grad_cell(ext, ox, oy, W, H, ox + wx, oy + wy);
  }
  __syncthreads();
  if (x >= W) return;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int y = y0 + (threadIdx.x >> 6) + 4 * j;
    if (y >= H) break;
    const size_t i = (size_t)y * P + x;
    const float wx = (float)x + u1v[j];
    const float wy = (float)y + u2v[j];
    const int fx = tap_floor(wx);
    const int fy = tap_floor(wy);
    float sum = 0.0f, sumx = 0.0f, sumy = 0.0f, wsum = 0.0f;
    const bool inwin = fx - 1 >= ox && fx + 2 < ox + kWarpWW && fy - 1 >= oy && fy + 2 < oy + kWarpWH;
    if (inwin)
      warp_gather_fn<FM>(
          [&](int cy, int cx) {
            const float4 g = win[(cy - oy) * kWarpWW + (cx - ox)];
            return Tap3{g.x, g.y, g.z};
          },
          wx, wy, fx, fy, sum, sumx, sumy, wsum);
    else
      warp_gather_img_global<FM>(I1, P, W, H, wx, wy, fx, fy, sum, sumx, sumy, wsum);
    const float coeff = approx(FM) ? __builtin_amdgcn_rcpf(wsum) : recip_rn(wsum);
    const float I1wv = sum * coeff;
    const float I1wxv = sumx * coeff;
    const float I1wyv = sumy * coeff;
    I1wx[i] = I1wxv;
    I1wy[i] = I1wyv;
    rho[i] = rho_c<FM>(I1wv, I1wxv, I1wyv, u1v[j], u2v[j], i0v[j]);
  }
}

// ---------------------------------------------------------------- K6+K8 fused
struct IterArgs {
  const float *I1wx, *I1wy, *rho;                                  // warp constants
  const float *u1s, *u2s, *u3s;                                    // state in
  const float *p11s, *p12s, *p21s, *p22s, *p31s, *p32s;
  float *u1d, *u2d, *u3d;                                          // state out
  float *p11d, *p12d, *p21d, *p22d, *p31d, *p32d;
  double *partials;                                                // per-block residual sums
  int W, H, P;                                                     // P = pitch in floats
  int segs, strip_rows;
  float l_t, theta, gamma, taut;
  int calc_err, p_zero;
  int taut_small;   // host: |taut| <= 2^20, so sqrt_nn may skip its (0, 2^-96) form (0: never)
  // speculation gate: a launch enqueued behind a residual check runs only if
  // that check's k_reduce found the predicted schedule (*gate == gate_seq); null: always
  const unsigned long long *gate;
  unsigned long long gate_seq;
};


template <bool G, int PX = 4>
struct Row {
  float wx[PX], wy[PX], rh[PX], u1[PX], u2[PX], p11[PX], p12[PX], p21[PX], p22[PX];
  float u3[PX], p31[PX], p32[PX];  // used only when G (dead otherwise)
};

// PX consecutive floats <-> one 8- or 16-byte vector access
template <int N> struct VecT;
template <> struct VecT<4> { using type = float4; };
template <> struct VecT<2> { using type = float2; };

__device__ __forceinline__ void unpack(float (&d)[4], const float4 &t) {
  d[0] = t.x; d[1] = t.y; d[2] = t.z; d[3] = t.w;
}
__device__ __forceinline__ void unpack(float (&d)[2], const float2 &t) {
  d[0] = t.x; d[1] = t.y;
}
__device__ __forceinline__ float4 pack(const float (&s)[4]) { return make_float4(s[0], s[1], s[2], s[3]); }
__device__ __forceinline__ float2 pack(const float (&s)[2]) { return make_float2(s[0], s[1]); }

template <int N>
__device__ __forceinline__ void ldv(float (&d)[N], const float *__restrict__ base, size_t off) {
  unpack(d, *reinterpret_cast<const typename VecT<N>::type *>(base + off));
}
template <int N>
__device__ __forceinline__ void stv(float *__restrict__ base, size_t off, const float (&s)[N]) {
  *reinterpret_cast<typename VecT<N>::type *>(base + off) = pack(s);
}
template <int N>
__device__ __forceinline__ void zerov(float (&d)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) d[i] = 0.0f;
}
__device__ __forceinline__ void ld4(float (&d)[4], const float *__restrict__ base, size_t off) { ldv<4>(d, base, off); }
__device__ __forceinline__ void st4(float *__restrict__ base, size_t off, const float (&s)[4]) { stv<4>(base, off, s); }
__device__ __forceinline__ void zero4(float (&d)[4]) { zerov<4>(d); }

template <bool G, int PX = 4>
__device__ __forceinline__ void load_row(Row<G, PX> &r, const IterArgs &a, size_t off) {
  ldv<PX>(r.wx, a.I1wx, off);
  ldv<PX>(r.wy, a.I1wy, off);
  ldv<PX>(r.rh, a.rho, off);
  ldv<PX>(r.u1, a.u1s, off);
  ldv<PX>(r.u2, a.u2s, off);
  if (G) ldv<PX>(r.u3, a.u3s, off);
  if (a.p_zero) {
    zerov<PX>(r.p11); zerov<PX>(r.p12); zerov<PX>(r.p21); zerov<PX>(r.p22);
    if (G) { zerov<PX>(r.p31); zerov<PX>(r.p32); }
  } else {
    ldv<PX>(r.p11, a.p11s, off);
    ldv<PX>(r.p12, a.p12s, off);
    ldv<PX>(r.p21, a.p21s, off);
    ldv<PX>(r.p22, a.p22s, off);
    if (G) { ldv<PX>(r.p31, a.p31s, off); ldv<PX>(r.p32, a.p32s, off); }
  }
}

// OpenCV `divergence` (tvl1flow.cu) at px k of this lane; pl = p1 at x-1, pu = p2 at y-1.
// Branch-free: every form is evaluated with its own association and the right one
// selected (the x == 0, y > 0 form associates differently from the interior one).
// YZ (the rolling pipelines): the caller's p2u is already +0.0f on row 0 (they zero p above
// the image when they produce it), so there is no row-0 select, and the column-0 form is
// evaluated only in a branch taken by wavefronts that hold a column <= 0 (c0w, wave-uniform:
// the first band; columns < 0 are halo lanes, never stored).  The empty asm keeps the
// compiler from flattening that branch into a select the other bands would pay.
template <bool YZ = false>
__device__ __forceinline__ float divergence(float p1, float p1l, float p2, float p2u, int x,
                                            int y, bool c0w = true) {
  // interior (p1 - p1l) + (p2 - p2u) and row 0 (p1 - p1l) + p2 are one form with p2u := 0
  // at y = 0 (p2 - +0 == p2 exactly, signed zeros included); column 0 (p1 + p2) - p2u and
  // the corner p1 + p2 likewise
  if (YZ) {
    float d = (p1 - p1l) + (p2 - p2u);
    if (c0w) {
      asm volatile("" ::: "memory");
      d = x <= 0 ? (p1 + p2) - p2u : d;
    }
    return d;
  }
  const float p2u0 = y > 0 ? p2u : 0.0f;
  const float rest = (p1 - p1l) + (p2 - p2u0);
  const float col0 = (p1 + p2) - p2u0;
  return x > 0 ? rest : col0;
}

// Contracting modes (FM != kIEEE, see kIEEE / kFast / kFma): fm_fma marks the fused sites.
__device__ __forceinline__ float fm_fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

__device__ __forceinline__ float th_quot(float rho, float gradv, bool mid);

// estimateU's TH step at one px: v = u^{n-1} + d from the warp constants (pointwise).
// CPUP: profile 1 (OpenCV's CPU estimateV): rho = rho_c + (I1wx*u1 + I1wy*u2) [+ gamma*u3]
template <bool G, int FM = 0, bool CPUP = false>
__device__ __forceinline__ void th_px(float I1wxv, float I1wyv, float rhoc, float u1o, float u2o,
                                      float u3o, const IterArgs &a, float &v1, float &v2,
                                      float &v3) {
  const float Ix2 = I1wxv * I1wxv;
  const float Iy2 = I1wyv * I1wyv;
  // warpBackward's grad = Ix2 + Iy2 (contracted: fma(I1wx, I1wx, Iy2))
  const float gradv = contracts(FM) ? fm_fma(I1wxv, I1wxv, Iy2) : Ix2 + Iy2;
  // gamma*u3 inside the parentheses (with gamma = 0 either association gives
  // the same bits, signed zeros included).  Contracted: rho_c + fma(gamma, u3, fma(I1wx,
  // u1, I1wy*u2)), with u3 = 0 (gamma ? u3 : 0) when gamma = 0 -- the fma still turns a
  // -0 sum into +0, as the reference's expression does.
  const float rho =
      CPUP ? (G ? rhoc + (I1wxv * u1o + I1wyv * u2o) + a.gamma * u3o
                : rhoc + (I1wxv * u1o + I1wyv * u2o))
      // (gamma = 0 in the G = false kernels: gamma*u3 is +0, added as the literal)
      : contracts(FM) ? rhoc + (G ? fm_fma(a.gamma, u3o, fm_fma(I1wxv, u1o, I1wyv * u2o))
                                  : fm_fma(I1wxv, u1o, I1wyv * u2o) + 0.0f)
           : rhoc + (I1wxv * u1o + I1wyv * u2o + (G ? a.gamma * u3o : 0.0f));
  // TH operator, branch-free: the three candidate steps are computed with the
  // reference's exact expressions and the applicable one selected.
  // (-l_t)*g == -(l_t*g) exactly (round-to-nearest is sign-symmetric): one product serves
  // both bounds, and each +-l_t*I1w* pair below likewise
  const float ltg = a.l_t * gradv;
  const bool lo = rho < -ltg;
  const bool hi = rho > ltg;
  const bool mid = gradv > kFltEps;
  // only selected when gradv > FLT_EPSILON
  const float fi = approx(FM) ? -rho * __builtin_amdgcn_rcpf(gradv) : th_quot(rho, gradv, mid);
  // d = lo ? l_t*I : hi ? -l_t*I : mid ? fi*I : 0 for I = I1wx, I1wy (gamma): the factor is
  // selected once and multiplied per component -- (-l_t)*I == -(l_t*I) exactly, and the
  // "none" case stays a selected +0 (0*I would be -0 for I < 0)
  const float f = lo ? a.l_t : hi ? -a.l_t : fi;
  const bool any = lo || hi || mid;
  const float d1 = any ? f * I1wxv : 0.0f;
  const float d2 = any ? f * I1wyv : 0.0f;
  const float d3 = any ? f * a.gamma : 0.0f;     // +-l_t*gamma
  v1 = u1o + d1;
  v2 = u2o + d2;
  v3 = G ? u3o + d3 : 0.0f;
}

// estimateU's second half at one px: u^n = v + theta * div(p^{n-1}).  pl = p*1 at x-1,
// pu = p*2 at y-1.
template <bool G, int FM = 0, bool YZ = false>
__device__ __forceinline__ void u_from_v(float v1, float v2, float v3, float p11, float p11l,
                                         float p12, float p12u, float p21, float p21l,
                                         float p22, float p22u, float p31, float p31l,
                                         float p32, float p32u, int x, int y,
                                         const IterArgs &a, float &n1, float &n2, float &n3,
                                         bool c0w = true) {
  const float div1 = divergence<YZ>(p11, p11l, p12, p12u, x, y, c0w);
  const float div2 = divergence<YZ>(p21, p21l, p22, p22u, x, y, c0w);
  n1 = contracts(FM) ? fm_fma(a.theta, div1, v1) : v1 + a.theta * div1;
  n2 = contracts(FM) ? fm_fma(a.theta, div2, v2) : v2 + a.theta * div2;
  if (G) {
    const float div3 = divergence<YZ>(p31, p31l, p32, p32u, x, y, c0w);
    n3 = contracts(FM) ? fm_fma(a.theta, div3, v3) : v3 + a.theta * div3;
  }
}

// estimateU's error term (u1Old - u1New)^2 + (u2Old - u2New)^2 (contracted: fma(d1, d1,
// d2*d2)); cuda::sum accumulates it in double.
template <int FM>
__device__ __forceinline__ float residual_px(float d1, float d2) {
  return contracts(FM) ? fm_fma(d1, d1, d2 * d2) : d1 * d1 + d2 * d2;
}

// estimateU at one px (x, y): the TH step from the warp constants and u^{n-1}, then
// u^n = v + theta * div(p^{n-1}).  Shared by every iteration kernel, so they all run
// exactly this sequence of IEEE float operations.
template <bool G, int FM = 0, bool CPUP = false, bool YZ = false>
__device__ __forceinline__ void estimate_u_px(float I1wxv, float I1wyv, float rhoc, float u1o,
                                              float u2o, float u3o, float p11, float p11l,
                                              float p12, float p12u, float p21, float p21l,
                                              float p22, float p22u, float p31, float p31l,
                                              float p32, float p32u, int x, int y,
                                              const IterArgs &a, float &n1, float &n2,
                                              float &n3, bool c0w = true) {
  float v1, v2, v3;
  th_px<G, FM, CPUP>(I1wxv, I1wyv, rhoc, u1o, u2o, u3o, a, v1, v2, v3);
  u_from_v<G, FM, YZ>(v1, v2, v3, p11, p11l, p12, p12u, p21, p21l, p22, p22u, p31, p31l, p32,
                      p32u, x, y, a, n1, n2, n3, c0w);
}

// estimateU for the PX px of this lane on row y.  up* = p12/p22/p32 of row y-1.
template <bool G, int PX = 4, int FM = 0, bool CPUP = false>
__device__ __forceinline__ void estimate_u(const Row<G, PX> &r, const float (&up12)[PX],
                                           const float (&up22)[PX], const float (&up32)[PX],
                                           int X0, int y, const IterArgs &a, float (&n1)[PX],
                                           float (&n2)[PX], float (&n3)[PX]) {
  float l11[PX], l21[PX], l31[PX];
  l11[0] = __shfl_up(r.p11[PX - 1], 1);
  l21[0] = __shfl_up(r.p21[PX - 1], 1);
  if (G) l31[0] = __shfl_up(r.p31[PX - 1], 1);
#pragma unroll
  for (int k = 1; k < PX; ++k) {
    l11[k] = r.p11[k - 1];
    l21[k] = r.p21[k - 1];
    if (G) l31[k] = r.p31[k - 1];
  }
#pragma unroll
  for (int k = 0; k < PX; ++k) {
    const float u3o = G ? r.u3[k] : 0.0f;
    const float p31 = G ? r.p31[k] : 0.0f, p31l = G ? l31[k] : 0.0f;
    const float p32 = G ? r.p32[k] : 0.0f;
    estimate_u_px<G, FM, CPUP>(r.wx[k], r.wy[k], r.rh[k], r.u1[k], r.u2[k], u3o, r.p11[k], l11[k],
                     r.p12[k], up12[k], r.p21[k], l21[k], r.p22[k], up22[k], p31, p31l, p32,
                     up32[k], X0 + k, y, a, n1[k], n2[k], n3[k]);
  }
}

// Correctly rounded sqrt of x >= 0 (or +inf): the compiler's IEEE sqrtf sequence
// (v_sqrt_f32 on x scaled by 2^32 below 2^-96, the two one-ulp neighbours tested with fma
// residuals, scaled back by 2^-16) without its final class test, which returns x itself
// for +-0 and +inf -- the sequence already gives exactly those (+0: the candidates are
// NaN and a denormal whose residual is +0; +inf: NaN residuals).  -0 cannot reach it.
__device__ __forceinline__ float sqrt_rn_core(float xs) {
  const float s = __builtin_amdgcn_sqrtf(xs);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u);
  const float sp = __uint_as_float(__float_as_uint(s) + 1u);
  const float rm = __builtin_fmaf(-sm, s, xs);
  const float rp = __builtin_fmaf(-sp, s, xs);
  const float r = rm <= 0.0f ? sm : s;
  return rp > 0.0f ? sp : r;
}
// x in (0, 2^-96) takes the scaled form (x*2^32, then *2^-16) in a branch the wavefront skips
// when none of its lanes has such an x: both differences under 2^-48 yet not both zero, which
// essentially never happens.  +0 (a locally constant u: every px of a first iteration on the
// coarsest level) needs no scaling -- the core returns +0 exactly -- so it no longer sends the
// wavefront into the scaled form, which made the branch slower than a select in the
// unrolled pipelines (r2).  One unsigned compare finds (0, 2^-96): bits(x) - 1 wraps +0 (and
// keeps NaN) above bits(2^-96) - 1.
// The same correctly rounded sqrt from full-rate instructions only (r6): y0 = v_rsq_f32(x +
// 2^-126), g0 = x*y0, h0 = y0/2, one fma residual d = x - g0^2 and g = g0 + d*h0.  Exhaustive
// on gfx950 (tools/sqrt_fma_check.hip, candidate C3): equal to RN(sqrt(x)) for every float in
// [2^-96, 2^128) and for +0 (x + 2^-126 == x from 2^-96 up; at +0 the rsq input is finite and
// g0 = +0 * y0 = +0, so no select).  sqrt_rn_core issues v_sqrt, two integer adds, two fmas,
// two half-rate compares and two half-rate selects; this issues v_rsq and five full-rate
// instructions: ~15 of a sqrt's ~35 SIMD issue cycles (DESIGN.md §4.7 of r6).  Not for +inf
// (an inf residual gives NaN), which a sum of squares of finite flow differences cannot
// reach; the scaled form of (0, 2^-96) keeps sqrt_rn_core (C3 is off by one ulp for 7 of
// those inputs).
__device__ __forceinline__ float sqrt_rn_fma(float x) {
  const float y0 = __builtin_amdgcn_rsqf(x + 0x1p-126f);
  const float g0 = x * y0;
  const float h0 = 0.5f * y0;
  const float d = __builtin_fmaf(-g0, g0, x);
  return __builtin_fmaf(d, h0, g0);
}

#ifndef TVL1_SQRT_FMA
#define TVL1_SQRT_FMA 1   // 0: r5's neighbour-test core on every lane (A/B builds only)
#endif
// tiny_exact (wave-uniform): whether x in (0, 2^-96) must get its correctly rounded root.  The
// only consumer, the projection's ng = 1 + taut*g (dual_px), is exactly 1 whenever |taut*g| <
// 2^-25, and below 2^-96 both RN(sqrt(x)) and sqrt_rn_fma(x) are under 1.5 * 2^-48 (rsq within
// 1 ulp, g0 <= sqrt(x), |d*h0| <= sqrt(x)/2): with |taut| <= 2^20 the scaled form cannot change
// a bit of ng, so dual_px skips its compare and branch then (DESIGN.md §4.7 of r6).
template <bool BR>
__device__ __forceinline__ float sqrt_nn(float x, bool tiny_exact = true) {
  (void)BR;
  float r = TVL1_SQRT_FMA ? sqrt_rn_fma(x) : sqrt_rn_core(x);
  if (TVL1_SQRT_FMA && !tiny_exact) return r;
  const bool tiny = __float_as_uint(x) - 1u < __float_as_uint(0x1p-96f) - 1u;
  if (__ballot(tiny)) {
    asm volatile("" ::: "memory");   // keep it a branch (see divergence)
    r = tiny ? sqrt_rn_core(x * 0x1p32f) * 0x1p-16f : r;
  }
  return r;
}

template <bool BR = false>
__device__ __forceinline__ float hypot_f(float a, float b, bool tiny_exact = true) {
  return sqrt_nn<BR>(a * a + b * b, tiny_exact);
}

// Correctly rounded a / d for the projection's d = ng = 1 + taut * |grad u| >= 1 (taut >= 0):
// the compiler's IEEE division sequence (div_scale, refined reciprocal, two fma
// corrections, div_fmas, div_fixup) minus the denominator's div_scale, which returns d
// unchanged unless d is denormal, 1/d is, or exp(a) - exp(d) >= 96 -- none can happen:
// |p| <= 1 (the projection keeps it there) gives |a| = |p + taut*du| <= 1 + taut*|grad u| = d.
// The refined reciprocal is shared by the two quotients with the same d.
struct Recip {
  float d, y;
};
__device__ __forceinline__ Recip recip_of(float d) { return Recip{d, recip_rn(d)}; }
__device__ __forceinline__ float div_by(float a, const Recip &R) {
  bool scaled;
  const float n = __builtin_amdgcn_div_scalef(a, R.d, true, &scaled);
  const float q0 = n * R.y;
  const float r0 = __builtin_fmaf(-R.d, q0, n);
  const float q1 = __builtin_fmaf(r0, R.y, q0);
  const float r1 = __builtin_fmaf(-R.d, q1, n);
  const float q = __builtin_amdgcn_div_fmasf(r1, R.y, q1, scaled);
  return __builtin_amdgcn_div_fixupf(q, R.d, a);
}

// Markstein's short quotient: with y = RN(1/d) (recip_of's refined reciprocal; exhaustive
// over 15 binades in tools/div_check.hip), q0 = RN(a*y), r0 = a - d*q0 (exact) and
// q1 = RN(q0 + r0*y) is the correctly rounded a / d whenever r0 does not underflow, i.e. for
// |a| >= 2^-103 when d >= 1 (tools/div_check.hip: 2^32 random quotients in each of the
// projection's and the TH step's ranges, edge numerators, no mismatch; mismatches start below
// 2^-103).  Callers send |a| < 2^-100, zero included, through div_by instead.
__device__ __forceinline__ float div_short(float a, const Recip &R) {
  const float q0 = a * R.y;
  const float r0 = __builtin_fmaf(-R.d, q0, a);
  return __builtin_fmaf(r0, R.y, q0);
}

// The TH step's -rho / grad (selected only where grad > FLT_EPSILON, so grad is in
// [2^-23, 2^15]: |I1wx|, |I1wy| <= 127.5): the short quotient; the IEEE division for lanes
// with |rho| < 2^-100 (zero included) behind a wave-uniform branch (a ballot), so the
// compiler cannot fold it into a select that would run both.  tools/div_check.hip:
// reciprocal exhaustive over those binades; 2^32 random TH quotients with |a| >= 2^-80 and
// 2^32 tiny numerators against d in [2^-23, 2^40): mismatches only for |a| < 2^-104.
__device__ __forceinline__ float th_quot(float rho, float gradv, bool mid) {
  float fi = div_short(-rho, recip_of(gradv));
  const bool bad = mid && __builtin_fabsf(rho) < 0x1p-100f;
  if (__ballot(bad)) fi = bad ? -rho / gradv : fi;
  return fi;
}

// estimateDualVariables for one (u, p*1, p*2) component at one px:
// p' = (p + taut * du) / ng, du from u at (x+1) and (y+1) (clamped at the image edge).
// EXACT: plain IEEE divisions, for taut < 0 or non-finite (k_iterate<G, true>; the host
// routes such parameters there), where ng >= 1 does not hold.
// CPUP: profile 1, |grad u| as glibc hypotf: (float) sqrt((double) a*a + (double) b*b)
template <bool EXACT = false, bool BR = false, int FM = 0, bool CPUP = false>
__device__ __forceinline__ void dual_px(float uc, float ur, float ud, bool has_right,
                                        bool has_down, float taut, float pa, float pb, float &oa,
                                        float &ob, bool taut_small = false) {
  const float right = has_right ? ur : uc;
  const float down = has_down ? ud : uc;
  const float ux = right - uc;
  const float uy = down - uc;
  // contracted (the reference's hypotf restated as sqrt(ux*ux + uy*uy)): ux*ux + uy*uy ->
  // fma(ux, ux, uy*uy); 1 + taut*g -> fma(taut, g, 1); p + taut*ux -> fma(taut, ux, p)
  if (approx(FM) && !EXACT) {
    const float g = __builtin_amdgcn_sqrtf(fm_fma(ux, ux, uy * uy));
    const float r = __builtin_amdgcn_rcpf(fm_fma(taut, g, 1.0f));
    oa = fm_fma(taut, ux, pa) * r;
    ob = fm_fma(taut, uy, pb) * r;
    return;
  }
  // taut_small (IterArgs, a kernel argument: wave-uniform): |taut| <= 2^20 (see sqrt_nn)
  const bool tiny_exact = !taut_small;
  const float g = CPUP ? (float)__builtin_sqrt((double)ux * ux + (double)uy * uy)
                  : contracts(FM) ? sqrt_nn<BR>(fm_fma(ux, ux, uy * uy), tiny_exact)
                                  : hypot_f<BR>(ux, uy, tiny_exact);
  const float ng = contracts(FM) ? fm_fma(taut, g, 1.0f) : 1.0f + taut * g;
  if (EXACT) {
    oa = (pa + taut * ux) / ng;
    ob = (pb + taut * uy) / ng;
  } else {
    // the short quotient for every lane, then the full sequence only for lanes with a tiny
    // or zero numerator, in a branch the wavefront skips when it has none (in the unrolled
    // pipelines too: +2.7 % there, where the sqrt's scaling branch was slower than a select)
    const Recip R = recip_of(ng);
    const float na = contracts(FM) ? fm_fma(taut, ux, pa) : pa + taut * ux;
    const float nb = contracts(FM) ? fm_fma(taut, uy, pb) : pb + taut * uy;
    oa = div_short(na, R);
    ob = div_short(nb, R);
    const bool tiny = __builtin_fabsf(na) < 0x1p-100f || __builtin_fabsf(nb) < 0x1p-100f;
    if (__ballot(tiny)) {
      oa = tiny ? div_by(na, R) : oa;
      ob = tiny ? div_by(nb, R) : ob;
    }
  }
}

// One projection component for the PX px of this lane.
template <int PX, bool EXACT = false, int FM = 0, bool CPUP = false>
__device__ __forceinline__ void dual_component(const float (&uc)[PX], const float (&un)[PX],
                                               bool has_down, int X0, int W, float taut,
                                               const float (&pa)[PX], const float (&pb)[PX],
                                               float (&oa)[PX], float (&ob)[PX],
                                               bool taut_small = false) {
  float ur[PX];
  ur[PX - 1] = __shfl_down(uc[0], 1);
#pragma unroll
  for (int k = 0; k < PX - 1; ++k) ur[k] = uc[k + 1];
#pragma unroll
  for (int k = 0; k < PX; ++k)
    dual_px<EXACT, true, FM, CPUP>(uc[k], ur[k], un[k], X0 + k + 1 < W, has_down, taut, pa[k], pb[k],
                         oa[k], ob[k], taut_small);
}

template <bool G, bool EXACT = false, bool CPUP = false>
__global__ __launch_bounds__(kBlock) void k_iterate(IterArgs a) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = blockIdx.x * (kBlock / kWave) + (threadIdx.x >> 6);
  const int seg = wave % a.segs;
  const int strip = wave / a.segs;
  const int y0 = strip * a.strip_rows;
  double acc = 0.0;
  if (y0 < a.H) {
    const int y1 = imin(y0 + a.strip_rows, a.H);
    const int X0 = seg * kSegPx - 4 + lane * 4;        // first px of this lane
    const int xa = imin(imax(X0, 0), a.P - 4);         // clamped, 16-B aligned load column
    const bool writer = lane >= 1 && lane <= kWave - 2 && X0 < a.W;

    float up12[4], up22[4], up32[4];
    if (y0 > 0 && !a.p_zero) {
      const size_t off = (size_t)(y0 - 1) * a.P + xa;
      ld4(up12, a.p12s, off);
      ld4(up22, a.p22s, off);
      if (G) ld4(up32, a.p32s, off);
      else zero4(up32);
    } else {
      zero4(up12); zero4(up22); zero4(up32);
    }
    Row<G> cur;
    load_row<G>(cur, a, (size_t)y0 * a.P + xa);
    float c1[4], c2[4], c3[4];
    estimate_u<G, 4, false, CPUP>(cur, up12, up22, up32, X0, y0, a, c1, c2, c3);

    for (int y = y0; y < y1; ++y) {
      const bool has_down = y + 1 < a.H;
      Row<G> nxt;
      float n1[4], n2[4], n3[4];
      if (has_down) {
        load_row<G>(nxt, a, (size_t)(y + 1) * a.P + xa);
        estimate_u<G, 4, false, CPUP>(nxt, cur.p12, cur.p22, cur.p32, X0, y + 1, a, n1, n2, n3);
      } else {  // last image row: forward difference in y is 0 (clamp)
#pragma unroll
        for (int k = 0; k < 4; ++k) { n1[k] = c1[k]; n2[k] = c2[k]; n3[k] = c3[k]; }
      }
      float q11[4], q12[4], q21[4], q22[4], q31[4], q32[4];
      dual_component<4, EXACT, false, CPUP>(c1, n1, has_down, X0, a.W, a.taut, cur.p11, cur.p12, q11, q12, a.taut_small);
      dual_component<4, EXACT, false, CPUP>(c2, n2, has_down, X0, a.W, a.taut, cur.p21, cur.p22, q21, q22, a.taut_small);
      if (G)
        dual_component<4, EXACT, false, CPUP>(c3, n3, has_down, X0, a.W, a.taut, cur.p31, cur.p32, q31, q32, a.taut_small);
      if (writer) {
        const size_t off = (size_t)y * a.P + xa;
        st4(a.u1d, off, c1);
        st4(a.u2d, off, c2);
        st4(a.p11d, off, q11);
        st4(a.p12d, off, q12);
        st4(a.p21d, off, q21);
        st4(a.p22d, off, q22);
        if (G) {
          st4(a.u3d, off, c3);
          st4(a.p31d, off, q31);
          st4(a.p32d, off, q32);
        }
        if (a.calc_err) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (X0 + k < a.W) {
              const float e1 = (cur.u1[k] - c1[k]) * (cur.u1[k] - c1[k]);
              const float e2 = (cur.u2[k] - c2[k]) * (cur.u2[k] - c2[k]);
              acc += (double)(e1 + e2);
            }
          }
        }
      }
      if (has_down) {
        cur = nxt;
#pragma unroll
        for (int k = 0; k < 4; ++k) { c1[k] = n1[k]; c2[k] = n2[k]; if (G) c3[k] = n3[k]; }
      }
    }
  }
  if (a.calc_err) {
    __shared__ double red[kBlock / kWave];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = 0.0;
      for (int i = 0; i < kBlock / kWave; ++i) s += red[i];
      a.partials[blockIdx.x] = s;
    }
  }
}

// ---------------------------------------------------------------- K6+K8 temporally blocked
// k_iterate_tb: runs `niter` (1..4) consecutive primal-dual iterations in ONE HBM pass.
//
// A workgroup owns a region of 64 x RH px (64/PX lanes per row, PX = 4 or 2 px per
// lane; every thread owns NG groups, rows rr, rr + RH/NG, ...).  It loads u, p and the warp
// constants once, iterates in registers, and stores only the interior that is still
// exact after niter iterations: each iteration invalidates one px at every internal
// region edge (u needs p at x-1, y-1; p needs u at x+1, y+1), so the region keeps a
// 4-px halo in x (float4 alignment) and a niter-px halo in y.  At the image border the
// clamp / special-divergence forms of OpenCV apply and nothing is invalidated.
//   x neighbours: wavefront shuffles (16 lanes per row);
//   y neighbours: 4 LDS planes (p12, p22 for estimateU; u1, u2 for the projection);
//   per px-iteration HBM traffic: (36 B / efficiency + 24 B) / niter instead of 60 B.
// Arithmetic is exactly the per-pixel sequence of k_iterate (bit-identical results).
struct TBArgs {
  IterArgs it;
  int niter;        // iterations in this pass (1..4); the residual is of the last one
  int tiles_x;      // regions per row
  int out_h;        // output rows per region = RH - 2*niter
};

// Pass body of the blocked kernel: stage the vertically read planes, run the pass's
// iterations on register-resident state, store the exact interior and the residual
// partial of the last iteration.  lds = NPL planes of RH x LPR vectors of PX floats.
template <bool G, int RH, int NG, int PX, int FM>
__device__ __forceinline__ void tb_iterate_store(const TBArgs &t,
                                                 typename VecT<PX>::type *__restrict__ lds,
                                                 Row<G, PX> (&r)[NG], const int (&Y)[NG], int X,
                                                 int c4, int rr) {
  constexpr int LPR = 64 / PX;                   // lanes per region row
  constexpr int NT = LPR * RH / NG;
  constexpr int HALF = RH / NG;
  constexpr int PL = RH * LPR;                   // vectors per LDS plane
  constexpr int HALO = 4 / PX;                   // lanes of the 4-px x halo
  using V = typename VecT<PX>::type;
  const IterArgs &a = t.it;
  const int K = t.niter;
  auto L = [&](int plane, int row) -> V & { return lds[plane * PL + row * LPR + c4]; };
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int row = rr + g * HALF;
    L(0, row) = pack(r[g].p12);
    L(1, row) = pack(r[g].p22);
    if (G) L(4, row) = pack(r[g].p32);
  }
  __syncthreads();

  // this thread's cells that the pass stores (region interior, inside the image)
  bool out_ok[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int row = rr + g * HALF;
    out_ok[g] = c4 >= HALO && c4 < LPR - HALO && row >= K && row < RH - K && Y[g] >= 0 && Y[g] < a.H &&
                X < a.W;
  }
  double acc = 0.0;   // residual of the last iteration over the stored cells
  for (int it = 0; it < K; ++it) {
    const bool last = it == K - 1;
    // ---- estimateU, one group at a time (keeps the live register set small)
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int row = rr + g * HALF;
      const int rowu = row > 0 ? row - 1 : 0;
      float up12[PX], up22[PX], up32[PX];
      unpack(up12, L(0, rowu));
      unpack(up22, L(1, rowu));
      if (G) unpack(up32, L(4, rowu));
      else zerov<PX>(up32);
      float n1[PX], n2[PX], n3[PX];
      estimate_u<G, PX, FM>(r[g], up12, up22, up32, X, Y[g], a, n1, n2, n3);
      if (last && a.calc_err && out_ok[g]) {
#pragma unroll
        for (int k = 0; k < PX; ++k) {
          if (X + k < a.W) {
            acc += (double)residual_px<FM>(r[g].u1[k] - n1[k], r[g].u2[k] - n2[k]);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < PX; ++k) {
        r[g].u1[k] = n1[k];
        r[g].u2[k] = n2[k];
        if (G) r[g].u3[k] = n3[k];
      }
      L(2, row) = pack(n1);
      L(3, row) = pack(n2);
      if (G) L(5, row) = pack(n3);
    }
    __syncthreads();
    // ---- estimateDualVariables
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int row = rr + g * HALF;
      const int rowd = row < RH - 1 ? row + 1 : RH - 1;
      const bool has_down = Y[g] + 1 < a.H;
      float d1[PX], d2[PX], d3[PX];
      unpack(d1, L(2, rowd));
      unpack(d2, L(3, rowd));
      float q11[PX], q12[PX], q21[PX], q22[PX], q31[PX], q32[PX];
      dual_component<PX, false, FM>(r[g].u1, d1, has_down, X, a.W, a.taut, r[g].p11, r[g].p12, q11, q12, a.taut_small);
      dual_component<PX, false, FM>(r[g].u2, d2, has_down, X, a.W, a.taut, r[g].p21, r[g].p22, q21, q22, a.taut_small);
      if (G) {
        unpack(d3, L(5, rowd));
        dual_component<PX, false, FM>(r[g].u3, d3, has_down, X, a.W, a.taut, r[g].p31, r[g].p32, q31, q32, a.taut_small);
      }
#pragma unroll
      for (int k = 0; k < PX; ++k) {
        r[g].p11[k] = q11[k]; r[g].p12[k] = q12[k];
        r[g].p21[k] = q21[k]; r[g].p22[k] = q22[k];
        if (G) { r[g].p31[k] = q31[k]; r[g].p32[k] = q32[k]; }
      }
    }
    if (!last) {
      // p12/p22 planes are not read during the projection phase: publish the new rows
      // now; the barrier orders them before the next estimateU and orders this
      // phase's u1/u2 reads before the next phase's u1/u2 writes.
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int row = rr + g * HALF;
        L(0, row) = pack(r[g].p12);
        L(1, row) = pack(r[g].p22);
        if (G) L(4, row) = pack(r[g].p32);
      }
      __syncthreads();
    }
  }

  // ---- store the exact interior: region cols 4..59, rows K..RH-K-1, inside the image
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    if (out_ok[g]) {
      const size_t off = (size_t)Y[g] * a.P + X;
      stv<PX>(a.u1d, off, r[g].u1);
      stv<PX>(a.u2d, off, r[g].u2);
      stv<PX>(a.p11d, off, r[g].p11);
      stv<PX>(a.p12d, off, r[g].p12);
      stv<PX>(a.p21d, off, r[g].p21);
      stv<PX>(a.p22d, off, r[g].p22);
      if (G) {
        stv<PX>(a.u3d, off, r[g].u3);
        stv<PX>(a.p31d, off, r[g].p31);
        stv<PX>(a.p32d, off, r[g].p32);
      }
    }
  }
  if (a.calc_err) {
    __shared__ double red[NT / kWave];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      double sum = 0.0;
      for (int i = 0; i < NT / kWave; ++i) sum += red[i];
      a.partials[blockIdx.x] = sum;
    }
  }
}

template <bool G, int RH, int NG, int PX = 4, int FM = 0>
__global__ __launch_bounds__((64 / PX) * RH / NG, PX == 2 ? 8 : 1) void k_iterate_tb(TBArgs t) {
  constexpr int LPR = 64 / PX;
  constexpr int HALF = RH / NG;
  constexpr int NPL = G ? 6 : 4;                 // LDS planes
  __shared__ typename VecT<PX>::type lds[NPL * RH * LPR];
  const IterArgs &a = t.it;
  if (gated_off(a.gate, a.gate_seq)) return;   // whole grid
  const int tid = threadIdx.x;
  const int c4 = tid % LPR;
  const int rr = tid / LPR;
  int bx, by;
  tile_of_block(blockIdx.x, gridDim.x, t.tiles_x, gridDim.x / t.tiles_x, bx, by);
  const int K = t.niter;
  const int xr0 = bx * 56 - 4;                   // region origin (16-B aligned)
  const int yr0 = by * t.out_h - K;
  const int X = xr0 + PX * c4;                   // first image column of this thread
  const int xa = imin(imax(X, 0), a.P - PX);
  Row<G, PX> r[NG];
  int Y[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    Y[g] = yr0 + rr + g * HALF;
    const int ya = imin(imax(Y[g], 0), a.H - 1);
    load_row<G, PX>(r[g], a, (size_t)ya * a.P + xa);
  }
  tb_iterate_store<G, RH, NG, PX, FM>(t, lds, r, Y, X, c4, rr);
}

// ---------------------------------------------------------------- K6+K8, tall blocked regions
// k_iterate_tb4<FM>: one pass of K <= 4 iterations over a 64 x 48 region (4-px x halo, K-row
// y halo: 56 x (48 - 2K) output px), 512 threads.  Each thread owns 2 px of NR = 3
// CONSECUTIVE rows, so the y-neighbours inside its rows are registers and only the rows
// between two threads go through LDS: the last row's p12 / p22 (estimateU's p at y-1 of the
// next thread's first row) and the first row's u1 / u2 (the projection's u at y+1 of the
// previous thread's last row) -- 16 KB, 2 barriers per iteration as in k_iterate_tb, with 6 px
// of work per thread between them.  Against k_iterate_tb's 64 x 32 regions the halo
// recompute falls from 1.52x to 1.37x at K = 4, at 4 waves per SIMD (128 VGPRs) instead of
// 8: the same time per pass on C2's level 4, and +0.7 % in flight.  (Four rows per
// thread, 64 x 64 regions, needs 165 VGPRs -- one block per CU -- and was 49 % slower.)  Same
// estimate_u / dual_component arithmetic, so the same bits (the region-edge rows take their
// own row as the neighbour, as k_iterate_tb's LDS clamp does; no stored cell depends on them).
constexpr int kTb4Groups = 16;   // row groups (threads per column) of a region (32: -6 %, r5)
constexpr int kTb4RowsPerThread = 3;

// The iterations of one k_iterate_tb4 region.  IN: the region lies inside the image with a
// margin (x > 0, y > 0, x + 1 < W, y + 1 < H for every px), so the border forms are constant
// and the divergence / projection selects fold away: the same operations as the general
// path takes for such px, hence the same bits.  The edge regions (the outer ring of tiles)
// take the general path.
template <int FM, int NR, bool IN>
__device__ __forceinline__ void tb4_iterations(Row<false, 2> (&r)[NR], const int (&Y)[NR],
                                               const bool (&out_ok)[NR], float2 (&lds)[4][kTb4Groups][32],
                                               const IterArgs &a, int K, int X, int q, int c4,
                                               double &acc) {
  constexpr int PX = 2, NGR = kTb4Groups;
  for (int it = 0; it < K; ++it) {
    const bool last = it == K - 1;
    // ---- estimateU (p^{n-1} at y-1: the row above in registers, or the previous group's
    // last row from LDS; u^{n-1} -> u^n in place)
    lds[0][q][c4] = pack(r[NR - 1].p12);
    lds[1][q][c4] = pack(r[NR - 1].p22);
    __syncthreads();
    float up12[PX], up22[PX], zero3[PX];
    zerov<PX>(zero3);
    if (q > 0) {
      unpack(up12, lds[0][q - 1][c4]);
      unpack(up22, lds[1][q - 1][c4]);
    } else {   // region row 0: its own row (k_iterate_tb's clamp)
#pragma unroll
      for (int k = 0; k < PX; ++k) up12[k] = r[0].p12[k], up22[k] = r[0].p22[k];
    }
    // every row's estimateU reads p of the row above, which no row's estimateU changes
#pragma unroll
    for (int g = 0; g < NR; ++g) {
      float n1[PX], n2[PX], n3[PX];
      if (g == 0)
        estimate_u<false, PX, FM>(r[0], up12, up22, zero3, IN ? 1 : X, IN ? 1 : Y[0], a, n1, n2, n3);
      else
        estimate_u<false, PX, FM>(r[g], r[g - 1].p12, r[g - 1].p22, zero3, IN ? 1 : X, IN ? 1 : Y[g], a,
                                  n1, n2, n3);
      if (last && a.calc_err && out_ok[g]) {
#pragma unroll
        for (int k = 0; k < PX; ++k)
          if (X + k < a.W) acc += (double)residual_px<FM>(r[g].u1[k] - n1[k], r[g].u2[k] - n2[k]);
      }
#pragma unroll
      for (int k = 0; k < PX; ++k) {
        r[g].u1[k] = n1[k];
        r[g].u2[k] = n2[k];
      }
    }
    // ---- estimateDualVariables (u^n at y+1: the row below, or the next group's first row)
    lds[2][q][c4] = pack(r[0].u1);
    lds[3][q][c4] = pack(r[0].u2);
    __syncthreads();
    float d1[PX], d2[PX];
    if (q < NGR - 1) {
      unpack(d1, lds[2][q + 1][c4]);
      unpack(d2, lds[3][q + 1][c4]);
    } else {   // region bottom row: its own row
#pragma unroll
      for (int k = 0; k < PX; ++k) d1[k] = r[NR - 1].u1[k], d2[k] = r[NR - 1].u2[k];
    }
#pragma unroll
    for (int g = 0; g < NR; ++g) {
      const bool has_down = IN || Y[g] + 1 < a.H;
      const int xd = IN ? 0 : X, wd = IN ? 64 : a.W;   // IN: has_right holds for both px
      float q11[PX], q12[PX], q21[PX], q22[PX];
      if (g < NR - 1) {
        dual_component<PX, false, FM>(r[g].u1, r[g + 1].u1, has_down, xd, wd, a.taut, r[g].p11, r[g].p12, q11, q12, a.taut_small);
        dual_component<PX, false, FM>(r[g].u2, r[g + 1].u2, has_down, xd, wd, a.taut, r[g].p21, r[g].p22, q21, q22, a.taut_small);
      } else {
        dual_component<PX, false, FM>(r[g].u1, d1, has_down, xd, wd, a.taut, r[g].p11, r[g].p12, q11, q12, a.taut_small);
        dual_component<PX, false, FM>(r[g].u2, d2, has_down, xd, wd, a.taut, r[g].p21, r[g].p22, q21, q22, a.taut_small);
      }
#pragma unroll
      for (int k = 0; k < PX; ++k) {
        r[g].p11[k] = q11[k]; r[g].p12[k] = q12[k];
        r[g].p21[k] = q21[k]; r[g].p22[k] = q22[k];
      }
    }
    // the next iteration's first barrier orders these LDS reads before the rewrite
  }
}

template <int FM, int NR, bool IN>
__device__ __forceinline__ void tb4_body(const TBArgs &t, float2 (&lds)[4][kTb4Groups][32], int xr0,
                                         int yr0) {
  constexpr int PX = 2, LPR = 32, NGR = kTb4Groups, kTb4Rows = NR * NGR;
  constexpr int HALO = 4 / PX;   // lanes of the 4-px x halo
  const IterArgs &a = t.it;
  const int tid = threadIdx.x;
  const int c4 = tid % LPR;
  const int q = tid / LPR;                     // row group: region rows NR q .. NR q + NR - 1
  const int K = t.niter;
  const int X = xr0 + PX * c4;
  const int xa = imin(imax(X, 0), a.P - PX);
  Row<false, PX> r[NR];
  int Y[NR];
  bool out_ok[NR];
#pragma unroll
  for (int g = 0; g < NR; ++g) {
    const int row = NR * q + g;
    Y[g] = yr0 + row;
    const int ya = imin(imax(Y[g], 0), a.H - 1);
    load_row<false, PX>(r[g], a, (size_t)ya * a.P + xa);
    out_ok[g] = c4 >= HALO && c4 < LPR - HALO && row >= K && row < kTb4Rows - K && Y[g] >= 0 &&
                Y[g] < a.H && X < a.W;
  }
  double acc = 0.0;
  tb4_iterations<FM, NR, IN>(r, Y, out_ok, lds, a, K, X, q, c4, acc);
#pragma unroll
  for (int g = 0; g < NR; ++g) {
    if (out_ok[g]) {
      const size_t off = (size_t)Y[g] * a.P + X;
      stv<PX>(a.u1d, off, r[g].u1);
      stv<PX>(a.u2d, off, r[g].u2);
      stv<PX>(a.p11d, off, r[g].p11);
      stv<PX>(a.p12d, off, r[g].p12);
      stv<PX>(a.p21d, off, r[g].p21);
      stv<PX>(a.p22d, off, r[g].p22);
    }
  }
  if (a.calc_err) {
    __shared__ double red[32 * NGR / kWave];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      double sum = 0.0;
      for (int i = 0; i < 32 * NGR / kWave; ++i) sum += red[i];
      a.partials[blockIdx.x] = sum;
    }
  }
}

template <int FM, int NR = kTb4RowsPerThread>
__global__ __launch_bounds__(32 * kTb4Groups, 4) void k_iterate_tb4(TBArgs t) {
  __shared__ float2 lds[4][kTb4Groups][32];   // [p12 last, p22 last, u1 first, u2 first][group][lane]
  if (gated_off(t.it.gate, t.it.gate_seq)) return;   // whole grid
  int bx, by;
  tile_of_block(blockIdx.x, gridDim.x, t.tiles_x, gridDim.x / t.tiles_x, bx, by);
  const int xr0 = bx * 56 - 4;
  const int yr0 = by * t.out_h - t.niter;
  // wave-uniform: the whole region inside the image with a 1-px margin (tb4_iterations' IN)
  if (xr0 >= 1 && yr0 >= 1 && xr0 + 64 < t.it.W && yr0 + NR * kTb4Groups < t.it.H)
    tb4_body<FM, NR, true>(t, lds, xr0, yr0);
  else
    tb4_body<FM, NR, false>(t, lds, xr0, yr0);
}

// ---------------------------------------------------------------- K6+K8 wavefront pipeline
// k_iterate_roll<G, K, PX>: K consecutive primal-dual iterations in ONE streaming pass.
// One wavefront owns a column band of 64*PX px (PX adjacent px per lane) of one row
// segment and walks down it, one row per step; no LDS, no barriers.
//
// Dependencies of iteration n of a pass (Jacobi: reads n-1, writes n):
//   u^n(y) <- u^{n-1}(y), p^{n-1}(y), p^{n-1}(x-1, y), p^{n-1}(y-1)      (estimateU)
//   p^n(y) <- p^{n-1}(y), u^n(y), u^n(x+1, y), u^n(y+1)                    (estimateDual)
// so once input row r is loaded, stage n computes u^n at row r-n+1 and p^n at row r-n.
// Per stage the wave keeps the two newest u rows and p rows in registers, plus the warp
// constants of the K newest input rows, and it stores u^K and p^K.  x neighbours across
// lanes are DPP wavefront shifts.  Every iteration invalidates one px at each band edge,
// so a band carries a halo of K px (rounded up to whole lanes) on both sides and stores
// its interior; a segment starts K rows above its output rows (their p^{n-1}(y-1) is
// missing) and reads K rows below them.  At the image border OpenCV's clamp / special
// divergence forms apply and nothing is invalidated.  HBM per px and pass: 36 B x
// 64PX/(64PX - 2 halo) x (rows + 2K)/rows loaded, 24 B stored -- for any K.  The pass is
// VALU-bound for K >= 3 (the halo is recomputed, so a small one matters) and HBM-bound for
// K <= 2.  Arithmetic is estimate_u_px / dual_px, the same as the other iteration kernels
// (bit-identical results).
constexpr int kRollMax = 4;
constexpr int kRollAhead = 2;   // input rows loaded ahead of the row entering the pipeline
// rows loaded ahead by k_iterate_roll<.., PX>: 16-byte loads (PX = 4) keep as many bytes in
// flight one row ahead as 8-byte loads two rows ahead, with one ring row less
template <int K, int PX>
constexpr int roll_ahead() { return PX == 4 ? 1 : kRollAhead; }
// ... by kb_iterate_roll: one row for the 3- and 4-iteration passes on 128-px bands (174
// instead of 189 VGPRs, the same 2 wavefronts per SIMD): strips +1.1 %, where the single-pair
// passes measured -0.3 % (profiles/r4/ab/roll_ahead_r4l/)
template <int K, int PX>
constexpr int kb_roll_ahead() { return K >= 3 && PX == 2 ? 1 : roll_ahead<K, PX>(); }

// The planes of a streaming pass as five buffer groups, one 4-SGPR descriptor each: the
// warp constants (I1wx, I1wy, rho), the u set read and the u set written (u1, u2, u3), the
// p set read and the p set written (p11, p12, p21, p22, p31, p32).  Plane k of a group sits
// at byte offset k * pstride from its base (the arena lays a set's planes out contiguously)
// and is addressed through the scalar offset.  One descriptor per plane (16) spilled SGPRs
// into VGPR lanes in the unrolled pipelines.  A group spans < 2 GiB (the host checks), so a
// masked store's offset kOOB lands past its records whatever the scalar offset.
struct RollBufs {
  const float *c;          // I1wx | I1wy | rho
  const float *us, *ps;    // u, p read
  float *ud, *pd;          // u, p written
  unsigned cb, ub, pb;     // group bytes (descriptor records) of c, u, p
  unsigned pstride;        // bytes between the planes of a group
};

struct RollArgs {
  RollBufs b;
  IterArgs it;
  int bands;      // column bands per row: ceil(W / (64 PX - 2 halo))
  int seg_rows;   // output rows per segment
  int waves;      // bands * segments
};

// lane i <- lane i-1 (DPP wave_shr:1; lane 0 gets 0).  bound_ctrl: the lane with no source
// is written 0 by the DPP move itself, so no "old" value has to be put in its destination
// first (one v_mov per shift)
__device__ __forceinline__ float from_left(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, true));
}
// lane i <- lane i+1 (DPP wave_shl:1; lane 63 gets 0)
__device__ __forceinline__ float from_right(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, true));
}

template <bool G, int PX>
struct RollIn {   // one input row at this lane's PX px
  float wx[PX], wy[PX], rh[PX], u1[PX], u2[PX], u3[PX];
  float p11[PX], p12[PX], p21[PX], p22[PX], p31[PX], p32[PX];
};

// p is loaded unconditionally (a branch here would make the compiler's wait counts
// conservative for every row); when p == 0 (first pass of a level) its column offset voffp is
// kOOB, so the buffer loads return +0.0f with no per-px select.
template <bool G, int PX>
__device__ __forceinline__ void roll_load(RollIn<G, PX> &v, const RollBufs &B, unsigned soff,
                                          unsigned voff, unsigned voffp) {
  const unsigned ps = B.pstride;
  bload<PX>(v.wx, B.c, B.cb, voff, soff);
  bload<PX>(v.wy, B.c, B.cb, voff, soff + ps);
  bload<PX>(v.rh, B.c, B.cb, voff, soff + 2 * ps);
  bload<PX>(v.u1, B.us, B.ub, voff, soff);
  bload<PX>(v.u2, B.us, B.ub, voff, soff + ps);
  if (G) bload<PX>(v.u3, B.us, B.ub, voff, soff + 2 * ps);
  bload<PX>(v.p11, B.ps, B.pb, voffp, soff);
  bload<PX>(v.p12, B.ps, B.pb, voffp, soff + ps);
  bload<PX>(v.p21, B.ps, B.pb, voffp, soff + 2 * ps);
  bload<PX>(v.p22, B.ps, B.pb, voffp, soff + 3 * ps);
  if (G) {
    bload<PX>(v.p31, B.ps, B.pb, voffp, soff + 4 * ps);
    bload<PX>(v.p32, B.ps, B.pb, voffp, soff + 5 * ps);
  }
}

// Pipeline registers (see k_iterate_roll).  Index [n][j]: stage n, px j of the lane.
template <bool G, int K, int PX>
struct RollPipe {
  float U1c[K + 1][PX], U2c[K + 1][PX], U3c[K + 1][PX];   // u^n(r-n+1)
  float U1p[K + 1][PX], U2p[K + 1][PX], U3p[K + 1][PX];   // u^n(r-n); [0] = input u(r)
  float P11c[K + 1][PX], P12c[K + 1][PX], P21c[K + 1][PX], P22c[K + 1][PX];   // p^n(r-n)
  float P31c[K + 1][PX], P32c[K + 1][PX];                                     // [0] = input p(r)
  float P11p[K + 1][PX], P12p[K + 1][PX], P21p[K + 1][PX], P22p[K + 1][PX];   // p^n(r-n-1)
  float P31p[K + 1][PX], P32p[K + 1][PX];
  float CX[K][PX], CY[K][PX], CR[K][PX];   // warp constants of input rows r, r-1, ...
};

// Lane geometry of a band: lane l holds px X + j, X = X0 + PX*l.
struct RollLane {
  int X;             // first px of the lane
  unsigned vload;    // byte offset of the (clamped) load column
  unsigned vloadp;   // the p loads' column offset: kOOB when p = 0 (the first pass of a level),
                     // where out-of-range buffer loads return +0.0f
  unsigned vst;      // byte offset of the lane's store column (out lanes only)
  bool out;          // lane is in the band interior and its first px inside the image
                     // (a second px at x = W lands in the row's pitch padding, which no
                     // in-image px ever reads)
  int ys, ye;        // output rows of the segment
  bool c0;           // wave-uniform: some lane of the wave holds a column <= 0 (the first band)
};

// x neighbours of px j of the lane: left = px j-1 (previous lane's last px for j = 0),
// right = px j+1 (next lane's first px for the last px).
template <int PX>
__device__ __forceinline__ float left_of(const float (&v)[PX], int j) {
  return j == 0 ? from_left(v[PX - 1]) : v[j - 1];
}
template <int PX>
__device__ __forceinline__ float right_of(const float (&v)[PX], int j) {
  return j == PX - 1 ? from_right(v[0]) : v[j + 1];
}

// One step of the pipeline: input row r (in `in`) enters stage 0, every stage advances
// one row, and input row r + kRollAhead is loaded into `ahead` (a ring of kRollAhead + 1
// rows, so no register holding a load in flight is ever copied).  Every load and store is
// issued unconditionally (rows clamped; masked stores use an out-of-range offset, which
// the buffer unit drops), so the compiler keeps this step's stores and the younger loads
// in flight with counted waits.  Stages run every step: before a segment's first rows
// reach them and past the image bottom they compute values no stored cell depends on (see
// the dependency list above; the border forms select, never combine).
// VIN: in.u1 / u2 / u3 hold stage 1's v = u^0 + TH step (th_px, computed by the caller)
// instead of u^0
// MID (k_iterate_roll_mid): stage 2 also sums its residual into *accm
template <bool G, int K, int PX, bool VIN = false, int FM = 0, bool MID = false>
__device__ __forceinline__ void roll_advance(RollPipe<G, K, PX> &S, const RollIn<G, PX> &in,
                                             const IterArgs &a, const RollBufs &B, int r,
                                             const RollLane &L, unsigned rowb, double &acc,
                                             double *accm = nullptr);

template <bool G, int K, int PX, int FM, int AH>
__device__ __forceinline__ void roll_step(RollPipe<G, K, PX> &S, const RollIn<G, PX> &in,
                                          RollIn<G, PX> &ahead, const IterArgs &a,
                                          const RollBufs &B, int r, const RollLane &L,
                                          unsigned rowb, double &acc) {
  roll_load<G, PX>(ahead, B, (unsigned)imin(r + AH, a.H - 1) * rowb, L.vload, L.vloadp);
  // keep the loads of row r + roll_ahead ahead of this step's stores: waiting for them
  // roll_ahead steps later then leaves the younger stores and loads in flight (vmcnt
  // counts in issue order)
  __builtin_amdgcn_sched_barrier(0);
  roll_advance<G, K, PX, false, FM>(S, in, a, B, r, L, rowb, acc);
}

// The compute and stores of one step: input row r (in `in`) enters stage 0 and every
// stage advances one row.
template <bool G, int K, int PX, bool VIN, int FM, bool MID>
__device__ __forceinline__ void roll_advance(RollPipe<G, K, PX> &S, const RollIn<G, PX> &in,
                                             const IterArgs &a, const RollBufs &B, int r,
                                             const RollLane &L, unsigned rowb, double &acc,
                                             double *accm) {
  const unsigned ps = B.pstride;
  static_assert(!VIN || K >= 2, "stage 1's u^0 (replaced by v) is the K = 1 residual's input");
  static_assert(!MID || (!G && K == 4 && !VIN), "the mid check: the 4-iteration pass, gamma = 0");
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    // shift every stage one row down
#pragma unroll
    for (int n = K; n >= 1; --n) {
      S.U1p[n][j] = S.U1c[n][j]; S.U2p[n][j] = S.U2c[n][j]; if (G) S.U3p[n][j] = S.U3c[n][j];
    }
#pragma unroll
    for (int n = K - 1; n >= 0; --n) {
      S.P11p[n][j] = S.P11c[n][j]; S.P12p[n][j] = S.P12c[n][j];
      S.P21p[n][j] = S.P21c[n][j]; S.P22p[n][j] = S.P22c[n][j];
      if (G) { S.P31p[n][j] = S.P31c[n][j]; S.P32p[n][j] = S.P32c[n][j]; }
    }
#pragma unroll
    for (int n = K - 1; n >= 1; --n) {
      S.CX[n][j] = S.CX[n - 1][j]; S.CY[n][j] = S.CY[n - 1][j]; S.CR[n][j] = S.CR[n - 1][j];
    }
    // (p = 0 on a level's first pass: the loads returned +0, RollLane::vloadp)
    S.CX[0][j] = in.wx[j]; S.CY[0][j] = in.wy[j]; S.CR[0][j] = in.rh[j];
    S.U1p[0][j] = in.u1[j]; S.U2p[0][j] = in.u2[j]; S.U3p[0][j] = G ? in.u3[j] : 0.0f;
    S.P11c[0][j] = in.p11[j]; S.P12c[0][j] = in.p12[j];
    S.P21c[0][j] = in.p21[j]; S.P22c[0][j] = in.p22[j];
    S.P31c[0][j] = G ? in.p31[j] : 0.0f; S.P32c[0][j] = G ? in.p32[j] : 0.0f;
  }

#pragma unroll
  for (int n = 1; n <= K; ++n) {
    const int yU = r - n + 1;    // estimateU row of stage n
    const bool stU = L.out && yU >= L.ys && yU < L.ye;
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      float n1, n2, n3 = 0.0f;
      if (VIN && n == 1)
        u_from_v<G, FM, true>(S.U1p[0][j], S.U2p[0][j], S.U3p[0][j], S.P11c[0][j],
                    left_of<PX>(S.P11c[0], j), S.P12c[0][j], S.P12p[0][j], S.P21c[0][j],
                    left_of<PX>(S.P21c[0], j), S.P22c[0][j], S.P22p[0][j], S.P31c[0][j],
                    G ? left_of<PX>(S.P31c[0], j) : 0.0f, S.P32c[0][j], S.P32p[0][j], L.X + j,
                    yU, a, n1, n2, n3, L.c0);
      else
        estimate_u_px<G, FM, false, true>(S.CX[n - 1][j], S.CY[n - 1][j], S.CR[n - 1][j], S.U1p[n - 1][j],
                         S.U2p[n - 1][j], S.U3p[n - 1][j], S.P11c[n - 1][j],
                         left_of<PX>(S.P11c[n - 1], j), S.P12c[n - 1][j], S.P12p[n - 1][j],
                         S.P21c[n - 1][j], left_of<PX>(S.P21c[n - 1], j), S.P22c[n - 1][j],
                         S.P22p[n - 1][j], S.P31c[n - 1][j],
                         G ? left_of<PX>(S.P31c[n - 1], j) : 0.0f, S.P32c[n - 1][j],
                         S.P32p[n - 1][j], L.X + j, yU, a, n1, n2, n3, L.c0);
      if (n == K && a.calc_err) {
        const float e = residual_px<FM>(S.U1p[n - 1][j] - n1, S.U2p[n - 1][j] - n2);
        acc += stU && L.X + j < a.W ? (double)e : 0.0;
      }
      if (MID && n == 2) {   // the check after this pass's first 2 iterations
        const float e = residual_px<FM>(S.U1p[n - 1][j] - n1, S.U2p[n - 1][j] - n2);
        *accm += stU && L.X + j < a.W ? (double)e : 0.0;
      }
      S.U1c[n][j] = n1; S.U2c[n][j] = n2; if (G) S.U3c[n][j] = n3;
    }
    // below the image: u^n(yU) := u^n(yU - 1), so the projection's y-difference at row H-1
    // is exactly +0 (OpenCV's has_down form) with no per-px select; rows >= H are never
    // stored (a wave-uniform branch, taken only while a segment drains past the bottom)
    if (yU >= a.H) {
#pragma unroll
      for (int j = 0; j < PX; ++j) {
        S.U1c[n][j] = S.U1p[n][j]; S.U2c[n][j] = S.U2p[n][j]; if (G) S.U3c[n][j] = S.U3p[n][j];
      }
    }
    if (n == K) {
      const unsigned vo = stU ? (unsigned)yU * rowb + L.vst : kOOB;
      bstorev<PX>(B.ud, B.ub, vo, S.U1c[n]);
      bstorev<PX>(B.ud, B.ub, vo, S.U2c[n], ps);
      if (G) bstorev<PX>(B.ud, B.ub, vo, S.U3c[n], 2 * ps);
    }

    const int yD = r - n;        // estimateDualVariables row of stage n
    // has_down: rows below the image repeat row H-1 (above)
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      const bool has_right = L.X + j + 1 < a.W;
      dual_px<false, false, FM>(S.U1p[n][j], right_of<PX>(S.U1p[n], j), S.U1c[n][j], has_right,
                                true, a.taut, S.P11p[n - 1][j], S.P12p[n - 1][j],
                                S.P11c[n][j], S.P12c[n][j], a.taut_small);
      dual_px<false, false, FM>(S.U2p[n][j], right_of<PX>(S.U2p[n], j), S.U2c[n][j], has_right,
                                true, a.taut, S.P21p[n - 1][j], S.P22p[n - 1][j],
                                S.P21c[n][j], S.P22c[n][j], a.taut_small);
      if (G)
        dual_px<false, false, FM>(S.U3p[n][j], right_of<PX>(S.U3p[n], j), S.U3c[n][j], has_right, true,
                a.taut, S.P31p[n - 1][j], S.P32p[n - 1][j], S.P31c[n][j], S.P32c[n][j], a.taut_small);
    }
    // above the image: p^n(yD < 0) := +0, the p2u the next stage's divergence reads on row 0
    // (divergence<YZ>; OpenCV's y == 0 form).  Only the first K steps of a segment that
    // starts at row 0 take this wave-uniform branch
    if (n < K && yD < 0) {
#pragma unroll
      for (int j = 0; j < PX; ++j) {
        S.P11c[n][j] = S.P12c[n][j] = S.P21c[n][j] = S.P22c[n][j] = 0.0f;
        if (G) S.P31c[n][j] = S.P32c[n][j] = 0.0f;
      }
    }
    if (n == K) {
      const unsigned vo = L.out && yD >= L.ys && yD < L.ye ? (unsigned)yD * rowb + L.vst : kOOB;
      bstorev<PX>(B.pd, B.pb, vo, S.P11c[n]);
      bstorev<PX>(B.pd, B.pb, vo, S.P12c[n], ps);
      bstorev<PX>(B.pd, B.pb, vo, S.P21c[n], 2 * ps);
      bstorev<PX>(B.pd, B.pb, vo, S.P22c[n], 3 * ps);
      if (G) {
        bstorev<PX>(B.pd, B.pb, vo, S.P31c[n], 4 * ps);
        bstorev<PX>(B.pd, B.pb, vo, S.P32c[n], 5 * ps);
      }
    }
  }
}

// ---- LDS-staged input rows (LDSR; the 3- and 4-iteration passes on 128-px bands).
// The register ring of rows loaded ahead (RollIn A, Bx, C: 54 VGPRs of <4, 2>'s 189) is
// what holds those passes at 2 wavefronts per SIMD, and they are bound per wavefront (one
// wavefront per SIMD: 1.65x the time).  Here the rows go HBM -> LDS by the
// buffer unit's LDS path (buffer_load_dwordx4 ... lds: 1 KiB per wave-instruction, lanes
// 0-31 one plane's 128 px, lanes 32-63 the next plane's), two slots per wavefront: the
// row read at step r is at least 2 steps old, and the slot read is refilled (row r + 2)
// right after the read.  The reads are inline ds_read_b64 (the lane's 2 px of each of the 9
// planes) with their own lgkmcnt wait, and the wait for the row's DMA is a counted vmcnt
// written here: the compiler's wait pass, which would otherwise wait for every DMA in
// flight before any LDS read, sees neither.  Same operands, same arithmetic: same bits.
constexpr int kRollLdsSlot = 1280;                 // floats: 5 pieces of 2 x 128
constexpr int kRollLdsWave = 2 * kRollLdsSlot;     // two slots per wavefront
constexpr int kRollDmaPerRow = 5;                  // DMA pieces per row (G = false)
constexpr int kRollStPerStep = 6;                  // b64 stores per step: u1, u2, p11..p22
#ifndef TVL1_ROLL_LDS
#define TVL1_ROLL_LDS 1
#endif
template <bool G, int K, int PX>
constexpr bool roll_lds_on() { return TVL1_ROLL_LDS && !G && K >= 3 && PX == 2; }

struct RollDma {   // per-lane byte offsets of the 5 pieces (the row in the scalar offset)
  unsigned c1, c2, u, p1, p2;
};

__device__ __forceinline__ void roll_dma_piece(const float *base, unsigned bytes, float *lds,
                                               unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(plane_rsrc(base, bytes),
                                           (__attribute__((address_space(3))) void *)lds, 16,
                                           (int)voff, (int)soff, 0, 0);
}

// row (scalar offset soff) -> LDS slot: [wx | wy] [rh | -] [u1 | u2] [p11 | p12] [p21 | p22]
__device__ __forceinline__ void roll_dma_row(float *slot, const RollBufs &B, unsigned soff,
                                             const RollDma &D) {
  roll_dma_piece(B.c, B.cb, slot, D.c1, soff);
  roll_dma_piece(B.c, B.cb, slot + 256, D.c2, soff);
  roll_dma_piece(B.us, B.ub, slot + 512, D.u, soff);
  roll_dma_piece(B.ps, B.pb, slot + 768, D.p1, soff);
  roll_dma_piece(B.ps, B.pb, slot + 1024, D.p2, soff);
}

// the lane's 2 px of the 9 planes of a slot (addr: LDS byte address of the slot + 8 * lane)
__device__ __forceinline__ void roll_lds_read(RollIn<false, 2> &in, unsigned addr, bool pz) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 wx, wy, rh, u1, u2, p11, p12, p21, p22;
  asm volatile(
      "ds_read_b64 %0, %9\n"
      "ds_read_b64 %1, %9 offset:512\n"
      "ds_read_b64 %2, %9 offset:1024\n"
      "ds_read_b64 %3, %9 offset:2048\n"
      "ds_read_b64 %4, %9 offset:2560\n"
      "ds_read_b64 %5, %9 offset:3072\n"
      "ds_read_b64 %6, %9 offset:3584\n"
      "ds_read_b64 %7, %9 offset:4096\n"
      "ds_read_b64 %8, %9 offset:4608\n"
      "s_waitcnt lgkmcnt(0)"
      // early-clobber: the reads after the first one still read the address operand
      : "=&v"(wx), "=&v"(wy), "=&v"(rh), "=&v"(u1), "=&v"(u2), "=&v"(p11), "=&v"(p12), "=&v"(p21),
        "=&v"(p22)
      : "v"(addr)
      : "memory");
  in.wx[0] = wx.x; in.wx[1] = wx.y;
  in.wy[0] = wy.x; in.wy[1] = wy.y;
  in.rh[0] = rh.x; in.rh[1] = rh.y;
  in.u1[0] = u1.x; in.u1[1] = u1.y;
  in.u2[0] = u2.x; in.u2[1] = u2.y;
  in.u3[0] = in.u3[1] = 0.0f;
  // p = 0 on a level's first pass (its pieces were loaded from kOOB)
  in.p11[0] = pz ? 0.0f : p11.x; in.p11[1] = pz ? 0.0f : p11.y;
  in.p12[0] = pz ? 0.0f : p12.x; in.p12[1] = pz ? 0.0f : p12.y;
  in.p21[0] = pz ? 0.0f : p21.x; in.p21[1] = pz ? 0.0f : p21.y;
  in.p22[0] = pz ? 0.0f : p22.x; in.p22[1] = pz ? 0.0f : p22.y;
  in.p31[0] = in.p31[1] = in.p32[0] = in.p32[1] = 0.0f;
}

// One step at input row r from LDS slot `slot` (LDS byte address `addr` + 8 * lane): wait for
// the row's DMA (issued 2 steps ago: the stores of that step, the next row's pieces and the
// stores of the step between are younger), read it, refill the slot with row r + 2, advance.
template <int K, int FM, bool MID = false>
__device__ __forceinline__ void roll_step_lds(RollPipe<false, K, 2> &S, float *slot, unsigned addr,
                                              const IterArgs &a, const RollBufs &B, int r,
                                              const RollLane &L, unsigned rowb, const RollDma &D,
                                              double &acc, double *accm = nullptr) {
  static_assert(2 * kRollStPerStep + kRollDmaPerRow == 17, "the vmcnt below");
  asm volatile("s_waitcnt vmcnt(17)" ::: "memory");
  RollIn<false, 2> in;
  roll_lds_read(in, addr, a.p_zero != 0);
  roll_dma_row(slot, B, (unsigned)imin(r + 2, a.H - 1) * rowb, D);
  __builtin_amdgcn_sched_barrier(0);
  roll_advance<false, K, 2, false, FM, MID>(S, in, a, B, r, L, rowb, acc, accm);
}

// halo of a band: K px, rounded up to whole lanes' worth of px (8-byte aligned loads)
template <int K, int PX>
constexpr int roll_halo() { return (K + PX - 1) / PX * PX; }

// The pass of one wavefront (band / segment wid < ra.waves); k_iterate_roll and the
// batched kb_iterate_roll differ only in how they find their planes and wid.
// PRIO: issue priority falling with the segment's progress (progress_prio), for
// k_iterate_roll: a launch is one round of the resident slots, and at equal priority the
// waves dispatched last on a SIMD would finish last (one C2 pair alone: <4,2> 317 -> 307 us,
// <2,2> 52.2 -> 50.5 us per launch; in flight neutral; the batched passes keep 0, where it
// measured -0.7 %: profiles/r3/ab_roll_prio.txt)
// AH: input rows loaded ahead (1: a 2-row ring, 2: a 3-row ring); LDSR: rows staged in
// LDS (lds: this wavefront's kRollLdsWave floats), see roll_step_lds
// MID (k_iterate_roll_mid, LDSR only): the residual after the first 2 of the 4 iterations
// too, to partials[waves + wid]
template <bool G, int K, int PX, int FM, int PRIO = 0, int AH = roll_ahead<K, PX>(),
          bool LDSR = false, bool MID = false>
__device__ __forceinline__ void roll_body(const RollArgs &ra, int wid, float *lds = nullptr) {
  static_assert(!MID || LDSR, "the mid check rides on the LDS-staged 4-iteration pass");
  constexpr int HALO = roll_halo<K, PX>();
  constexpr int BW = 64 * PX;            // band width (px)
  // The long pipelines (and the gamma ones) run at 2 waves/SIMD with VGPRs to spare but
  // SGPRs at the 106 cap: their float parameters live in VGPRs (an opaque copy, same
  // values), which ends the SGPR spills of k_iterate_roll<4, 2> and <2, 4>.
  IterArgs a = ra.it;
  if (G || K * PX >= 8) {
    asm volatile("v_mov_b32 %0, %1" : "=v"(a.l_t) : "s"(a.l_t));
    asm volatile("v_mov_b32 %0, %1" : "=v"(a.theta) : "s"(a.theta));
    asm volatile("v_mov_b32 %0, %1" : "=v"(a.taut) : "s"(a.taut));
    if (G) asm volatile("v_mov_b32 %0, %1" : "=v"(a.gamma) : "s"(a.gamma));
  }
  const RollBufs &B = ra.b;
  const int lane = threadIdx.x & 63;
  const int band = wid % ra.bands, seg = wid / ra.bands;
  RollLane L;
  L.X = band * (BW - 2 * HALO) - HALO + PX * lane;
  // load column: clamped so all PX px lie in the row's pitch (px >= W are never used by
  // a px < W: the right clamp and the x = 0 divergence form select)
  L.vload = 4u * imin(imax(L.X, 0), a.P - PX);
  L.vloadp = a.p_zero ? kOOB : L.vload;
  L.out = PX * lane >= HALO && PX * lane < BW - HALO && L.X < a.W;
  L.vst = 4u * (unsigned)imax(L.X, 0);
  const unsigned rowb = 4u * (unsigned)a.P;                 // row pitch in bytes
  L.ys = seg * ra.seg_rows;
  L.ye = imin(L.ys + ra.seg_rows, a.H);
  L.c0 = band * (BW - 2 * HALO) - HALO <= 0;   // lane 0's first px (wave-uniform)
  const int r0 = imax(L.ys - K, 0);

  RollPipe<G, K, PX> S;
#pragma unroll
  for (int n = 0; n <= K; ++n)
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      S.U1c[n][j] = S.U2c[n][j] = S.U3c[n][j] = S.U1p[n][j] = S.U2p[n][j] = S.U3p[n][j] = 0.0f;
      S.P11c[n][j] = S.P12c[n][j] = S.P21c[n][j] = S.P22c[n][j] = S.P31c[n][j] = S.P32c[n][j] = 0.0f;
      S.P11p[n][j] = S.P12p[n][j] = S.P21p[n][j] = S.P22p[n][j] = S.P31p[n][j] = S.P32p[n][j] = 0.0f;
    }
#pragma unroll
  for (int n = 0; n < K; ++n)
#pragma unroll
    for (int j = 0; j < PX; ++j) S.CX[n][j] = S.CY[n][j] = S.CR[n][j] = 0.0f;

  // Each prologue row load is followed by dropped (out-of-range) stores, as many as a
  // step issues: the loop is then entered with the same memory operations in flight as
  // its back edge carries, so the waits at the top of the loop are counted past the
  // younger stores and loads on both paths.
  auto dummy_stores = [&]() {
    float z[PX];
#pragma unroll
    for (int j = 0; j < PX; ++j) z[j] = 0.0f;
    const unsigned ps = B.pstride;
    bstorev<PX>(B.ud, B.ub, kOOB, z);
    bstorev<PX>(B.ud, B.ub, kOOB, z, ps);
    if (G) bstorev<PX>(B.ud, B.ub, kOOB, z, 2 * ps);
    bstorev<PX>(B.pd, B.pb, kOOB, z);
    bstorev<PX>(B.pd, B.pb, kOOB, z, ps);
    bstorev<PX>(B.pd, B.pb, kOOB, z, 2 * ps);
    bstorev<PX>(B.pd, B.pb, kOOB, z, 3 * ps);
    if (G) {
      bstorev<PX>(B.pd, B.pb, kOOB, z, 4 * ps);
      bstorev<PX>(B.pd, B.pb, kOOB, z, 5 * ps);
    }
  };
  double acc = 0.0, accm = 0.0;
  if constexpr (LDSR) {   // two LDS slots, steps unrolled by 2
    static_assert(!G && PX == 2, "LDS-staged rows: the 9 planes of G = false, 2 px per lane");
    const int X0 = band * (BW - 2 * HALO) - HALO;
    const bool hi = lane >= 32;
    const unsigned col = 4u * (unsigned)imin(imax(X0 + 4 * (lane & 31), 0), a.P - 4);
    const unsigned ps = B.pstride;
    RollDma D;
    D.c1 = col + (hi ? ps : 0u);
    D.c2 = hi ? kOOB : col + 2 * ps;
    D.u = col + (hi ? ps : 0u);
    D.p1 = a.p_zero ? kOOB : col + (hi ? ps : 0u);
    D.p2 = a.p_zero ? kOOB : col + 2 * ps + (hi ? ps : 0u);
    float *s0 = lds, *s1 = lds + kRollLdsSlot;
    const unsigned a0 =
        (unsigned)(size_t)(__attribute__((address_space(3))) float *)s0 + 8u * (unsigned)lane;
    const unsigned a1 = a0 + 4u * kRollLdsSlot;
    roll_dma_row(s0, B, (unsigned)r0 * rowb, D);
    dummy_stores();
    roll_dma_row(s1, B, (unsigned)imin(r0 + 1, a.H - 1) * rowb, D);
    dummy_stores();
    const int halves = (L.ye + K - r0 + 1) / 2;
    for (int h = 0, r = r0; h < halves; ++h, r += 2) {
      progress_prio<PRIO>(h, halves);
      roll_step_lds<K, FM, MID>(S, s0, a0, a, B, r, L, rowb, D, acc, &accm);
      roll_step_lds<K, FM, MID>(S, s1, a1, a, B, r + 1, L, rowb, D, acc, &accm);
    }
    // the last steps' refills (rows past the segment) land before the block's LDS is
    // released to another block
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if constexpr (AH == 1) {   // 2-row ring, steps unrolled by 2
    RollIn<G, PX> A, Bx;
    roll_load<G, PX>(A, B, (unsigned)r0 * rowb, L.vload, L.vloadp);
    dummy_stores();
    const int halves = (L.ye + K - r0 + 1) / 2;
    for (int h = 0, r = r0; h < halves; ++h, r += 2) {
      progress_prio<PRIO>(h, halves);
      roll_step<G, K, PX, FM, AH>(S, A, Bx, a, B, r, L, rowb, acc);
      roll_step<G, K, PX, FM, AH>(S, Bx, A, a, B, r + 1, L, rowb, acc);
    }
  } else {   // 3-row ring, steps unrolled by 3
    static_assert(AH == 2, "the step loop below is unrolled for a 3-row ring");
    RollIn<G, PX> A, Bx, C;
    roll_load<G, PX>(A, B, (unsigned)r0 * rowb, L.vload, L.vloadp);
    dummy_stores();
    roll_load<G, PX>(Bx, B, (unsigned)imin(r0 + 1, a.H - 1) * rowb, L.vload, L.vloadp);
    dummy_stores();
    // steps r0 .. r0 + 3*thirds - 1 >= ye - 1 + K (rows >= H drain the pipeline)
    const int thirds = (L.ye + K - r0 + 2) / 3;
    for (int h = 0, r = r0; h < thirds; ++h, r += 3) {
      progress_prio<PRIO>(h, thirds);
      roll_step<G, K, PX, FM, AH>(S, A, C, a, B, r, L, rowb, acc);
      roll_step<G, K, PX, FM, AH>(S, Bx, A, a, B, r + 1, L, rowb, acc);
      roll_step<G, K, PX, FM, AH>(S, C, Bx, a, B, r + 2, L, rowb, acc);
    }
  }
  if (a.calc_err) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) a.partials[wid] = acc;
  }
  if constexpr (MID) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) accm += __shfl_xor(accm, o);
    if (lane == 0) a.partials[ra.waves + wid] = accm;
  }
}

template <bool G, int K, int PX, int FM = 0>
__global__ __launch_bounds__(256) void k_iterate_roll(RollArgs ra) {
  constexpr bool LDSR = roll_lds_on<G, K, PX>();
  __shared__ float lds[LDSR ? 4 * kRollLdsWave : 1];
  // wave-uniform (scalar) band / segment
  const int wid =
      __builtin_amdgcn_readfirstlane(xcd_chunk(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6));
  if (wid >= ra.waves || gated_off(ra.it.gate, ra.it.gate_seq)) return;   // whole wavefronts
  roll_body<G, K, PX, FM, 1, roll_ahead<K, PX>(), LDSR>(
      ra, wid, lds + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * (LDSR ? kRollLdsWave : 0));
}

// k_iterate_roll_mid<FM>: k_iterate_roll<false, 4, 2> that also sums the residual of the
// check after its first 2 iterations (partials[waves + wid]), so that two 2-iteration passes
// of a warp that is converging (procOneScale checking every second iteration, error just
// above eps^2 W H) run as one 4-iteration pass and one launch (DESIGN.md §4.1 of r6).  Stage
// 2's values are the ones a 2-iteration pass computes (same operations on the same operands),
// so its residual is that pass's over the same px; the host reads it first, and when the warp
// stops there it recomputes the 2-iteration state from the pass's input set, which the pass
// leaves untouched.  The end check must be a calc_err pass.
#ifndef TVL1_MID_MINW   // minimum waves per SIMD the mid-check pass is compiled for (A/B)
#define TVL1_MID_MINW 1
#endif
template <int FM>
__global__ __launch_bounds__(256, TVL1_MID_MINW) void k_iterate_roll_mid(RollArgs ra) {
  __shared__ float lds[4 * kRollLdsWave];
  const int wid =
      __builtin_amdgcn_readfirstlane(xcd_chunk(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6));
  if (wid >= ra.waves || gated_off(ra.it.gate, ra.it.gate_seq)) return;   // whole wavefronts
  roll_body<false, 4, 2, FM, 1, roll_ahead<4, 2>(), true, true>(
      ra, wid, lds + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * kRollLdsWave);
}

// ---------------------------------------------------------------- K5 + first pass, two roles
// k_warp_iter<M>: warpBackward and the warp's first pass (2 iterations ending in the first
// check) in one launch, the two jobs on different wavefronts of a block.  A block owns one
// k_iterate_roll<false, 2, 2> band (128 px: 124 output px + a 2-px halo each side) over a
// segment of rows, with three wavefronts:
//   * two producers run k_warp_ring's streaming warpBackward for the band's 128 columns
//     of one row per step (64 each): an LDS ring of I1 window rows r-M .. r+M (slots
//     x0-M .. x0+127+M, centeredGradient per slot), the same taps and order.  Each step
//     they write the row's warp constants and v = u + TH step of the first iteration
//     (pointwise, th_px) into a 2-row LDS C ring, and the constants to HBM too when the
//     warp may need further passes (store_c);
//   * one consumer runs the k_iterate_roll<false, 2, 2> pipeline (roll_advance: the same
//     arithmetic), taking each input row's constants and v from the C ring one step after
//     the producers wrote it, and only p from HBM.
// One LDS-only barrier per step orders the window row writes before the gathers and each
// C ring row before its read (2 C ring rows: a row is overwritten two steps after it was
// written, after the consumer's read at the step between).  The consumer's step is the
// longer one; the producers' wait at the barrier is issue time for the other blocks'
// wavefronts on the SIMD.  Against k_warp_ring + the pass, the constants (12 B/px stored
// and loaded, unless store_c) and one u load (8 B/px) stay on chip, and the gather's LDS
// latency hides behind the consumer's arithmetic.
struct WarpIterArgs {
  RollArgs ra;           // pass geometry (bands of 124 output px) and planes
  const float *I0, *I1;  // level images
  int store_c;           // also store I1wx / I1wy / rho (ra.it.I1wx, ...) for later passes
};

// window ring rows: 16 for the shipped margin M = 6 (a power of two: slot = row & 15);
// tighter margins take 2M + 2 rows (slot = row mod R, rows >= -64R)
template <int M>
constexpr int wi_rows() { return M == 6 ? 16 : 2 * M + 2; }
template <int M>
__device__ __forceinline__ int wi_slot(int r) {
  constexpr int R = wi_rows<M>();
  if ((R & (R - 1)) == 0) return r & (R - 1);
  return (int)((unsigned)(r + 64 * R) % (unsigned)R);
}
// band width BW (px): 128 = 64 consumer lanes x 2 px + 2 producers (default), or 64 =
// 64 lanes x 1 px + 1 producer (consumer and producer steps of similar length)
template <int M, int BW>
constexpr int wi_ww() { return BW + 2 * ring_mx<M>(); }

// window row r enters the ring: slot 64p + lane, and (producer 0, lanes < 2M) 128 + lane
template <int M, int BW>
__device__ __forceinline__ void wi_ring_put(float *__restrict__ ring, const WarpRowI &v, int r,
                                            int p, int lane) {
  constexpr int WW = wi_ww<M, BW>();
  float *dst = ring + wi_slot<M>(r) * ring_pitch(WW);
  const int k0 = 64 * p + lane;
  dst[k0] = v.c0;
  dst[WW + k0] = 0.5f * (v.r0 - v.l0);
  dst[2 * WW + k0] = 0.5f * (v.s0 - v.n0);
  if (p == 0 && lane < 2 * ring_mx<M>()) {
    dst[BW + lane] = v.c1;
    dst[WW + BW + lane] = 0.5f * (v.r1 - v.l1);
    dst[2 * WW + BW + lane] = 0.5f * (v.s1 - v.n1);
  }
}

// Producer lane geometry: column xc (the lane's px, clamped into the image), window
// column of slot 0 (xw0), C ring index ci, and whether the px is a stored output px.
struct WiLane {
  int xc, xw0, ci;
  unsigned xcb;
  bool outc;
};

// THP: the producer also does the first iteration's TH step and the C ring carries v (one
// consumer wavefront); otherwise it carries u^0 and stage 1's wavefront does the step (two
// consumers, where the producers set the block's pace: 1.5 % faster, tools/wi_probe.hip)
template <int M, int FM, int BW, bool THP = true>
__device__ __forceinline__ void wi_prod_step(float *__restrict__ ring, float *__restrict__ cring,
                                             const WarpRowI &cur, WarpRowI &ahead,
                                             const WarpRingArgs &wa, const WarpIterArgs &w,
                                             int g, int p, int lane, const WiLane &P,
                                             const unsigned (&xs)[2][3], int ys, int ye,
                                             unsigned nb, unsigned rowb) {
  constexpr int WW = wi_ww<M, BW>();
  // loads for row g + kWarpAhead: window row g + kWarpAhead + M and its flow row
  warp_ring_load(ahead, wa, nb, rowb, g + kWarpAhead + M, xs);
  warp_flow_load(ahead, wa, nb, rowb, g + kWarpAhead, P.xcb);
  __builtin_amdgcn_sched_barrier(0);
  wi_ring_put<M, BW>(ring, cur, g + M, p, lane);
  lds_barrier();
  // rows past the image bottom repeat row H-1 (the pass clamps its input rows)
  const int gy = imin(g, wa.H - 1);
  const float wx = (float)P.xc + cur.u1;
  const float wy = (float)gy + cur.u2;
  const int fx = tap_floor(wx);
  const int fy = tap_floor(wy);
  float sum = 0.0f, sumx = 0.0f, sumy = 0.0f, wsum = 0.0f;
  const bool inwin = fx - 1 >= P.xw0 && fx + 2 < P.xw0 + WW && fy - 1 >= gy - M && fy + 2 <= gy + M;
  if (inwin) {
    warp_gather_fn<FM>(
        [&](int cy, int cx) {
          const float *q = ring + wi_slot<M>(cy) * ring_pitch(WW) + (cx - P.xw0);
          return Tap3{q[0], q[WW], q[2 * WW]};
        },
        wx, wy, fx, fy, sum, sumx, sumy, wsum);
  } else {
    warp_gather_fn<FM>(
        [&](int cy, int cx) {
          const int rx = imin(imax(cx, 0), wa.W - 1), ry = imin(imax(cy, 0), wa.H - 1);
          const float *row = wa.I1 + (size_t)ry * wa.P;
          const float gx = 0.5f * (row[imin(rx + 1, wa.W - 1)] - row[imax(rx - 1, 0)]);
          const float gyv = 0.5f * (wa.I1[(size_t)imin(ry + 1, wa.H - 1) * wa.P + rx] -
                                    wa.I1[(size_t)imax(ry - 1, 0) * wa.P + rx]);
          return Tap3{row[rx], gx, gyv};
        },
        wx, wy, fx, fy, sum, sumx, sumy, wsum);
  }
  const float coeff = approx(FM) ? __builtin_amdgcn_rcpf(wsum) : recip_rn(wsum);
  const float I1wv = sum * coeff;
  const float I1wxv = sumx * coeff;
  const float I1wyv = sumy * coeff;
  const float rh = rho_c<FM>(I1wv, I1wxv, I1wyv, cur.u1, cur.u2, cur.i0);
  // the first iteration's TH step is pointwise: the producer does it (the consumer sets
  // the block's pace), and the C ring carries v = u^0 + d instead of u^0
  float v1 = cur.u1, v2 = cur.u2, v3;
  if (THP) th_px<false, FM>(I1wxv, I1wyv, rh, cur.u1, cur.u2, 0.0f, w.ra.it, v1, v2, v3);
  float *c = cring + (g & 1) * (5 * BW) + P.ci;
  c[0] = I1wxv;
  c[BW] = I1wyv;
  c[2 * BW] = rh;
  c[3 * BW] = v1;
  c[4 * BW] = v2;
  if (w.store_c) {
    const unsigned vo = P.outc && g >= ys && g < ye ? (unsigned)g * rowb + P.xcb : kOOB;
    bstore<kWarpStoreAux>(wa.I1wx, nb, vo, 0, I1wxv);
    bstore<kWarpStoreAux>(wa.I1wy, nb, vo, 0, I1wyv);
    bstore<kWarpStoreAux>(wa.rho, nb, vo, 0, rh);
  }
}

template <int PX>
struct WiP {   // the consumer's HBM input of one row: p at its PX px
  float p11[PX], p12[PX], p21[PX], p22[PX];
};

template <int PX>
__device__ __forceinline__ void wi_p_load(WiP<PX> &v, const RollBufs &B, unsigned soff,
                                          unsigned voff) {
  const unsigned ps = B.pstride;
  bload<PX>(v.p11, B.ps, B.pb, voff, soff);
  bload<PX>(v.p12, B.ps, B.pb, voff, soff + ps);
  bload<PX>(v.p21, B.ps, B.pb, voff, soff + 2 * ps);
  bload<PX>(v.p22, B.ps, B.pb, voff, soff + 3 * ps);
}

template <int FM, int PX>
__device__ __forceinline__ void wi_cons_step(RollPipe<false, 2, PX> &S,
                                             const float *__restrict__ cring, const WiP<PX> &cur,
                                             WiP<PX> &ahead, const IterArgs &a,
                                             const RollBufs &B, int r, const RollLane &L,
                                             int lane, unsigned rowb, double &acc) {
  wi_p_load(ahead, B, (unsigned)imin(r + kRollAhead, a.H - 1) * rowb, L.vloadp);
  __builtin_amdgcn_sched_barrier(0);
  lds_barrier();   // C ring row r was written at the previous step
  constexpr int BW = 64 * PX;
  RollIn<false, PX> in;
  const float *c = cring + (r & 1) * (5 * BW) + PX * lane;
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    in.wx[j] = c[j];
    in.wy[j] = c[BW + j];
    in.rh[j] = c[2 * BW + j];
    in.u1[j] = c[3 * BW + j];   // v (roll_advance<.., VIN>)
    in.u2[j] = c[4 * BW + j];
    in.u3[j] = 0.0f;
    in.p11[j] = cur.p11[j]; in.p12[j] = cur.p12[j];
    in.p21[j] = cur.p21[j]; in.p22[j] = cur.p22[j];
    in.p31[j] = in.p32[j] = 0.0f;
  }
  roll_advance<false, 2, PX, true, FM>(S, in, a, B, r, L, rowb, acc);
}

// ---- the two-consumer form (NC = 2): one wavefront per iteration of the pass.
// The single consumer's step (2 iterations x 2 px, ~480 VALU) was the block's critical
// path against the producers' ~290.  Here stage 1 and stage 2 of the
// k_iterate_roll<false, 2, 2> pipeline run on two wavefronts, each over the whole band (so
// the x-neighbours stay DPP shifts inside the wave), stage 2 one step behind stage 1.  They
// evaluate exactly roll_advance's operations on exactly its operands; only the wave doing
// them changes.  Stage 1 also does both TH steps (pointwise: iteration 1's on u^0, which the
// producers then pass instead of v, and iteration 2's on u^1; estimate_u_px = th_px then
// u_from_v), which leaves the producers' gather as the shortest critical path measured.
// Hand-off ring (LDS, 2 slots of kWiH planes x BW floats): for input row r, stage 1 writes
// v^2(r) (u^1(r) + TH step), u^1(r) (the residual's old u) and p^1(r-1); stage 2 reads the
// slot one barrier later.  A slot is overwritten two steps after it was written, after the
// read at the step between.
constexpr int kWiH = 8;

template <int PX>
struct WiS1 {   // stage 1 registers (k_iterate_roll's RollPipe stage 0 / 1 entries)
  float U1c[PX], U2c[PX];                        // u^1(r)
  float U1p[PX], U2p[PX];                        // u^1(r-1)
  float P11c[PX], P12c[PX], P21c[PX], P22c[PX];  // p^0(r)
  float P11p[PX], P12p[PX], P21p[PX], P22p[PX];  // p^0(r-1)
};

template <int PX>
struct WiS2 {   // stage 2 registers (RollPipe stage 1 / 2 entries)
  float V1p[PX], V2p[PX];                        // v^2(r-1)
  float W1p[PX], W2p[PX];                        // u^1(r-1)
  float Q11c[PX], Q12c[PX], Q21c[PX], Q22c[PX];  // p^1(r-1)
  float Q11p[PX], Q12p[PX], Q21p[PX], Q22p[PX];  // p^1(r-2)
  float U1c[PX], U2c[PX];                        // u^2(r-1)
  float U1p[PX], U2p[PX];                        // u^2(r-2)
};

template <int PX>
__device__ __forceinline__ void lds_put(float *__restrict__ p, const float (&v)[PX]) {
  if constexpr (PX == 2) *reinterpret_cast<float2 *>(p) = make_float2(v[0], v[1]);
  else
#pragma unroll
    for (int j = 0; j < PX; ++j) p[j] = v[j];
}
template <int PX>
__device__ __forceinline__ void lds_get(float (&v)[PX], const float *__restrict__ p) {
  if constexpr (PX == 2) {
    const float2 t = *reinterpret_cast<const float2 *>(p);
    v[0] = t.x;
    v[1] = t.y;
  } else {
#pragma unroll
    for (int j = 0; j < PX; ++j) v[j] = p[j];
  }
}

// Stage 1 at input row r: u^1(r) = v(r) + theta div p^0 (roll_advance's VIN stage 1),
// p^1(r-1) from u^1(r-1), u^1(r) and p^0(r-1), and iteration 2's TH step on u^1(r).
template <int FM, int PX, bool THP = true>
__device__ __forceinline__ void wi_s1_step(WiS1<PX> &S, const float *__restrict__ cring,
                                           float *__restrict__ hring, const WiP<PX> &cur,
                                           WiP<PX> &ahead, const IterArgs &a, const RollBufs &B,
                                           int r, const RollLane &L, int lane, unsigned rowb) {
  wi_p_load(ahead, B, (unsigned)imin(r + kRollAhead, a.H - 1) * rowb, L.vloadp);
  __builtin_amdgcn_sched_barrier(0);
  lds_barrier();   // C ring row r was written at the previous step; hand-off slot r & 1 read
  constexpr int BW = 64 * PX;
  const float *c = cring + (r & 1) * (5 * BW) + PX * lane;
  float wx[PX], wy[PX], rh[PX], v1[PX], v2[PX];
  lds_get<PX>(wx, c);
  lds_get<PX>(wy, c + BW);
  lds_get<PX>(rh, c + 2 * BW);
  lds_get<PX>(v1, c + 3 * BW);   // v = u^0 + TH step, or u^0 (!THP: the step is done here)
  lds_get<PX>(v2, c + 4 * BW);
  if (!THP) {
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      float t3;
      th_px<false, FM>(wx[j], wy[j], rh[j], v1[j], v2[j], 0.0f, a, v1[j], v2[j], t3);
    }
  }
#pragma unroll
  for (int j = 0; j < PX; ++j) {   // (p = 0 on a level's first pass: RollLane::vloadp)
    S.U1p[j] = S.U1c[j]; S.U2p[j] = S.U2c[j];
    S.P11p[j] = S.P11c[j]; S.P12p[j] = S.P12c[j]; S.P21p[j] = S.P21c[j]; S.P22p[j] = S.P22c[j];
    S.P11c[j] = cur.p11[j]; S.P12c[j] = cur.p12[j];
    S.P21c[j] = cur.p21[j]; S.P22c[j] = cur.p22[j];
  }
  const int yU = r;
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    float n1, n2, n3;
    u_from_v<false, FM, true>(v1[j], v2[j], 0.0f, S.P11c[j], left_of<PX>(S.P11c, j), S.P12c[j],
                              S.P12p[j], S.P21c[j], left_of<PX>(S.P21c, j), S.P22c[j], S.P22p[j],
                              0.0f, 0.0f, 0.0f, 0.0f, L.X + j, yU, a, n1, n2, n3, L.c0);
    S.U1c[j] = n1; S.U2c[j] = n2;
  }
  // the rolling pipeline's edge rules (roll_advance): u below the image repeats row H-1,
  // p above it is +0 -- wave-uniform branches instead of per-px selects
  if (yU >= a.H) {
#pragma unroll
    for (int j = 0; j < PX; ++j) { S.U1c[j] = S.U1p[j]; S.U2c[j] = S.U2p[j]; }
  }
  const int yD = r - 1;
  float q11[PX], q12[PX], q21[PX], q22[PX], t1[PX], t2[PX];
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    const bool has_right = L.X + j + 1 < a.W;
    dual_px<false, false, FM>(S.U1p[j], right_of<PX>(S.U1p, j), S.U1c[j], has_right, true,
                              a.taut, S.P11p[j], S.P12p[j], q11[j], q12[j], a.taut_small);
    dual_px<false, false, FM>(S.U2p[j], right_of<PX>(S.U2p, j), S.U2c[j], has_right, true,
                              a.taut, S.P21p[j], S.P22p[j], q21[j], q22[j], a.taut_small);
    float t3;
    th_px<false, FM>(wx[j], wy[j], rh[j], S.U1c[j], S.U2c[j], 0.0f, a, t1[j], t2[j], t3);
  }
  if (yD < 0) {
#pragma unroll
    for (int j = 0; j < PX; ++j) q11[j] = q12[j] = q21[j] = q22[j] = 0.0f;
  }
  float *h = hring + (r & 1) * (kWiH * BW) + PX * lane;
  lds_put<PX>(h, t1);
  lds_put<PX>(h + BW, t2);
  lds_put<PX>(h + 2 * BW, S.U1c);
  lds_put<PX>(h + 3 * BW, S.U2c);
  lds_put<PX>(h + 4 * BW, q11);
  lds_put<PX>(h + 5 * BW, q12);
  lds_put<PX>(h + 6 * BW, q21);
  lds_put<PX>(h + 7 * BW, q22);
}

// Stage 2 at input row r (one barrier after stage 1's step r): u^2(r-1) = v^2(r-1) +
// theta div p^1, the residual term (u^1(r-1) - u^2(r-1))^2, p^2(r-2); stores u^2 and p^2.
template <int FM, int PX>
__device__ __forceinline__ void wi_s2_step(WiS2<PX> &S, const float *__restrict__ hring,
                                           const IterArgs &a, const RollBufs &B, int r,
                                           const RollLane &L, int lane, unsigned rowb,
                                           double &acc) {
  lds_barrier();   // hand-off row r was written at the previous step
  constexpr int BW = 64 * PX;
  const unsigned ps = B.pstride;
  const float *h = hring + (r & 1) * (kWiH * BW) + PX * lane;
  float v1[PX], v2[PX], w1[PX], w2[PX];
  lds_get<PX>(v1, h);
  lds_get<PX>(v2, h + BW);
  lds_get<PX>(w1, h + 2 * BW);
  lds_get<PX>(w2, h + 3 * BW);
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    S.U1p[j] = S.U1c[j]; S.U2p[j] = S.U2c[j];
    S.Q11p[j] = S.Q11c[j]; S.Q12p[j] = S.Q12c[j]; S.Q21p[j] = S.Q21c[j]; S.Q22p[j] = S.Q22c[j];
  }
  lds_get<PX>(S.Q11c, h + 4 * BW);
  lds_get<PX>(S.Q12c, h + 5 * BW);
  lds_get<PX>(S.Q21c, h + 6 * BW);
  lds_get<PX>(S.Q22c, h + 7 * BW);
  const int yU = r - 1;
  const bool stU = L.out && yU >= L.ys && yU < L.ye;
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    float n1, n2, n3;
    u_from_v<false, FM, true>(S.V1p[j], S.V2p[j], 0.0f, S.Q11c[j], left_of<PX>(S.Q11c, j),
                              S.Q12c[j], S.Q12p[j], S.Q21c[j], left_of<PX>(S.Q21c, j), S.Q22c[j],
                              S.Q22p[j], 0.0f, 0.0f, 0.0f, 0.0f, L.X + j, yU, a, n1, n2, n3, L.c0);
    if (a.calc_err) {
      const float e = residual_px<FM>(S.W1p[j] - n1, S.W2p[j] - n2);
      acc += stU && L.X + j < a.W ? (double)e : 0.0;
    }
    S.U1c[j] = n1; S.U2c[j] = n2;
  }
  {
    const unsigned vo = stU ? (unsigned)yU * rowb + L.vst : kOOB;
    bstorev<PX>(B.ud, B.ub, vo, S.U1c);
    bstorev<PX>(B.ud, B.ub, vo, S.U2c, ps);
  }
  if (yU >= a.H) {   // u below the image repeats row H-1 (wi_s1_step)
#pragma unroll
    for (int j = 0; j < PX; ++j) { S.U1c[j] = S.U1p[j]; S.U2c[j] = S.U2p[j]; }
  }
  const int yD = r - 2;
  float o11[PX], o12[PX], o21[PX], o22[PX];
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    const bool has_right = L.X + j + 1 < a.W;
    dual_px<false, false, FM>(S.U1p[j], right_of<PX>(S.U1p, j), S.U1c[j], has_right, true,
                              a.taut, S.Q11p[j], S.Q12p[j], o11[j], o12[j], a.taut_small);
    dual_px<false, false, FM>(S.U2p[j], right_of<PX>(S.U2p, j), S.U2c[j], has_right, true,
                              a.taut, S.Q21p[j], S.Q22p[j], o21[j], o22[j], a.taut_small);
  }
  {
    const unsigned vo = L.out && yD >= L.ys && yD < L.ye ? (unsigned)yD * rowb + L.vst : kOOB;
    bstorev<PX>(B.pd, B.pb, vo, o11);
    bstorev<PX>(B.pd, B.pb, vo, o12, ps);
    bstorev<PX>(B.pd, B.pb, vo, o21, 2 * ps);
    bstorev<PX>(B.pd, B.pb, vo, o22, 3 * ps);
  }
#pragma unroll
  for (int j = 0; j < PX; ++j) {   // row r's hand-off values are row r-1's at the next step
    S.V1p[j] = v1[j]; S.V2p[j] = v2[j];
    S.W1p[j] = w1[j]; S.W2p[j] = w2[j];
  }
}

// NC = 2 also moves the first iteration's TH step from the producers to stage 1's wavefront.
// One block's work: band `band`, output rows ys .. ye-1, residual partial in slot `pslot`.
template <int M, int FM, int BW, int PRIO = 0, int NC = 1>
__device__ __forceinline__ void warp_iter_seg(const WarpIterArgs &w, int band, int ys, int ye,
                                              int pslot, float *__restrict__ ring,
                                              float *__restrict__ cring,
                                              float *__restrict__ hring = nullptr) {
  constexpr int K = 2, PX = BW / 64, HALO = roll_halo<2, PX>(), WW = wi_ww<M, BW>();
  static_assert(BW == 64 || BW == 128, "one producer per 64 columns, PX = 1 or 2");
  static_assert(2 * M + 2 <= wi_rows<M>(), "window ring too small for the margin");
  static_assert(2 * ring_mx<M>() <= 64, "second window slot per lane");
  static_assert(ring_pitch(WW) % 32 == 0, "row pitch: no bank conflicts between ring rows");
  static_assert(kRollAhead == 2 && kWarpAhead == 2, "the step loops are unrolled by 3");
  static_assert(NC == 1 || NC == 2, "one consumer wave, or one per iteration");
  (void)WW;
  const RollArgs &ra = w.ra;
  const IterArgs &a = ra.it;
  const int lane = threadIdx.x & 63;
  // wave 0 consumer, 1-2 producers (measured: a consumer on wave 1 or 2 of some blocks, or
  // a raised s_setprio for it, is slower).  NC = 2: waves 0 / 1 stages 1 / 2, 2-3 producers
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int X0 = band * (BW - 2 * HALO) - HALO;   // the band's first px
  const unsigned nb = 4u * (unsigned)a.P * (unsigned)a.H;
  const unsigned rowb = 4u * (unsigned)a.P;
  const int r0 = imax(ys - K, 0);
  // consumer steps r0 .. r0 + 3*thirds - 1 >= ye - 1 + K; the producers run one row ahead
  // and 3 (thirds + 1) steps, the consumer 1 + 3 thirds + 2 barriers
  const int thirds = (ye + K - r0 + 2) / 3;
  if (NC == 2 && wv < 2) {
    // stage 1: barriers 0 (prologue), 1 .. 3 thirds (steps), 2 final; stage 2: barriers
    // 0, 1 (prologue), 2 .. 3 thirds + 1 (steps), 1 final -- as many as the producers'
    RollLane L;
    L.X = X0 + PX * lane;
    L.vload = 4u * imin(imax(L.X, 0), a.P - PX);
    L.vloadp = a.p_zero ? kOOB : L.vload;
    L.out = PX * lane >= HALO && PX * lane < BW - HALO && L.X < a.W;
    L.vst = 4u * (unsigned)imax(L.X, 0);
    L.ys = ys;
    L.ye = ye;
    L.c0 = X0 <= 0;
    const RollBufs &Bf = ra.b;
    if (wv == 0) {
      WiS1<PX> S;
#pragma unroll
      for (int j = 0; j < PX; ++j) {
        S.U1c[j] = S.U2c[j] = S.U1p[j] = S.U2p[j] = 0.0f;
        S.P11c[j] = S.P12c[j] = S.P21c[j] = S.P22c[j] = 0.0f;
        S.P11p[j] = S.P12p[j] = S.P21p[j] = S.P22p[j] = 0.0f;
      }
      WiP<PX> A, B, C;
      wi_p_load(A, Bf, (unsigned)r0 * rowb, L.vloadp);
      wi_p_load(B, Bf, (unsigned)imin(r0 + 1, a.H - 1) * rowb, L.vloadp);
      lds_barrier();   // the producers' first step (row r0)
      for (int h = 0, r = r0; h < thirds; ++h, r += 3) {
        progress_prio<PRIO>(h, thirds);
        wi_s1_step<FM, PX, false>(S, cring, hring, A, C, a, Bf, r, L, lane, rowb);
        wi_s1_step<FM, PX, false>(S, cring, hring, B, A, a, Bf, r + 1, L, lane, rowb);
        wi_s1_step<FM, PX, false>(S, cring, hring, C, B, a, Bf, r + 2, L, lane, rowb);
      }
      lds_barrier();
      lds_barrier();
    } else {
      WiS2<PX> S;
#pragma unroll
      for (int j = 0; j < PX; ++j) {
        S.V1p[j] = S.V2p[j] = S.W1p[j] = S.W2p[j] = 0.0f;
        S.Q11c[j] = S.Q12c[j] = S.Q21c[j] = S.Q22c[j] = 0.0f;
        S.Q11p[j] = S.Q12p[j] = S.Q21p[j] = S.Q22p[j] = 0.0f;
        S.U1c[j] = S.U2c[j] = S.U1p[j] = S.U2p[j] = 0.0f;
      }
      lds_barrier();
      lds_barrier();
      double acc = 0.0;
      for (int h = 0, r = r0; h < thirds; ++h, r += 3) {
        progress_prio<PRIO>(h, thirds);
        wi_s2_step<FM, PX>(S, hring, a, Bf, r, L, lane, rowb, acc);
        wi_s2_step<FM, PX>(S, hring, a, Bf, r + 1, L, lane, rowb, acc);
        wi_s2_step<FM, PX>(S, hring, a, Bf, r + 2, L, lane, rowb, acc);
      }
      lds_barrier();
      if (a.calc_err) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if (lane == 0) a.partials[pslot] = acc;
      }
    }
  } else if (NC == 1 && wv == 0) {
    RollLane L;
    L.X = X0 + PX * lane;
    L.vload = 4u * imin(imax(L.X, 0), a.P - PX);
    L.vloadp = a.p_zero ? kOOB : L.vload;
    L.out = PX * lane >= HALO && PX * lane < BW - HALO && L.X < a.W;
    L.vst = 4u * (unsigned)imax(L.X, 0);
    L.ys = ys;
    L.ye = ye;
    L.c0 = X0 <= 0;
    RollPipe<false, K, PX> S;
#pragma unroll
    for (int n = 0; n <= K; ++n)
#pragma unroll
      for (int j = 0; j < PX; ++j) {
        S.U1c[n][j] = S.U2c[n][j] = S.U3c[n][j] = S.U1p[n][j] = S.U2p[n][j] = S.U3p[n][j] = 0.0f;
        S.P11c[n][j] = S.P12c[n][j] = S.P21c[n][j] = S.P22c[n][j] = S.P31c[n][j] = S.P32c[n][j] = 0.0f;
        S.P11p[n][j] = S.P12p[n][j] = S.P21p[n][j] = S.P22p[n][j] = S.P31p[n][j] = S.P32p[n][j] = 0.0f;
      }
#pragma unroll
    for (int n = 0; n < K; ++n)
#pragma unroll
      for (int j = 0; j < PX; ++j) S.CX[n][j] = S.CY[n][j] = S.CR[n][j] = 0.0f;
    // as many dropped stores after each prologue load as a step issues (k_iterate_roll)
    const RollBufs &Bf = ra.b;
    auto dummy_stores = [&]() {
      float z[PX];
#pragma unroll
      for (int j = 0; j < PX; ++j) z[j] = 0.0f;
      const unsigned ps = Bf.pstride;
      bstorev<PX>(Bf.ud, Bf.ub, kOOB, z);
      bstorev<PX>(Bf.ud, Bf.ub, kOOB, z, ps);
      bstorev<PX>(Bf.pd, Bf.pb, kOOB, z);
      bstorev<PX>(Bf.pd, Bf.pb, kOOB, z, ps);
      bstorev<PX>(Bf.pd, Bf.pb, kOOB, z, 2 * ps);
      bstorev<PX>(Bf.pd, Bf.pb, kOOB, z, 3 * ps);
    };
    WiP<PX> A, B, C;
    wi_p_load(A, Bf, (unsigned)r0 * rowb, L.vloadp);
    dummy_stores();
    wi_p_load(B, Bf, (unsigned)imin(r0 + 1, a.H - 1) * rowb, L.vloadp);
    dummy_stores();
    lds_barrier();   // the producers' first step (row r0)
    double acc = 0.0;
    for (int h = 0, r = r0; h < thirds; ++h, r += 3) {
      progress_prio<PRIO>(h, thirds);
      wi_cons_step<FM, PX>(S, cring, A, C, a, Bf, r, L, lane, rowb, acc);
      wi_cons_step<FM, PX>(S, cring, B, A, a, Bf, r + 1, L, lane, rowb, acc);
      wi_cons_step<FM, PX>(S, cring, C, B, a, Bf, r + 2, L, lane, rowb, acc);
    }
    lds_barrier();   // the producers' last two steps
    lds_barrier();
    if (a.calc_err) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
      if (lane == 0) a.partials[pslot] = acc;
    }
  } else {
    const int p = wv - NC;
    WarpRingArgs wa;
    wa.I0 = w.I0;
    wa.I1 = w.I1;
    wa.u1 = a.u1s;
    wa.u2 = a.u2s;
    wa.I1wx = const_cast<float *>(a.I1wx);
    wa.I1wy = const_cast<float *>(a.I1wy);
    wa.rho = const_cast<float *>(a.rho);
    wa.W = a.W;
    wa.H = a.H;
    wa.P = a.P;
    WiLane P;
    P.xw0 = X0 - ring_mx<M>();
    P.ci = 64 * p + lane;
    const int px = X0 + P.ci;
    P.xc = imin(imax(px, 0), a.W - 1);
    P.xcb = 4u * (unsigned)P.xc;
    P.outc = P.ci >= HALO && P.ci < BW - HALO && px >= 0 && px < a.W;
    // the lane's window slots (clamped column, its clamped x-1 and x+1): 64p + lane, and
    // 128 + lane for producer 0's lanes < 2M (other lanes re-read the first slot)
    unsigned xs[2][3];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int slot = k == 1 && p == 0 && lane < 2 * ring_mx<M>() ? BW + lane : P.ci;
      const int cc = imin(imax(P.xw0 + slot, 0), a.W - 1);
      xs[k][0] = 4u * cc;
      xs[k][1] = 4u * imax(cc - 1, 0);
      xs[k][2] = 4u * imin(cc + 1, a.W - 1);
    }
    // ring prologue: window rows r0 - M .. r0 + M - 1, loads issued M rows at a time
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      WarpRowI t[M];
#pragma unroll
      for (int i = 0; i < M; ++i) warp_ring_load(t[i], wa, nb, rowb, r0 - M + b * M + i, xs);
#pragma unroll
      for (int i = 0; i < M; ++i) wi_ring_put<M, BW>(ring, t[i], r0 - M + b * M + i, p, lane);
    }
    WarpRowI A, B, C;
    warp_ring_load(A, wa, nb, rowb, r0 + M, xs);
    warp_flow_load(A, wa, nb, rowb, r0, P.xcb);
    warp_ring_load(B, wa, nb, rowb, r0 + 1 + M, xs);
    warp_flow_load(B, wa, nb, rowb, r0 + 1, P.xcb);
    for (int h = 0, g = r0; h <= thirds; ++h, g += 3) {
      progress_prio<PRIO>(h, thirds);
      constexpr bool THP = NC == 1;
      wi_prod_step<M, FM, BW, THP>(ring, cring, A, C, wa, w, g, p, lane, P, xs, ys, ye, nb, rowb);
      wi_prod_step<M, FM, BW, THP>(ring, cring, B, A, wa, w, g + 1, p, lane, P, xs, ys, ye, nb, rowb);
      wi_prod_step<M, FM, BW, THP>(ring, cring, C, B, wa, w, g + 2, p, lane, P, xs, ys, ye, nb, rowb);
    }
  }
}

template <int M, int FM, int BW, int PRIO = 0, int NC = 1>
__device__ __forceinline__ void warp_iter_body(const WarpIterArgs &w, int wid, float *__restrict__ ring,
                                               float *__restrict__ cring,
                                               float *__restrict__ hring = nullptr) {
  const RollArgs &ra = w.ra;
  const int band = wid % ra.bands, seg = wid / ra.bands;
  const int ys = seg * ra.seg_rows, ye = imin(ys + ra.seg_rows, ra.it.H);
  warp_iter_seg<M, FM, BW, PRIO, NC>(w, band, ys, ye, wid, ring, cring, hring);
}

template <int M, int FM = 0, int BW = 128, int PRIO = 1, int NC = 1>
__global__ __launch_bounds__(64 * NC + BW) void k_warp_iter(WarpIterArgs w) {
  __shared__ float ring[wi_rows<M>() * ring_pitch(wi_ww<M, BW>())];
  __shared__ float cring[2 * 5 * BW];
  __shared__ float hring[NC == 2 ? 2 * kWiH * BW : 1];
  const int wid = __builtin_amdgcn_readfirstlane(xcd_chunk(blockIdx.x, gridDim.x));
  if (wid >= w.ra.waves || gated_off(w.ra.it.gate, w.ra.it.gate_seq)) return;   // whole blocks
  warp_iter_body<M, FM, BW, PRIO, NC>(w, wid, ring, cring, hring);
}

// K7: fixed-order sum of the per-block partials (one block).
// The residual goes to coherent host memory; with seq_out set, the check's sequence number
// follows it there (after a system-scope fence), so the host can poll for it instead of
// waiting on an event.
//
// Speculation.  A check enqueued behind an earlier one runs only if that
// check's prediction held (g.in: *g.in == g.in_seq).  With g.out set, the reduce also
// evaluates the stopping rule for the launch enqueued behind it, exactly as the host does
// (engine: procOneScale's loop, in double), and writes its own sequence number to *g.out if
// the predicted next step is the one the host will take, 0 otherwise.  Predictions: pk = 0,
// the warp stops here; pk > 0, it continues with a pass of pk iterations ending in a check
// (pcalc) or not.
struct CheckGate {
  const unsigned long long *in;
  unsigned long long in_seq;
  unsigned long long *out;
  double thr;         // eps^2 * W * H
  int n, iters, kmax, eps_pos;
  int pk, pcalc;
};

// procOneScale's schedule from a residual: iterations up to and including the next check
// (the host's copy is sched_after in tvl1_engine.hip; the same double operations)
__host__ __device__ inline int sched_after(double prev, double thr, int n, int iters, int kmax,
                                           int eps_pos, bool *calc_end, double *prev_end) {
  int k = 0;
  bool ce = false;
  while (k < kmax && n + k < iters) {
    const bool calc = eps_pos && ((n + k) & 1) && prev < thr;
    ++k;
    if (calc) {
      ce = true;
      break;
    }
    prev -= thr;
  }
  *calc_end = ce;
  *prev_end = prev;
  return k;
}

TVL1_PLAIN __global__ void k_reduce(const double *__restrict__ partials, int n, double *__restrict__ out,
                         unsigned long long *seq_out, unsigned long long seq, CheckGate g) {
  if (gated_off(g.in, g.in_seq)) return;
  __shared__ double s[kBlock];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += kBlock) acc += partials[i];
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int o = kBlock / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double e = s[0];
    out[0] = e;
    if (g.out) {
      const bool ends = !(e > g.thr && g.n < g.iters);
      bool ok = ends;
      if (g.pk > 0) {
        bool ce;
        double pe;
        const int k = sched_after(e, g.thr, g.n, g.iters, g.kmax, g.eps_pos, &ce, &pe);
        ok = !ends && k == g.pk && (int)ce == g.pcalc;
      }
      *g.out = ok ? seq : 0ull;
    }
    if (seq_out) {
      __threadfence_system();
      *(volatile unsigned long long *)seq_out = seq;
    }
  }
}

// ---------------------------------------------------------------- misc
// Build-only median (cv::medianBlur CV_32F, ksize 3 or 5, BORDER_REPLICATE); blockIdx.z = component.
TVL1_PLAIN __global__ void k_median(const float *__restrict__ s1, const float *__restrict__ s2, int W,
                         int H, int P, int ksize, float *__restrict__ d1,
                         float *__restrict__ d2) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= W || y >= H) return;
  const float *src = blockIdx.z == 0 ? s1 : s2;
  float *dst = blockIdx.z == 0 ? d1 : d2;
  const int r = ksize / 2;
  float v[25];
  int n = 0;
  for (int dy = -r; dy <= r; ++dy)
    for (int dx = -r; dx <= r; ++dx)
      v[n++] = src[(size_t)imin(imax(y + dy, 0), H - 1) * P + imin(imax(x + dx, 0), W - 1)];
  for (int i = 1; i < n; ++i) {
    const float t = v[i];
    int j = i - 1;
    while (j >= 0 && v[j] > t) {
      v[j + 1] = v[j];
      --j;
    }
    v[j + 1] = t;
  }
  dst[(size_t)y * P + x] = v[n / 2];
}

// Final flow (u1[0], u2[0]) -> caller's pitched planar outputs (A.4 + cuda::split).
TVL1_PLAIN __global__ void k_output(const float *__restrict__ u1, const float *__restrict__ u2, int W,
                         int H, int P, float *__restrict__ ou, float *__restrict__ ov,
                         size_t opitch) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= W || y >= H) return;
  reinterpret_cast<float *>(reinterpret_cast<char *>(ou) + (size_t)y * opitch)[x] = u1[(size_t)y * P + x];
  reinterpret_cast<float *>(reinterpret_cast<char *>(ov) + (size_t)y * opitch)[x] = u2[(size_t)y * P + x];
}

// solve_wrapper post-ops (optflow.cpp:411-473): map = flow + (x, y) (mode 1); the
// features branch with output_type "flow" (mode 2: (flow + grid) warped by the
// alignment, identity here, minus grid); then zero where I1 <= 1
// (threshold THRESH_BINARY_INV + setTo(0, mask)).
TVL1_PLAIN __global__ void k_postprocess(float *__restrict__ u, float *__restrict__ v, size_t fp,
                              const uint8_t *__restrict__ I1, size_t p1, int W, int H,
                              int mode) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= W || y >= H) return;
  float *ur = reinterpret_cast<float *>(reinterpret_cast<char *>(u) + (size_t)y * fp);
  float *vr = reinterpret_cast<float *>(reinterpret_cast<char *>(v) + (size_t)y * fp);
  float a = ur[x], b = vr[x];
  if (mode >= 1) {  // map = flow + pixel grid
    a = a + (float)x;
    b = b + (float)y;
  }
  if (mode == 2) {  // features path with output_type "flow": flow = map - grid
    a = a - (float)x;
    b = b - (float)y;
  }
  if (I1[(size_t)y * p1 + x] <= 1) {
    a = 0.0f;
    b = 0.0f;
  }
  ur[x] = a;
  vr[x] = b;
}

// k_postprocess over n same-size pairs of a batch (tvl1_postprocess_batch): pair b =
// blockIdx.z, its flow at u / v + b * fstride bytes and its frame1 at I1 + b * s1 bytes.
TVL1_PLAIN __global__ void k_postprocess_batch(float *__restrict__ u, float *__restrict__ v,
                                               size_t fp, size_t fstride,
                                               const uint8_t *__restrict__ I1, size_t p1, size_t s1,
                                               int W, int H, int mode) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= W || y >= H) return;
  const size_t b = blockIdx.z;
  float *ur = reinterpret_cast<float *>(reinterpret_cast<char *>(u) + b * fstride + (size_t)y * fp);
  float *vr = reinterpret_cast<float *>(reinterpret_cast<char *>(v) + b * fstride + (size_t)y * fp);
  float a = ur[x], c = vr[x];
  if (mode >= 1) {
    a = a + (float)x;
    c = c + (float)y;
  }
  if (mode == 2) {
    a = a - (float)x;
    c = c - (float)y;
  }
  if (I1[b * s1 + (size_t)y * p1 + x] <= 1) {
    a = 0.0f;
    c = 0.0f;
  }
  ur[x] = a;
  vr[x] = c;
}

// tvl1_gather_flow: out[i] = (u[off[i]], v[off[i]]) (element offsets), one lane per point.
TVL1_PLAIN __global__ void k_gather_flow(const float *__restrict__ u, const float *__restrict__ v,
                                         const int64_t *__restrict__ off, int n,
                                         float2 *__restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t o = off[i];
  out[i] = make_float2(u[o], v[o]);
}

}  // namespace tvl1k
