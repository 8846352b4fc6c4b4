// tvl1_align.hpp — feature pre-alignment: the reference's find_alignment
// (/root/reference/src/features.cpp:46-167) and the cv::cuda::warpAffine calls around it
// (optflow.cpp:369-371 on frame1, :429-443 on the map fields), MI355X-native.
//
//   * keypoints: ORB's recipe (cv::cuda::ORB, features.cpp:56-61) -- a scale pyramid
//     (scaleFactor, nlevels), FAST-9 corners (fastThreshold) at least edgeThreshold px from
//     the border, ranked by the Harris response (k = 0.04, 7x7 window) after 3x3
//     non-maximum suppression, the best nfeatures kept with ORB's per-level quota;
//     orientation by the intensity centroid of the radius-15 disc (its unit vector, no
//     trigonometry); 256-bit rotated-BRIEF descriptors (WTA_K = 2) from a fixed
//     pseudo-random pattern of point pairs in the 31x31 patch;
//   * matching: brute-force Hamming 2-NN on the GPU (cuda::DescriptorMatcher::
//     createBFMatcher(NORM_HAMMING)->knnMatch(.., 2)), the reference's ratio test and
//     distance sort (features.cpp:98-113);
//   * model: cv::findHomography(RANSAC | LMEDS, ransac threshold) restated on the host --
//     4-point normalised DLT hypotheses, inlier count (RANSAC) or median residual (LMEDS),
//     a least-squares DLT refit on the inliers; then the reference's zoom check and the
//     top 2x3 of the homography as the affine (features.cpp:131-166).
//
// PARITY UNPINNED against OpenCV and approximate by construction: OpenCV's ORB bit pattern
// (bit_pattern_31_), its FAST score and its RNG are not restated, and SURF (features = 2,
// non-free) is served by the same ORB path with a warning.  The contract kept is the
// reference's: the same inputs (JSON keys with their defaults), an affine that maps frame1
// onto frame0, the same rejection rules and messages.  This pipeline itself is restated
// bit for bit by oracle/tvl1_oracle_align.c (test infrastructure): keypoints, descriptors,
// the 2-NN match list, the fit and the warps are compared exactly (tests/test_align_gpu.py),
// and known affine motions of synthetic slices are recovered.
#pragma once

#include <algorithm>
#include <cmath>
#include <vector>

namespace tvl1k {

constexpr int kOrbPatch = 31, kOrbHalf = 15, kOrbBits = 256;

// FAST-9 on a float level image (values 0..255) at px (x, y): a contiguous arc of >= 9 of
// the 16 radius-3 circle px all brighter than c + t or all darker than c - t.
constexpr int kFastDx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
constexpr int kFastDy[16] = {-3, -3, -2, -1, 0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3};

// Block = 64 x 16 px (4 wavefronts x 4 rows).  The image tile with a 4-px apron and the
// Sobel gradients of the 70 x 22 window positions are staged in LDS, so a corner's 7 x 7
// Harris sum reads LDS instead of ~400 scattered global loads.  Same expressions in the same
// order as a direct evaluation: the scores do not depend on the tiling.
constexpr int kFhW = 64, kFhH = 16, kFhTW = kFhW + 8, kFhTH = kFhH + 8;
constexpr int kFhGW = kFhW + 6, kFhGH = kFhH + 6;
__global__ void __launch_bounds__(256) ka_fast_harris(const float *__restrict__ I, int W, int H,
                                                      int P, int border, float t,
                                                      float *__restrict__ score) {
  __shared__ float img[kFhTH][kFhTW];
  __shared__ float gxs[kFhGH][kFhGW], gys[kFhGH][kFhGW];
  const int x0 = blockIdx.x * kFhW, y0 = blockIdx.y * kFhH;
  for (int i = threadIdx.x; i < kFhTW * kFhTH; i += 256) {
    const int ty = i / kFhTW, tx = i - ty * kFhTW;
    const int yy = imin(imax(y0 - 4 + ty, 0), H - 1), xx = imin(imax(x0 - 4 + tx, 0), W - 1);
    img[ty][tx] = I[(size_t)yy * P + xx];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kFhGW * kFhGH; i += 256) {
    const int gy = i / kFhGW, gx = i - gy * kFhGW;
    const int ty = gy + 1, tx = gx + 1;   // gradient position (x0-3+gx, y0-3+gy) in the tile
    const float *r0 = img[ty - 1], *r1 = img[ty], *r2 = img[ty + 1];
    gxs[gy][gx] = (r0[tx + 1] - r0[tx - 1]) + 2.f * (r1[tx + 1] - r1[tx - 1]) +
                  (r2[tx + 1] - r2[tx - 1]);
    gys[gy][gx] = (r2[tx - 1] - r0[tx - 1]) + 2.f * (r2[tx] - r0[tx]) + (r2[tx + 1] - r0[tx + 1]);
  }
  __syncthreads();
  const int lx = threadIdx.x & 63;
  const int x = x0 + lx;
  for (int ly = threadIdx.x >> 6; ly < kFhH; ly += 4) {
    const int y = y0 + ly;
    if (x >= W || y >= H) continue;
    float out = 0.0f;
    if (x >= border && y >= border && x < W - border && y < H - border) {
      const float c = img[ly + 4][lx + 4];
      unsigned bright = 0, dark = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const float v = img[ly + 4 + kFastDy[k]][lx + 4 + kFastDx[k]];
        bright |= (v > c + t ? 1u : 0u) << k;
        dark |= (v < c - t ? 1u : 0u) << k;
      }
      auto arc9 = [](unsigned m) {
        const unsigned mm = m | (m << 16);   // wrap around the circle
        unsigned run = mm;
#pragma unroll
        for (int k = 1; k < 9; ++k) run &= mm >> k;
        return run != 0;
      };
      if (arc9(bright) || arc9(dark)) {
        // Harris response over a 7x7 window of Sobel gradients (scaled to 0..1 intensities)
        float a = 0.f, b = 0.f, cc = 0.f;
        for (int dy = -3; dy <= 3; ++dy)
          for (int dx = -3; dx <= 3; ++dx) {
            const float gx = gxs[ly + 3 + dy][lx + 3 + dx];
            const float gy = gys[ly + 3 + dy][lx + 3 + dx];
            a += gx * gx;
            b += gy * gy;
            cc += gx * gy;
          }
        const float s = 1.0f / (4.f * 255.f * 49.f);
        a *= s * s;
        b *= s * s;
        cc *= s * s;
        out = fmaxf(a * b - cc * cc - 0.04f * (a + b) * (a + b), 1e-30f);
      }
    }
    score[(size_t)y * W + x] = out;
  }
}

// blurForDescriptor: 7x7 Gaussian, sigma 2 (ORB's GaussianBlur before the descriptors)
__global__ void ka_blur7(const float *__restrict__ I, int W, int H, int P, float *__restrict__ O) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= W || y >= H) return;
  const float g[7] = {0.07015933f, 0.13107488f, 0.19071282f, 0.21610594f, 0.19071282f,
                      0.13107488f, 0.07015933f};
  float s = 0.f;
  for (int dy = -3; dy <= 3; ++dy) {
    const float *r = I + (size_t)imin(imax(y + dy, 0), H - 1) * P;
    float t = 0.f;
    for (int dx = -3; dx <= 3; ++dx) t += g[dx + 3] * r[imin(imax(x + dx, 0), W - 1)];
    s += g[dy + 3] * t;
  }
  O[(size_t)y * P + x] = s;
}

// 3x3 non-maximum suppression of the corner scores.  A survivor is appended to its level's
// key list as the unique 64-bit key (score bits << 32) | ~(y * W + x): positive float bits
// order like the scores, and equal scores order by position (top-left first), so "the best
// quota keys" is one well-defined set whatever order the atomics append in.  No two
// survivors are neighbours (ties go to the top-left one), so a level has at most
// ceil(W/2) * ceil(H/2) of them: cap is that bound and nothing is ever dropped.
// A block covers a 64 x kNmsRows tile: its survivors are gathered in LDS (at most one per
// 2 x 2 px) and claimed with ONE global atomic per block -- same-address atomics are
// serialised at the L2, so one per survivor (~10^5 per level) cost a millisecond a level.
constexpr int kNmsRows = 64;
__global__ void __launch_bounds__(256) ka_nms(const float *__restrict__ score, int W, int H,
                                              uint64_t *__restrict__ keys,
                                              unsigned *__restrict__ count, unsigned cap) {
  __shared__ uint64_t lk[32 * (kNmsRows / 2)];
  __shared__ unsigned ln, lbase;
  const int tx = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) ln = 0;
  __syncthreads();
  const int x = blockIdx.x * 64 + tx;
  for (int r = wv; r < kNmsRows; r += 4) {
    const int y = blockIdx.y * kNmsRows + r;
    if (x < 1 || y < 1 || x >= W - 1 || y >= H - 1) continue;
    const float s = score[(size_t)y * W + x];
    bool keep = s > 0.0f;
    for (int dy = -1; dy <= 1 && keep; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        if (!dx && !dy) continue;
        const float o = score[(size_t)(y + dy) * W + x + dx];
        // ties broken by position so exactly one of two equal neighbours survives
        if (o > s || (o == s && (dy < 0 || (dy == 0 && dx < 0)))) keep = false;
      }
    if (keep)
      lk[atomicAdd(&ln, 1u)] =
          ((uint64_t)__float_as_uint(s) << 32) | (uint64_t)(0xFFFFFFFFu - (unsigned)(y * W + x));
  }
  __syncthreads();
  const unsigned n = ln;
  if (n == 0) return;
  if (threadIdx.x == 0) lbase = atomicAdd(count, n);
  __syncthreads();
  for (unsigned i = threadIdx.x; i < n; i += 256)
    if (lbase + i < cap) keys[lbase + i] = lk[i];
}

// KeyPointsFilter::retainBest per level: the quota largest keys of each level, by an MSB-first
// radix select (8 passes of 8 bits, histograms in LDS) to the quota-th largest key T, then
// every key >= T copied out (exactly quota of them: keys are unique).  One workgroup per
// level; the host orders the <= quota survivors.
struct SelLevel {
  unsigned off, cap, quota;
};
__global__ void __launch_bounds__(1024) ka_select(const uint64_t *__restrict__ keys,
                                                  const unsigned *__restrict__ count,
                                                  const SelLevel *__restrict__ lv,
                                                  uint64_t *__restrict__ out, unsigned kmax,
                                                  unsigned *__restrict__ nsel) {
  __shared__ unsigned hist[256];
  __shared__ uint64_t s_prefix, s_mask;
  __shared__ unsigned s_k, s_n;
  const int l = blockIdx.x;
  const SelLevel L = lv[l];
  const unsigned n = min(count[l], L.cap);
  const uint64_t *K = keys + L.off;
  uint64_t *O = out + (size_t)l * kmax;
  const unsigned t = threadIdx.x;
  if (n <= L.quota) {
    for (unsigned i = t; i < n; i += blockDim.x) O[i] = K[i];
    if (t == 0) nsel[l] = n;
    return;
  }
  if (t == 0) {
    s_prefix = 0;
    s_mask = 0;
    s_k = L.quota;
    s_n = 0;
  }
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (unsigned i = t; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    const uint64_t prefix = s_prefix, mask = s_mask;
    for (unsigned i = t; i < n; i += blockDim.x) {
      const uint64_t k = K[i];
      if ((k & mask) == prefix) atomicAdd(&hist[(unsigned)(k >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    if (t == 0) {
      unsigned k = s_k, cum = 0;
      int d = 255;
      for (; d > 0; --d) {
        if (cum + hist[d] >= k) break;
        cum += hist[d];
      }
      s_k = k - cum;   // rank of T among the keys of digit d
      s_prefix = prefix | ((uint64_t)d << shift);
      s_mask = mask | ((uint64_t)0xFF << shift);
    }
    __syncthreads();
  }
  const uint64_t T = s_prefix;
  for (unsigned i = t; i < n; i += blockDim.x) {
    const uint64_t k = K[i];
    if (k >= T) O[atomicAdd(&s_n, 1u)] = k;
  }
  __syncthreads();
  if (t == 0) nsel[l] = s_n;
}

struct OrbKp {
  float x, y;        // level coordinates
  float angle;       // radians (filled by ka_describe)
  int level;
};

// Orientation (intensity centroid over the radius-15 disc) and the 256-bit rotated BRIEF
// descriptor of each keypoint; one thread per keypoint.  pat: 256 x (ax, ay, bx, by).
__global__ void ka_describe(const float *const *__restrict__ levels, const int *__restrict__ lP,
                            OrbKp *__restrict__ kps, int n, const int4 *__restrict__ pat,
                            uint32_t *__restrict__ desc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  OrbKp k = kps[i];
  const float *I = levels[k.level];
  const int P = lP[k.level];
  const int cx = (int)k.x, cy = (int)k.y;
  float m01 = 0.f, m10 = 0.f;
  for (int v = -kOrbHalf; v <= kOrbHalf; ++v)
    for (int u = -kOrbHalf; u <= kOrbHalf; ++u) {
      if (u * u + v * v > kOrbHalf * kOrbHalf) continue;
      const float val = I[(size_t)(cy + v) * P + cx + u];
      m10 += u * val;
      m01 += v * val;
    }
  // the rotation of the intensity-centroid direction as (cos, sin) = (m10, m01) / |m|:
  // correctly rounded IEEE operations only, so oracle/tvl1_oracle_align.c restates the
  // descriptor bit for bit (atan2f / cosf / sinf differ between the device library and
  // glibc).  The angle is reported for the caller, never used.
  const float r = sqrtf(m10 * m10 + m01 * m01);
  const float cs = r > 0.f ? m10 / r : 1.f, sn = r > 0.f ? m01 / r : 0.f;
  k.angle = atan2f(m01, m10);
  kps[i] = k;
  for (int w = 0; w < kOrbBits / 32; ++w) {
    uint32_t bits = 0;
    for (int j = 0; j < 32; ++j) {
      const int4 q = pat[w * 32 + j];
      const int ax = (int)rintf(q.x * cs - q.y * sn), ay = (int)rintf(q.x * sn + q.y * cs);
      const int bx = (int)rintf(q.z * cs - q.w * sn), by = (int)rintf(q.z * sn + q.w * cs);
      const float va = I[(size_t)(cy + ay) * P + cx + ax];
      const float vb = I[(size_t)(cy + by) * P + cx + bx];
      bits |= (va < vb ? 1u : 0u) << j;
    }
    desc[(size_t)i * (kOrbBits / 32) + w] = bits;
  }
}

// Brute-force Hamming 2-NN of every query descriptor against all train descriptors
// (cuda BFMatcher knnMatch k = 2).  Grid (query groups of 64, train segments): a wavefront
// holds 64 queries in registers and streams its train segment through LDS, 64 descriptors
// per tile; each segment's stable top-2 (ties: lower train index) goes to part[], and
// ka_match2_merge folds the segments in index order, which gives exactly the top-2 of one
// sequential scan.
struct Top2 {
  int b0, b1, d0, d1;
};
__device__ __forceinline__ void top2_push(Top2 &t, int h, int j) {
  if (h < t.d0) {
    t.d1 = t.d0;
    t.b1 = t.b0;
    t.d0 = h;
    t.b0 = j;
  } else if (h < t.d1) {
    t.d1 = h;
    t.b1 = j;
  }
}
__global__ void __launch_bounds__(64) ka_match2(const uint32_t *__restrict__ q, int nq,
                                                const uint32_t *__restrict__ t, int nt, int seg,
                                                Top2 *__restrict__ part) {
  __shared__ uint32_t tile[64 * 8];
  const int lane = threadIdx.x;
  const int i = blockIdx.x * 64 + lane;
  const int j0 = blockIdx.y * seg, j1 = min(nt, j0 + seg);
  uint32_t d[8];
#pragma unroll
  for (int w = 0; w < 8; ++w) d[w] = i < nq ? q[(size_t)i * 8 + w] : 0u;
  Top2 r{-1, -1, 1 << 30, 1 << 30};
  for (int jt = j0; jt < j1; jt += 64) {
    const int nj = min(64, j1 - jt);
    __syncthreads();
    if (lane < nj) {
#pragma unroll
      for (int w = 0; w < 8; ++w) tile[w * 64 + lane] = t[(size_t)(jt + lane) * 8 + w];
    }
    __syncthreads();
    for (int k = 0; k < nj; ++k) {
      int h = 0;
#pragma unroll
      for (int w = 0; w < 8; ++w) h += __popc(d[w] ^ tile[w * 64 + k]);
      top2_push(r, h, jt + k);
    }
  }
  if (i < nq) part[(size_t)blockIdx.y * nq + i] = r;
}
__global__ void ka_match2_merge(const Top2 *__restrict__ part, int nq, int nseg,
                                int2 *__restrict__ best, int2 *__restrict__ dist) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  Top2 r = part[i];
  for (int s = 1; s < nseg; ++s) {
    const Top2 p = part[(size_t)s * nq + i];
    if (p.b0 >= 0) top2_push(r, p.d0, p.b0);
    if (p.b1 >= 0) top2_push(r, p.d1, p.b1);
  }
  best[i] = make_int2(r.b0, r.b1);
  dist[i] = make_int2(r.d0, r.d1);
}

// cv::cuda::warpAffine(src, dst, M, dsize, INTER_LINEAR, BORDER_CONSTANT 0): dst(x, y) =
// src(iM (x, y, 1)) with iM = the inverse of M (float coefficients), bilinear taps
// (cuda LinearFilter form) with out-of-image taps 0.
__device__ __forceinline__ float affine_sample(const float *__restrict__ src, int sw, int sh,
                                               size_t sp, float xs, float ys) {
  const float x1f = floorf(xs), y1f = floorf(ys);
  const int x1 = (int)x1f, y1 = (int)y1f, x2 = x1 + 1, y2 = y1 + 1;
  auto at = [&](int yy, int xx) -> float {
    return (xx >= 0 && yy >= 0 && xx < sw && yy < sh) ? src[(size_t)yy * sp + xx] : 0.0f;
  };
  float out = 0.0f;
  out = out + at(y1, x1) * (((float)x2 - xs) * ((float)y2 - ys));
  out = out + at(y1, x2) * ((xs - (float)x1) * ((float)y2 - ys));
  out = out + at(y2, x1) * (((float)x2 - xs) * (ys - (float)y1));
  out = out + at(y2, x2) * ((xs - (float)x1) * (ys - (float)y1));
  return out;
}

struct Affine {
  float m[6];   // the inverse transform, row-major 2x3
};

__global__ void ka_warp_u8(const uint8_t *__restrict__ src, size_t sp, int sw, int sh,
                           uint8_t *__restrict__ dst, size_t dp, int dw, int dh, Affine iM) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= dw || y >= dh) return;
  const float xs = iM.m[0] * x + iM.m[1] * y + iM.m[2];
  const float ys = iM.m[3] * x + iM.m[4] * y + iM.m[5];
  const float x1f = floorf(xs), y1f = floorf(ys);
  const int x1 = (int)x1f, y1 = (int)y1f, x2 = x1 + 1, y2 = y1 + 1;
  auto at = [&](int yy, int xx) -> float {
    return (xx >= 0 && yy >= 0 && xx < sw && yy < sh) ? (float)src[(size_t)yy * sp + xx] : 0.0f;
  };
  float out = 0.0f;
  out = out + at(y1, x1) * (((float)x2 - xs) * ((float)y2 - ys));
  out = out + at(y1, x2) * ((xs - (float)x1) * ((float)y2 - ys));
  out = out + at(y2, x1) * (((float)x2 - xs) * (ys - (float)y1));
  out = out + at(y2, x2) * ((xs - (float)x1) * (ys - (float)y1));
  dst[(size_t)y * dp + x] = (uint8_t)fminf(fmaxf(rintf(out), 0.0f), 255.0f);
}

// solve_wrapper's features branch (optflow.cpp:411-443, 468-473) on a flow ROI: map =
// flow + grid, warped by the affine (the map planes staged in m1/m2), then flow = warped -
// grid (output_type "flow") or the warped map, and 0 where I1 <= 1.  Two launches: stage,
// then warp (a px reads other px of the staged map).
__global__ void ka_map_stage(const float *__restrict__ u, const float *__restrict__ v, size_t fp,
                             int W, int H, float *__restrict__ m1, float *__restrict__ m2) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= W || y >= H) return;
  const float *ur = reinterpret_cast<const float *>(reinterpret_cast<const char *>(u) + (size_t)y * fp);
  const float *vr = reinterpret_cast<const float *>(reinterpret_cast<const char *>(v) + (size_t)y * fp);
  m1[(size_t)y * W + x] = ur[x] + (float)x;
  m2[(size_t)y * W + x] = vr[x] + (float)y;
}
__global__ void ka_map_warp(const float *__restrict__ m1, const float *__restrict__ m2, int W, int H,
                            Affine iM, int flow_out, const uint8_t *__restrict__ I1, size_t p1,
                            float *__restrict__ u, float *__restrict__ v, size_t fp) {
  const int x = blockIdx.x * 64 + threadIdx.x;
  const int y = blockIdx.y * 4 + threadIdx.y;
  if (x >= W || y >= H) return;
  const float xs = iM.m[0] * x + iM.m[1] * y + iM.m[2];
  const float ys = iM.m[3] * x + iM.m[4] * y + iM.m[5];
  float a = affine_sample(m1, W, H, W, xs, ys);
  float b = affine_sample(m2, W, H, W, xs, ys);
  if (flow_out) {
    a = a - (float)x;
    b = b - (float)y;
  }
  if (I1[(size_t)y * p1 + x] <= 1) a = b = 0.0f;
  reinterpret_cast<float *>(reinterpret_cast<char *>(u) + (size_t)y * fp)[x] = a;
  reinterpret_cast<float *>(reinterpret_cast<char *>(v) + (size_t)y * fp)[x] = b;
}

// ---------------------------------------------------------------- host: homography
struct Pt {
  double x, y;
};

// normalised DLT of a homography from n >= 4 correspondences (a -> b); false if degenerate
static bool dlt_homography(const std::vector<Pt> &a, const std::vector<Pt> &b, double H[9]) {
  const size_t n = a.size();
  if (n < 4) return false;
  auto norm = [](const std::vector<Pt> &p, double T[9]) {
    double mx = 0, my = 0;
    for (auto &q : p) mx += q.x, my += q.y;
    mx /= p.size();
    my /= p.size();
    double d = 0;
    for (auto &q : p) d += std::hypot(q.x - mx, q.y - my);
    d /= p.size();
    const double s = d > 0 ? std::sqrt(2.0) / d : 1.0;
    const double t[9] = {s, 0, -s * mx, 0, s, -s * my, 0, 0, 1};
    std::copy(t, t + 9, T);
  };
  double Ta[9], Tb[9];
  norm(a, Ta);
  norm(b, Tb);
  // normal equations of A h = 0 with h8 = 1 (8 unknowns), least squares
  double M[8][9] = {};
  for (size_t i = 0; i < n; ++i) {
    const double x = Ta[0] * a[i].x + Ta[2], y = Ta[4] * a[i].y + Ta[5];
    const double u = Tb[0] * b[i].x + Tb[2], w = Tb[4] * b[i].y + Tb[5];
    const double r1[9] = {x, y, 1, 0, 0, 0, -u * x, -u * y, u};
    const double r2[9] = {0, 0, 0, x, y, 1, -w * x, -w * y, w};
    for (int j = 0; j < 8; ++j)
      for (int k = 0; k < 9; ++k) M[j][k] += r1[j] * r1[k] + r2[j] * r2[k];
  }
  for (int c = 0; c < 8; ++c) {   // Gaussian elimination with partial pivoting
    int p = c;
    for (int r = c + 1; r < 8; ++r)
      if (std::fabs(M[r][c]) > std::fabs(M[p][c])) p = r;
    if (std::fabs(M[p][c]) < 1e-12) return false;
    for (int k = 0; k < 9; ++k) std::swap(M[c][k], M[p][k]);
    for (int r = 0; r < 8; ++r) {
      if (r == c) continue;
      const double f = M[r][c] / M[c][c];
      for (int k = c; k < 9; ++k) M[r][k] -= f * M[c][k];
    }
  }
  double Hn[9];
  for (int j = 0; j < 8; ++j) Hn[j] = M[j][8] / M[j][j];
  Hn[8] = 1.0;
  // H = Tb^-1 Hn Ta
  const double sb = Tb[0];
  const double Tbi[9] = {1 / sb, 0, -Tb[2] / sb, 0, 1 / sb, -Tb[5] / sb, 0, 0, 1};
  double T1[9] = {};
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      for (int k = 0; k < 3; ++k) T1[r * 3 + c] += Hn[r * 3 + k] * Ta[k * 3 + c];
  for (int r = 0; r < 9; ++r) H[r] = 0;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      for (int k = 0; k < 3; ++k) H[r * 3 + c] += Tbi[r * 3 + k] * T1[k * 3 + c];
  if (std::fabs(H[8]) < 1e-15) return false;
  for (int r = 0; r < 9; ++r) H[r] /= H[8];
  return std::isfinite(H[0]) && std::isfinite(H[4]);
}

static inline double reproj_err2(const double H[9], const Pt &a, const Pt &b) {
  const double w = H[6] * a.x + H[7] * a.y + H[8];
  const double x = (H[0] * a.x + H[1] * a.y + H[2]) / w, y = (H[3] * a.x + H[4] * a.y + H[5]) / w;
  return (x - b.x) * (x - b.x) + (y - b.y) * (y - b.y);
}

// findHomography's last step: Levenberg-Marquardt on the 8 free entries (H[8] = 1) over the
// inliers' reprojection residuals (HomographyRefineCallback: r = H(a) - b, analytic
// Jacobian), at most `iters` steps.  The LM form of OpenCV's LMSolver: the normal
// equations' diagonal scaled by (1 + lambda), lambda from 1e-3, /10 after a step that lowers
// the error and x10 (the step rejected) otherwise.
static void lm_refine(const std::vector<Pt> &a, const std::vector<Pt> &b, double H[9], int iters) {
  const size_t n = a.size();
  if (n < 4) return;
  auto err = [&](const double *h) {
    double e = 0.0;
    for (size_t i = 0; i < n; ++i) {
      const double hh[9] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], 1.0};
      e += reproj_err2(hh, a[i], b[i]);
    }
    return e;
  };
  double h[8];
  for (int k = 0; k < 8; ++k) h[k] = H[k] / H[8];
  double e = err(h), lambda = 1e-3;
  for (int it = 0; it < iters; ++it) {
    double A[8][8] = {}, g[8] = {};
    for (size_t i = 0; i < n; ++i) {
      const double x = a[i].x, y = a[i].y;
      const double w = h[6] * x + h[7] * y + 1.0;
      if (std::fabs(w) < 1e-12) continue;
      const double iw = 1.0 / w;
      const double X = (h[0] * x + h[1] * y + h[2]) * iw, Y = (h[3] * x + h[4] * y + h[5]) * iw;
      const double rx = X - b[i].x, ry = Y - b[i].y;
      const double jx[8] = {x * iw, y * iw, iw, 0, 0, 0, -X * x * iw, -X * y * iw};
      const double jy[8] = {0, 0, 0, x * iw, y * iw, iw, -Y * x * iw, -Y * y * iw};
      for (int r = 0; r < 8; ++r) {
        g[r] += jx[r] * rx + jy[r] * ry;
        for (int c = 0; c < 8; ++c) A[r][c] += jx[r] * jx[c] + jy[r] * jy[c];
      }
    }
    for (;;) {   // solve (A + lambda diag(A)) d = -g; retry with a larger lambda on failure
      double M[8][9];
      for (int r = 0; r < 8; ++r) {
        for (int c = 0; c < 8; ++c) M[r][c] = A[r][c] * (r == c ? 1.0 + lambda : 1.0);
        M[r][8] = -g[r];
      }
      bool ok = true;
      for (int c = 0; c < 8 && ok; ++c) {
        int p = c;
        for (int r = c + 1; r < 8; ++r)
          if (std::fabs(M[r][c]) > std::fabs(M[p][c])) p = r;
        if (std::fabs(M[p][c]) < 1e-300) {
          ok = false;
          break;
        }
        for (int k = 0; k < 9; ++k) std::swap(M[c][k], M[p][k]);
        for (int r = 0; r < 8; ++r) {
          if (r == c) continue;
          const double f = M[r][c] / M[c][c];
          for (int k = c; k < 9; ++k) M[r][k] -= f * M[c][k];
        }
      }
      if (!ok) return;
      double hn[8];
      for (int k = 0; k < 8; ++k) hn[k] = h[k] + M[k][8] / M[k][k];
      const double en = err(hn);
      if (std::isfinite(en) && en < e) {
        std::copy(hn, hn + 8, h);
        e = en;
        lambda = std::max(lambda / 10.0, 1e-16);
        break;
      }
      lambda *= 10.0;
      if (lambda > 1e16) return;
    }
  }
  for (int k = 0; k < 8; ++k) H[k] = h[k];
  H[8] = 1.0;
}

// cv::findHomography(src, dst, method, ransacReprojThreshold) restated: RANSAC (8) or LMEDS
// (4), iteration counts as OpenCV's registrators (below), a DLT refit on the inliers, then
// 10 Levenberg-Marquardt steps on their reprojection error (fundam.cpp's createLMSolver(
// HomographyRefineCallback, 10)).  Deterministic (fixed seed).  Returns false when no model
// is found; mask (n entries, optional) gets the inliers.
// The minimal-sample generator: a 64-bit LCG (Knuth's MMIX constants), its high 32 bits
// reduced mod n -- fully specified, so the oracle draws the same samples.
struct SampleRng {
  uint64_t s = 0x12345678u;
  int operator()(int n) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return (int)((uint32_t)(s >> 32) % (uint32_t)n);
  }
};

static bool find_homography(const std::vector<Pt> &a, const std::vector<Pt> &b, int method,
                            double thresh, double H[9], uint8_t *mask = nullptr) {
  const int n = (int)a.size();
  if (n < 4) return false;
  SampleRng pick;
  const bool lmeds = method == 4;
  const double t2 = thresh * thresh;
  double best[9];
  int best_in = -1;
  double best_med = 1e300;
  // RANSAC: <= 2000 iterations, cut by the 0.995-confidence rule as inliers are found.
  // LMEDS: OpenCV's LMeDS registrator fixes its count from an assumed outlier ratio of 0.45:
  // round(log(1 - 0.995) / log(1 - 0.55^4)) = 55 iterations.
  int iters = lmeds ? (int)std::lround(std::log(1 - 0.995) / std::log(1 - std::pow(1 - 0.45, 4)))
                    : 2000;
  for (int it = 0; it < iters; ++it) {
    int s[4];
    for (int k = 0; k < 4; ++k) {
      bool dup;
      do {
        s[k] = pick(n);
        dup = false;
        for (int j = 0; j < k; ++j) dup |= s[j] == s[k];
      } while (dup);
    }
    std::vector<Pt> sa = {a[s[0]], a[s[1]], a[s[2]], a[s[3]]}, sb = {b[s[0]], b[s[1]], b[s[2]], b[s[3]]};
    double h[9];
    if (!dlt_homography(sa, sb, h)) continue;
    if (lmeds) {
      std::vector<double> e(n);
      for (int i = 0; i < n; ++i) e[i] = reproj_err2(h, a[i], b[i]);
      std::nth_element(e.begin(), e.begin() + n / 2, e.end());
      if (e[n / 2] < best_med) {
        best_med = e[n / 2];
        std::copy(h, h + 9, best);
      }
    } else {
      int in = 0;
      for (int i = 0; i < n; ++i) in += reproj_err2(h, a[i], b[i]) <= t2;
      if (in > best_in) {
        best_in = in;
        std::copy(h, h + 9, best);
        const double ratio = (double)in / n;   // RANSACUpdateNumIters, confidence 0.995
        const double denom = std::log(1.0 - std::pow(ratio, 4));
        if (denom < 0) iters = std::min(iters, (int)std::ceil(std::log(1 - 0.995) / denom));
      }
    }
  }
  if (!lmeds && best_in < 4) return false;
  if (lmeds && best_med >= 1e300) return false;
  // inliers of the best hypothesis, then a least-squares refit.  LMEDS: OpenCV's robust
  // sigma from the median, floored at 0.001 px (LMeDSPointSetRegistrator::run), squared
  const double sg = lmeds ? std::max(2.5 * 1.4826 * (1 + 5.0 / std::max(1, n - 4)) * std::sqrt(best_med), 0.001) : 0;
  const double lt2 = lmeds ? sg * sg : t2;
  std::vector<Pt> ia, ib;
  for (int i = 0; i < n; ++i) {
    const bool in = reproj_err2(best, a[i], b[i]) <= lt2;
    if (mask) mask[i] = in ? 1 : 0;
    if (in) {
      ia.push_back(a[i]);
      ib.push_back(b[i]);
    }
  }
  double h[9];
  if (ia.size() >= 4 && dlt_homography(ia, ib, h)) std::copy(h, h + 9, best);
  if (ia.size() > 4) lm_refine(ia, ib, best, 10);
  std::copy(best, best + 9, H);
  return true;
}

// ORB's fixed test pattern stand-in: 256 point pairs in the 31x31 patch, each coordinate the
// sum of three uniform integers in [-6, 6] (near-Gaussian, sigma 6.5 ~ patch / 5), pairs
// outside the radius-13 disc redrawn (|rotated offset| <= 13 < 15).  Integer arithmetic
// from SampleRng's generator only, so the oracle regenerates the same table.
static std::vector<int> orb_pattern() {
  SampleRng rng;
  rng.s = 0x0B5EEDu;
  auto coord = [&]() { return rng(13) + rng(13) + rng(13) - 18; };
  std::vector<int> p;
  p.reserve(kOrbBits * 4);
  while ((int)p.size() < kOrbBits * 4) {
    const int x = coord(), y = coord();
    if (x * x + y * y > 13 * 13) continue;
    p.push_back(x);
    p.push_back(y);
  }
  return p;
}

}  // namespace tvl1k
