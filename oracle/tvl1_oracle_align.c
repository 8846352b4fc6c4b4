/*
 * tvl1_oracle_align.c — TEST INFRASTRUCTURE ONLY (see tvl1_oracle.h).
 *
 * CPU restatement of this build's feature pre-alignment, the path that
 * replaces the reference's find_alignment (/root/reference/src/features.cpp:46-167) and the
 * cv::cuda::warpAffine calls around it (/root/reference/src/optflow.cpp:366-377, 411-443).
 * It follows fibsem-optflow_amd/csrc/tvl1_align.hpp and the host half of
 * tvl1_find_alignment in tvl1_engine.hip operation for operation, so that the GPU's
 * keypoints, descriptors, match lists, homography and warps are compared bit for bit
 * (tests/test_align_gpu.py):
 *   - ORB pyramid: level 0 = float(u8); level l = cv::resize INTER_LINEAR of level l-1
 *     (orc_resize_hp, the same half-pixel kernel as k_resize_hp) at round(W / sf^l);
 *   - FAST-9 (threshold t, contiguous arc >= 9 of the radius-3 circle) at least `border`
 *     px inside, scored by the 7x7 Harris response of Sobel gradients (k = 0.04);
 *   - 3x3 non-maximum suppression (ties to the top-left px), the per-level quota of the
 *     best unique (score, position) keys, best first;
 *   - orientation as the unit vector of the radius-15 intensity centroid, 256 rBRIEF tests
 *     from the build's integer pattern table (the same generator as orb_pattern());
 *   - brute-force Hamming 2-NN (ties to the lower train index), the reference's ratio test
 *     over its min(train rows - 1, queries) loop bound (features.cpp:105-112) and distance
 *     sort, and findHomography: RANSAC / LMEDS over 4-point normalised DLTs with the build's
 *     fixed-seed sample generator, a DLT refit on the inliers and 10 Levenberg-Marquardt
 *     steps, then the reference's zoom check (features.cpp:131-166);
 *   - cv::cuda::warpAffine(INTER_LINEAR, BORDER_CONSTANT 0) on u8 and on the map fields:
 *     the inverse affine (invertAffineTransform, double, stored as float), float source
 *     coordinates, LinearFilter's bilinear taps, saturate_cast rounding for u8.
 *
 * PARITY UNPINNED against OpenCV: its bit_pattern_31_ table, FAST score and RNG are not in
 * the reference or this image (the pattern is a stand-in), and SURF is served by ORB.  This
 * file pins the GPU implementation to its own stated definition.
 */
#include "tvl1_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define IDX(x, y, w) ((size_t)(y) * (size_t)(w) + (size_t)(x))

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }

enum { ORB_HALF = 15, ORB_BITS = 256, MAXL = 64 };

/* ---------------------------------------------------------------- the pattern table */
/* SampleRng (tvl1_align.hpp): 64-bit LCG, high 32 bits mod n */
typedef struct {
  uint64_t s;
} Rng;
static int rng_next(Rng *r, int n) {
  r->s = r->s * 6364136223846793005ull + 1442695040888963407ull;
  return (int)((uint32_t)(r->s >> 32) % (uint32_t)n);
}

/* orb_pattern(): 512 points (256 pairs), coordinates the sum of three uniform [-6, 6] */
static void orb_pattern(int pat[ORB_BITS * 4]) {
  Rng r = {0x0B5EEDu};
  int k = 0;
  while (k < ORB_BITS * 4) {
    const int x = rng_next(&r, 13) + rng_next(&r, 13) + rng_next(&r, 13) - 18;
    const int y = rng_next(&r, 13) + rng_next(&r, 13) + rng_next(&r, 13) - 18;
    if (x * x + y * y > 13 * 13) continue;
    pat[k++] = x;
    pat[k++] = y;
  }
}

/* ---------------------------------------------------------------- pyramid geometry */
typedef struct {
  int L;
  int w[MAXL], h[MAXL], quota[MAXL];
} Geom;

/* orb_geom (tvl1_engine.hip) */
static void orb_geom(int W, int H, const tvl1_align_params *ap, Geom *g) {
  g->L = imin(imax(1, ap->nlevels), MAXL);
  const double sf = ap->scale_factor;
  for (int l = 0; l < g->L; ++l) {
    const double scale = 1.0 / pow(sf, l - ap->first_level);
    g->w[l] = l == 0 ? W : imax(1, (int)lrint(W * scale));
    g->h[l] = l == 0 ? H : imax(1, (int)lrint(H * scale));
  }
  const double f = 1.0 / sf;
  double nd = ap->nfeatures * (1 - f) / (1 - pow(f, g->L));
  int sum = 0;
  for (int l = 0; l < g->L - 1; ++l) {
    g->quota[l] = (int)lrint(nd);
    sum += g->quota[l];
    nd *= f;
  }
  g->quota[g->L - 1] = imax(ap->nfeatures - sum, 0);
}

/* ---------------------------------------------------------------- FAST-9 + Harris */
static const int kFastDx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
static const int kFastDy[16] = {-3, -3, -2, -1, 0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3};

static int arc9(unsigned m) {
  const unsigned mm = m | (m << 16);
  unsigned run = mm;
  for (int k = 1; k < 9; ++k) run &= mm >> k;
  return run != 0;
}

/* ka_fast_harris at one px (x, y) of a level image I (w x h, packed) */
static float fast_harris(const float *I, int w, int h, int x, int y, int border, float t) {
  if (!(x >= border && y >= border && x < w - border && y < h - border)) return 0.0f;
  const float c = I[IDX(x, y, w)];
  unsigned bright = 0, dark = 0;
  for (int k = 0; k < 16; ++k) {
    const float v = I[IDX(x + kFastDx[k], y + kFastDy[k], w)];
    bright |= (v > c + t ? 1u : 0u) << k;
    dark |= (v < c - t ? 1u : 0u) << k;
  }
  if (!(arc9(bright) || arc9(dark))) return 0.0f;
  float a = 0.f, b = 0.f, cc = 0.f;
  for (int dy = -3; dy <= 3; ++dy)
    for (int dx = -3; dx <= 3; ++dx) {
      const int px = x + dx, py = y + dy;
      const float *r0 = I + IDX(0, py - 1, w), *r1 = I + IDX(0, py, w), *r2 = I + IDX(0, py + 1, w);
      const float gx = (r0[px + 1] - r0[px - 1]) + 2.f * (r1[px + 1] - r1[px - 1]) +
                       (r2[px + 1] - r2[px - 1]);
      const float gy = (r2[px - 1] - r0[px - 1]) + 2.f * (r2[px] - r0[px]) + (r2[px + 1] - r0[px + 1]);
      a += gx * gx;
      b += gy * gy;
      cc += gx * gy;
    }
  const float s = 1.0f / (4.f * 255.f * 49.f);
  a *= s * s;
  b *= s * s;
  cc *= s * s;
  return fmaxf(a * b - cc * cc - 0.04f * (a + b) * (a + b), 1e-30f);
}

static float key_score(uint64_t k) {
  const uint32_t b = (uint32_t)(k >> 32);
  float f;
  memcpy(&f, &b, sizeof f);
  return f;
}

static int cmp_key_desc(const void *pa, const void *pb) {
  const uint64_t a = *(const uint64_t *)pa, b = *(const uint64_t *)pb;
  return a < b ? 1 : (a > b ? -1 : 0);
}

/* ---------------------------------------------------------------- keypoints + descriptors */
typedef struct {
  int n;
  float *x, *y;      /* level coordinates */
  int *level;
  double *px, *py;   /* level-0 coordinates */
  float *resp;
  uint32_t *desc;    /* 8 words per keypoint */
} OrbOut;

static void orb_free(OrbOut *o) {
  free(o->x);
  free(o->y);
  free(o->level);
  free(o->px);
  free(o->py);
  free(o->resp);
  free(o->desc);
  memset(o, 0, sizeof *o);
}

/* ka_blur7 */
static void blur7(const float *I, int w, int h, float *O) {
  const float g[7] = {0.07015933f, 0.13107488f, 0.19071282f, 0.21610594f, 0.19071282f,
                      0.13107488f, 0.07015933f};
#pragma omp parallel for schedule(static)
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      float s = 0.f;
      for (int dy = -3; dy <= 3; ++dy) {
        const float *r = I + IDX(0, imin(imax(y + dy, 0), h - 1), w);
        float t = 0.f;
        for (int dx = -3; dx <= 3; ++dx) t += g[dx + 3] * r[imin(imax(x + dx, 0), w - 1)];
        s += g[dy + 3] * t;
      }
      O[IDX(x, y, w)] = s;
    }
}

/* ka_describe for one keypoint */
static void describe(const float *I, int w, int cx, int cy, const int *pat, uint32_t *d) {
  float m01 = 0.f, m10 = 0.f;
  for (int v = -ORB_HALF; v <= ORB_HALF; ++v)
    for (int u = -ORB_HALF; u <= ORB_HALF; ++u) {
      if (u * u + v * v > ORB_HALF * ORB_HALF) continue;
      const float val = I[IDX(cx + u, cy + v, w)];
      m10 += (float)u * val;
      m01 += (float)v * val;
    }
  const float r = sqrtf(m10 * m10 + m01 * m01);
  const float cs = r > 0.f ? m10 / r : 1.f, sn = r > 0.f ? m01 / r : 0.f;
  for (int wd = 0; wd < ORB_BITS / 32; ++wd) {
    uint32_t bits = 0;
    for (int j = 0; j < 32; ++j) {
      const int *q = pat + 4 * (wd * 32 + j);
      const int ax = (int)rintf((float)q[0] * cs - (float)q[1] * sn);
      const int ay = (int)rintf((float)q[0] * sn + (float)q[1] * cs);
      const int bx = (int)rintf((float)q[2] * cs - (float)q[3] * sn);
      const int by = (int)rintf((float)q[2] * sn + (float)q[3] * cs);
      const float va = I[IDX(cx + ax, cy + ay, w)];
      const float vb = I[IDX(cx + bx, cy + by, w)];
      bits |= (va < vb ? 1u : 0u) << j;
    }
    d[wd] = bits;
  }
}

/* orb_detect (tvl1_engine.hip) on a host frame */
static int orb_run(const uint8_t *img, size_t pitch, int W, int H, const tvl1_align_params *ap,
                   OrbOut *out) {
  memset(out, 0, sizeof *out);
  Geom g;
  orb_geom(W, H, ap, &g);
  float *lev[MAXL];
  for (int l = 0; l < g.L; ++l) {
    lev[l] = (float *)malloc(sizeof(float) * (size_t)g.w[l] * g.h[l]);
    if (!lev[l]) return -1;
  }
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) lev[0][IDX(x, y, W)] = (float)img[(size_t)y * pitch + x];
  for (int l = 1; l < g.L; ++l)
    orc_resize_hp(lev[l - 1], g.w[l - 1], g.h[l - 1], lev[l], g.w[l], g.h[l],
                  (double)g.w[l - 1] / g.w[l], (double)g.h[l - 1] / g.h[l], 0);
  const int border = imax(ap->edge_threshold, ORB_HALF + 1);
  const float t = (float)ap->fast_threshold;
  int cap = 0;
  for (int l = 0; l < g.L; ++l) cap += g.quota[l];
  out->x = (float *)malloc(sizeof(float) * (cap + 1));
  out->y = (float *)malloc(sizeof(float) * (cap + 1));
  out->level = (int *)malloc(sizeof(int) * (cap + 1));
  out->px = (double *)malloc(sizeof(double) * (cap + 1));
  out->py = (double *)malloc(sizeof(double) * (cap + 1));
  out->resp = (float *)malloc(sizeof(float) * (cap + 1));
  for (int l = 0; l < g.L; ++l) {
    const int w = g.w[l], h = g.h[l];
    if (w <= 2 * border || h <= 2 * border || g.quota[l] == 0) continue;
    float *score = (float *)malloc(sizeof(float) * (size_t)w * h);
    uint64_t *keys = (uint64_t *)malloc(sizeof(uint64_t) * ((size_t)(w + 1) / 2 * ((h + 1) / 2) + 1));
#pragma omp parallel for schedule(static)
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) score[IDX(x, y, w)] = fast_harris(lev[l], w, h, x, y, border, t);
    size_t nk = 0;   /* ka_nms, in raster order (the set, not the order, matters) */
    for (int y = 1; y < h - 1; ++y)
      for (int x = 1; x < w - 1; ++x) {
        const float s = score[IDX(x, y, w)];
        int keep = s > 0.0f;
        for (int dy = -1; dy <= 1 && keep; ++dy)
          for (int dx = -1; dx <= 1; ++dx) {
            if (!dx && !dy) continue;
            const float o = score[IDX(x + dx, y + dy, w)];
            if (o > s || (o == s && (dy < 0 || (dy == 0 && dx < 0)))) keep = 0;
          }
        if (keep) {
          uint32_t sb;
          memcpy(&sb, &s, sizeof sb);
          keys[nk++] = ((uint64_t)sb << 32) | (uint64_t)(0xFFFFFFFFu - (unsigned)(y * w + x));
        }
      }
    /* ka_select + the host's best-first order: the quota largest keys, descending */
    qsort(keys, nk, sizeof(uint64_t), cmp_key_desc);
    const size_t m = nk < (size_t)g.quota[l] ? nk : (size_t)g.quota[l];
    const double scale = pow(ap->scale_factor, l - ap->first_level);
    for (size_t i = 0; i < m; ++i) {
      const unsigned pos = 0xFFFFFFFFu - (unsigned)(keys[i] & 0xFFFFFFFFu);
      const float x = (float)(pos % (unsigned)w), y = (float)(pos / (unsigned)w);
      const int k = out->n++;
      out->x[k] = x;
      out->y[k] = y;
      out->level[k] = l;
      out->px[k] = x * scale;
      out->py[k] = y * scale;
      out->resp[k] = key_score(keys[i]);
    }
    free(score);
    free(keys);
  }
  if (ap->blur_for_descriptor)
    for (int l = 0; l < g.L; ++l) {
      float *b = (float *)malloc(sizeof(float) * (size_t)g.w[l] * g.h[l]);
      blur7(lev[l], g.w[l], g.h[l], b);
      free(lev[l]);
      lev[l] = b;
    }
  int pat[ORB_BITS * 4];
  orb_pattern(pat);
  out->desc = (uint32_t *)malloc(sizeof(uint32_t) * 8 * (size_t)(out->n + 1));
#pragma omp parallel for schedule(static)
  for (int i = 0; i < out->n; ++i)
    describe(lev[out->level[i]], g.w[out->level[i]], (int)out->x[i], (int)out->y[i], pat,
             out->desc + 8 * (size_t)i);
  for (int l = 0; l < g.L; ++l) free(lev[l]);
  return out->n;
}

int orc_orb_detect(const uint8_t *img, size_t pitch, int w, int h, const tvl1_align_params *ap,
                   float *kp, uint8_t *desc, int cap) {
  OrbOut o;
  const int n = orb_run(img, pitch, w, h, ap, &o);
  if (n < 0) return -1;
  const int m = imin(n, cap);
  for (int i = 0; i < m; ++i) {
    kp[5 * i + 0] = (float)o.px[i];
    kp[5 * i + 1] = (float)o.py[i];
    kp[5 * i + 2] = (float)o.level[i];
    kp[5 * i + 3] = 0.0f;   /* the angle is not restated (reported only, atan2f) */
    kp[5 * i + 4] = o.resp[i];
  }
  if (m > 0) memcpy(desc, o.desc, (size_t)m * 32);
  orb_free(&o);
  return n;
}

/* ---------------------------------------------------------------- matching */
static void top2_push(int *b0, int *b1, int *d0, int *d1, int hd, int j) {
  if (hd < *d0) {
    *d1 = *d0;
    *b1 = *b0;
    *d0 = hd;
    *b0 = j;
  } else if (hd < *d1) {
    *d1 = hd;
    *b1 = j;
  }
}

static void match_knn2(const uint32_t *q, int nq, const uint32_t *t, int nt, int32_t *idx,
                       int32_t *dist) {
#pragma omp parallel for schedule(static)
  for (int i = 0; i < nq; ++i) {
    int b0 = -1, b1 = -1, d0 = 1 << 30, d1 = 1 << 30;
    for (int j = 0; j < nt; ++j) {
      int hd = 0;
      for (int w = 0; w < 8; ++w) hd += __builtin_popcount(q[8 * (size_t)i + w] ^ t[8 * (size_t)j + w]);
      top2_push(&b0, &b1, &d0, &d1, hd, j);
    }
    idx[2 * i] = b0;
    idx[2 * i + 1] = b1;
    dist[2 * i] = d0;
    dist[2 * i + 1] = d1;
  }
}

void orc_match_knn2(const uint8_t *q, int nq, const uint8_t *t, int nt, int32_t *idx,
                    int32_t *dist) {
  /* the descriptors as 8 little-endian words each (the device layout) */
  uint32_t *qw = (uint32_t *)malloc(sizeof(uint32_t) * 8 * (size_t)(nq + 1));
  uint32_t *tw = (uint32_t *)malloc(sizeof(uint32_t) * 8 * (size_t)(nt + 1));
  memcpy(qw, q, (size_t)nq * 32);
  if (nt > 0) memcpy(tw, t, (size_t)nt * 32);
  match_knn2(qw, nq, tw, nt, idx, dist);
  free(qw);
  free(tw);
}

/* ---------------------------------------------------------------- findHomography */
typedef struct {
  double x, y;
} Pt;

static void dlt_norm(const Pt *p, size_t n, double T[9]) {
  double mx = 0, my = 0;
  for (size_t i = 0; i < n; ++i) mx += p[i].x, my += p[i].y;
  mx /= n;
  my /= n;
  double d = 0;
  for (size_t i = 0; i < n; ++i) d += hypot(p[i].x - mx, p[i].y - my);
  d /= n;
  const double s = d > 0 ? sqrt(2.0) / d : 1.0;
  const double t[9] = {s, 0, -s * mx, 0, s, -s * my, 0, 0, 1};
  memcpy(T, t, sizeof t);
}

/* dlt_homography (tvl1_align.hpp) */
static int dlt_homography(const Pt *a, const Pt *b, size_t n, double H[9]) {
  if (n < 4) return 0;
  double Ta[9], Tb[9];
  dlt_norm(a, n, Ta);
  dlt_norm(b, n, Tb);
  double M[8][9];
  memset(M, 0, sizeof M);
  for (size_t i = 0; i < n; ++i) {
    const double x = Ta[0] * a[i].x + Ta[2], y = Ta[4] * a[i].y + Ta[5];
    const double u = Tb[0] * b[i].x + Tb[2], w = Tb[4] * b[i].y + Tb[5];
    const double r1[9] = {x, y, 1, 0, 0, 0, -u * x, -u * y, u};
    const double r2[9] = {0, 0, 0, x, y, 1, -w * x, -w * y, w};
    for (int j = 0; j < 8; ++j)
      for (int k = 0; k < 9; ++k) M[j][k] += r1[j] * r1[k] + r2[j] * r2[k];
  }
  for (int c = 0; c < 8; ++c) {
    int p = c;
    for (int r = c + 1; r < 8; ++r)
      if (fabs(M[r][c]) > fabs(M[p][c])) p = r;
    if (fabs(M[p][c]) < 1e-12) return 0;
    for (int k = 0; k < 9; ++k) {
      const double tmp = M[c][k];
      M[c][k] = M[p][k];
      M[p][k] = tmp;
    }
    for (int r = 0; r < 8; ++r) {
      if (r == c) continue;
      const double f = M[r][c] / M[c][c];
      for (int k = c; k < 9; ++k) M[r][k] -= f * M[c][k];
    }
  }
  double Hn[9];
  for (int j = 0; j < 8; ++j) Hn[j] = M[j][8] / M[j][j];
  Hn[8] = 1.0;
  const double sb = Tb[0];
  const double Tbi[9] = {1 / sb, 0, -Tb[2] / sb, 0, 1 / sb, -Tb[5] / sb, 0, 0, 1};
  double T1[9] = {0};
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      for (int k = 0; k < 3; ++k) T1[r * 3 + c] += Hn[r * 3 + k] * Ta[k * 3 + c];
  for (int r = 0; r < 9; ++r) H[r] = 0;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      for (int k = 0; k < 3; ++k) H[r * 3 + c] += Tbi[r * 3 + k] * T1[k * 3 + c];
  if (fabs(H[8]) < 1e-15) return 0;
  for (int r = 0; r < 9; ++r) H[r] /= H[8];
  return isfinite(H[0]) && isfinite(H[4]);
}

static double reproj_err2(const double H[9], Pt a, Pt b) {
  const double w = H[6] * a.x + H[7] * a.y + H[8];
  const double x = (H[0] * a.x + H[1] * a.y + H[2]) / w, y = (H[3] * a.x + H[4] * a.y + H[5]) / w;
  return (x - b.x) * (x - b.x) + (y - b.y) * (y - b.y);
}

static double lm_err(const Pt *a, const Pt *b, size_t n, const double *h) {
  double e = 0.0;
  const double hh[9] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], 1.0};
  for (size_t i = 0; i < n; ++i) e += reproj_err2(hh, a[i], b[i]);
  return e;
}

/* lm_refine (tvl1_align.hpp) */
static void lm_refine(const Pt *a, const Pt *b, size_t n, double H[9], int iters) {
  if (n < 4) return;
  double h[8];
  for (int k = 0; k < 8; ++k) h[k] = H[k] / H[8];
  double e = lm_err(a, b, n, h), lambda = 1e-3;
  for (int it = 0; it < iters; ++it) {
    double A[8][8], g[8];
    memset(A, 0, sizeof A);
    memset(g, 0, sizeof g);
    for (size_t i = 0; i < n; ++i) {
      const double x = a[i].x, y = a[i].y;
      const double w = h[6] * x + h[7] * y + 1.0;
      if (fabs(w) < 1e-12) continue;
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
    for (;;) {
      double M[8][9];
      for (int r = 0; r < 8; ++r) {
        for (int c = 0; c < 8; ++c) M[r][c] = A[r][c] * (r == c ? 1.0 + lambda : 1.0);
        M[r][8] = -g[r];
      }
      int ok = 1;
      for (int c = 0; c < 8 && ok; ++c) {
        int p = c;
        for (int r = c + 1; r < 8; ++r)
          if (fabs(M[r][c]) > fabs(M[p][c])) p = r;
        if (fabs(M[p][c]) < 1e-300) {
          ok = 0;
          break;
        }
        for (int k = 0; k < 9; ++k) {
          const double tmp = M[c][k];
          M[c][k] = M[p][k];
          M[p][k] = tmp;
        }
        for (int r = 0; r < 8; ++r) {
          if (r == c) continue;
          const double f = M[r][c] / M[c][c];
          for (int k = c; k < 9; ++k) M[r][k] -= f * M[c][k];
        }
      }
      if (!ok) return;
      double hn[8];
      for (int k = 0; k < 8; ++k) hn[k] = h[k] + M[k][8] / M[k][k];
      const double en = lm_err(a, b, n, hn);
      if (isfinite(en) && en < e) {
        memcpy(h, hn, sizeof h);
        e = en;
        lambda = fmax(lambda / 10.0, 1e-16);
        break;
      }
      lambda *= 10.0;
      if (lambda > 1e16) return;
    }
  }
  for (int k = 0; k < 8; ++k) H[k] = h[k];
  H[8] = 1.0;
}

static int cmp_double(const void *pa, const void *pb) {
  const double a = *(const double *)pa, b = *(const double *)pb;
  return a < b ? -1 : (a > b ? 1 : 0);
}

/* find_homography (tvl1_align.hpp) */
static int find_homography(const Pt *a, const Pt *b, int n, int method, double thresh,
                           double H[9], uint8_t *mask) {
  if (n < 4) return 0;
  Rng rng = {0x12345678u};
  const int lmeds = method == 4;
  const double t2 = thresh * thresh;
  double best[9] = {0};
  int best_in = -1;
  double best_med = 1e300;
  int iters = lmeds ? (int)lround(log(1 - 0.995) / log(1 - pow(1 - 0.45, 4))) : 2000;
  double *e = lmeds ? (double *)malloc(sizeof(double) * n) : NULL;
  for (int it = 0; it < iters; ++it) {
    int s[4];
    for (int k = 0; k < 4; ++k) {
      int dup;
      do {
        s[k] = rng_next(&rng, n);
        dup = 0;
        for (int j = 0; j < k; ++j) dup |= s[j] == s[k];
      } while (dup);
    }
    const Pt sa[4] = {a[s[0]], a[s[1]], a[s[2]], a[s[3]]};
    const Pt sb[4] = {b[s[0]], b[s[1]], b[s[2]], b[s[3]]};
    double h[9];
    if (!dlt_homography(sa, sb, 4, h)) continue;
    if (lmeds) {
      for (int i = 0; i < n; ++i) e[i] = reproj_err2(h, a[i], b[i]);
      qsort(e, n, sizeof(double), cmp_double);   /* the n/2-th smallest, as nth_element */
      if (e[n / 2] < best_med) {
        best_med = e[n / 2];
        memcpy(best, h, sizeof best);
      }
    } else {
      int in = 0;
      for (int i = 0; i < n; ++i) in += reproj_err2(h, a[i], b[i]) <= t2;
      if (in > best_in) {
        best_in = in;
        memcpy(best, h, sizeof best);
        const double ratio = (double)in / n;
        const double denom = log(1.0 - pow(ratio, 4));
        if (denom < 0) iters = imin(iters, (int)ceil(log(1 - 0.995) / denom));
      }
    }
  }
  free(e);
  if (!lmeds && best_in < 4) return 0;
  if (lmeds && best_med >= 1e300) return 0;
  /* LMEDS: sigma = 2.5 * 1.4826 * (1 + 5 / (n - 4)) * sqrt(median), floored at 0.001 px */
  double sg = lmeds ? 2.5 * 1.4826 * (1 + 5.0 / imax(1, n - 4)) * sqrt(best_med) : 0;
  if (lmeds && sg < 0.001) sg = 0.001;
  const double lt2 = lmeds ? sg * sg : t2;
  Pt *ia = (Pt *)malloc(sizeof(Pt) * n), *ib = (Pt *)malloc(sizeof(Pt) * n);
  size_t ni = 0;
  for (int i = 0; i < n; ++i) {
    const int in = reproj_err2(best, a[i], b[i]) <= lt2;
    if (mask) mask[i] = in ? 1 : 0;
    if (in) {
      ia[ni] = a[i];
      ib[ni] = b[i];
      ++ni;
    }
  }
  double h[9];
  if (ni >= 4 && dlt_homography(ia, ib, ni, h)) memcpy(best, h, sizeof best);
  if (ni > 4) lm_refine(ia, ib, ni, best, 10);
  free(ia);
  free(ib);
  memcpy(H, best, sizeof best);
  return 1;
}

int orc_find_homography(const double *src_xy, const double *dst_xy, int n, int method,
                        double thresh, double H[9], uint8_t *mask) {
  Pt *a = (Pt *)malloc(sizeof(Pt) * (n + 1)), *b = (Pt *)malloc(sizeof(Pt) * (n + 1));
  for (int i = 0; i < n; ++i) {
    a[i].x = src_xy[2 * i];
    a[i].y = src_xy[2 * i + 1];
    b[i].x = dst_xy[2 * i];
    b[i].y = dst_xy[2 * i + 1];
  }
  const int ok = find_homography(a, b, n, method, thresh, H, mask);
  free(a);
  free(b);
  return ok;
}

/* ---------------------------------------------------------------- find_alignment */
typedef struct {
  int qi, ti, d;
} Good;

static int cmp_good(const void *pa, const void *pb) {   /* stable: distance, then order */
  const Good *a = (const Good *)pa, *b = (const Good *)pb;
  if (a->d != b->d) return a->d < b->d ? -1 : 1;
  return a->qi < b->qi ? -1 : (a->qi > b->qi ? 1 : 0);
}

int orc_find_alignment(const uint8_t *frame1, size_t pitch1, int w1, int h1,
                       const uint8_t *frame0, size_t pitch0, int w0, int h0,
                       const tvl1_align_params *ap, float affine[6], int *n_good,
                       int *outcome) {
  OrbOut q, t;
  if (orb_run(frame1, pitch1, w1, h1, ap, &q) < 0) return -1;
  if (orb_run(frame0, pitch0, w0, h0, ap, &t) < 0) {
    orb_free(&q);
    return -1;
  }
  const int nq = q.n, nt = t.n;
  int32_t *idx = (int32_t *)malloc(sizeof(int32_t) * 2 * (nq + 1));
  int32_t *dist = (int32_t *)malloc(sizeof(int32_t) * 2 * (nq + 1));
  if (nq > 0 && nt > 0) match_knn2(q.desc, nq, t.desc, nt, idx, dist);
  Good *good = (Good *)malloc(sizeof(Good) * (nq + 1));
  int ng = 0;
  const int lim = imin(nt - 1, nq);   /* features.cpp:105-112's loop bound */
  for (int i = 0; i < lim; ++i)
    if (idx[2 * i + 1] >= 0 && (float)dist[2 * i] < ap->ratio * (float)dist[2 * i + 1])
      good[ng++] = (Good){i, idx[2 * i], dist[2 * i]};
  qsort(good, ng, sizeof(Good), cmp_good);
  if (n_good) *n_good = ng;
  const float ident[6] = {1, 0, 0, 0, 1, 0};
  int oc = 0;
  if (ng > 10) {
    Pt *p0 = (Pt *)malloc(sizeof(Pt) * ng), *p1 = (Pt *)malloc(sizeof(Pt) * ng);
    for (int i = 0; i < ng; ++i) {
      p0[i].x = q.px[good[i].qi];
      p0[i].y = q.py[good[i].qi];
      p1[i].x = t.px[good[i].ti];
      p1[i].y = t.py[good[i].ti];
    }
    double H[9];
    const int ok = find_homography(p0, p1, ng, ap->method, ap->ransac_threshold, H, NULL);
    if (!ok || fabs(1 - H[0]) > 0.20 || fabs(1 - H[4]) > 0.20) {
      memcpy(affine, ident, sizeof ident);
      oc = 2;
    } else {
      for (int k = 0; k < 6; ++k) affine[k] = (float)H[k];
    }
    free(p0);
    free(p1);
  } else {
    memcpy(affine, ident, sizeof ident);
    oc = 1;
  }
  if (outcome) *outcome = oc;
  free(idx);
  free(dist);
  free(good);
  orb_free(&q);
  orb_free(&t);
  return 0;
}

/* ---------------------------------------------------------------- warpAffine */
/* cv::invertAffineTransform in double, stored as float (affine_inverse) */
static void affine_inverse(const float M[6], float iM[6]) {
  const double a = M[0], b = M[1], cc = M[2], d = M[3], e = M[4], f = M[5];
  double D = a * e - b * d;
  D = D != 0 ? 1.0 / D : 0.0;
  const double A11 = e * D, A22 = a * D, A12 = -b * D, A21 = -d * D;
  iM[0] = (float)A11;
  iM[1] = (float)A12;
  iM[2] = (float)(-A11 * cc - A12 * f);
  iM[3] = (float)A21;
  iM[4] = (float)A22;
  iM[5] = (float)(-A21 * cc - A22 * f);
}

/* LinearFilter over BORDER_CONSTANT 0: four taps in (x1, y1), (x2, y1), (x1, y2), (x2, y2)
 * order, each weight a product of two float differences */
#define AFFINE_TAPS(AT, xs, ys, out)                                                  \
  do {                                                                                \
    const float x1f = floorf(xs), y1f = floorf(ys);                                   \
    const int x1 = (int)x1f, y1 = (int)y1f, x2 = x1 + 1, y2 = y1 + 1;                 \
    out = 0.0f;                                                                       \
    out = out + AT(y1, x1) * (((float)x2 - xs) * ((float)y2 - ys));                   \
    out = out + AT(y1, x2) * ((xs - (float)x1) * ((float)y2 - ys));                   \
    out = out + AT(y2, x1) * (((float)x2 - xs) * (ys - (float)y1));                   \
    out = out + AT(y2, x2) * ((xs - (float)x1) * (ys - (float)y1));                   \
  } while (0)

void orc_warp_affine_u8(const uint8_t *src, size_t sp, int sw, int sh, uint8_t *dst, size_t dp,
                        int dw, int dh, const float affine[6]) {
  float m[6];
  affine_inverse(affine, m);
#define AT_U8(yy, xx) \
  (((xx) >= 0 && (yy) >= 0 && (xx) < sw && (yy) < sh) ? (float)src[(size_t)(yy) * sp + (xx)] : 0.0f)
#pragma omp parallel for schedule(static)
  for (int y = 0; y < dh; ++y)
    for (int x = 0; x < dw; ++x) {
      const float xs = m[0] * x + m[1] * y + m[2];
      const float ys = m[3] * x + m[4] * y + m[5];
      float out;
      AFFINE_TAPS(AT_U8, xs, ys, out);
      dst[(size_t)y * dp + x] = (uint8_t)fminf(fmaxf(rintf(out), 0.0f), 255.0f);
    }
#undef AT_U8
}

void orc_postprocess_affine(float *u, float *v, size_t fp, const uint8_t *I1, size_t p1, int W,
                            int H, int flow_output, const float affine[6]) {
  float m[6];
  affine_inverse(affine, m);
  float *m1 = (float *)malloc(sizeof(float) * (size_t)W * H);
  float *m2 = (float *)malloc(sizeof(float) * (size_t)W * H);
  for (int y = 0; y < H; ++y) {   /* ka_map_stage: map = flow + grid */
    const float *ur = (const float *)((const char *)u + (size_t)y * fp);
    const float *vr = (const float *)((const char *)v + (size_t)y * fp);
    for (int x = 0; x < W; ++x) {
      m1[IDX(x, y, W)] = ur[x] + (float)x;
      m2[IDX(x, y, W)] = vr[x] + (float)y;
    }
  }
#define AT_M1(yy, xx) \
  (((xx) >= 0 && (yy) >= 0 && (xx) < W && (yy) < H) ? m1[(size_t)(yy) * W + (xx)] : 0.0f)
#define AT_M2(yy, xx) \
  (((xx) >= 0 && (yy) >= 0 && (xx) < W && (yy) < H) ? m2[(size_t)(yy) * W + (xx)] : 0.0f)
#pragma omp parallel for schedule(static)
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {   /* ka_map_warp */
      const float xs = m[0] * x + m[1] * y + m[2];
      const float ys = m[3] * x + m[4] * y + m[5];
      float a, b;
      AFFINE_TAPS(AT_M1, xs, ys, a);
      AFFINE_TAPS(AT_M2, xs, ys, b);
      if (flow_output) {
        a = a - (float)x;
        b = b - (float)y;
      }
      if (I1[(size_t)y * p1 + x] <= 1) a = b = 0.0f;
      ((float *)((char *)u + (size_t)y * fp))[x] = a;
      ((float *)((char *)v + (size_t)y * fp))[x] = b;
    }
#undef AT_M1
#undef AT_M2
  free(m1);
  free(m2);
}
