/*
 * tvl1_oracle_dualtvl1.c — TEST INFRASTRUCTURE ONLY (see tvl1_oracle.h).
 *
 * Profile 1 (tvl1_params.profile): the schedule of
 * OpenCV's CPU cv::DualTVL1OpticalFlow (opencv/modules/video/src/tvl1flow.cpp, 3.4.1),
 * which BASELINE.json configs[0] names ("OpenCV DualTVL1 CPU") but which the reference
 * CLI cannot run (it only calls the CUDA solver, /root/reference/src/optflow.cpp:518).
 * Restated from the published OpenCV 3.4.1 sources as recalled; OpenCV is absent here.
 *
 * PARITY UNPINNED, and more loosely than profile 0: besides the absent reference, these
 * details are recalled, not verified:
 *   - cv::resize INTER_LINEAR on CV_32F: half-pixel source coordinate computed in double
 *     and cast to float, x clamped to the edge columns (fx := 0), y NOT clamped (the two
 *     rows are clamped, the weights kept), separable float weights 1-f, f;
 *   - remap INTER_CUBIC: map x + u rounded to 1/32 px (cvRound), Keys a = -0.75 table
 *     (interpolateCubic), 4x4 taps, BORDER_CONSTANT 0 (taps outside add nothing);
 *   - the residual of every inner iteration, here summed in double and cast to float;
 *   - |grad u| as hypotf, here (float) sqrt((double) a*a + (double) b*b) (glibc);
 *   - IPP / SIMD code paths OpenCV may take instead of the generic loops.
 * Everything else (TH step, divergence, projection, median, stopping rule) follows
 * the same expressions as profile 0 (tvl1_oracle.c), with the CPU's association of rho.
 */
#include "tvl1_oracle.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define IDX(x, y, w) ((size_t)(y) * (size_t)(w) + (size_t)(x))

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }

double orc_survey_bytes(int L, const int *ws, const int *hs, int warps, const int64_t *iters);

/* cv::resize INTER_LINEAR, CV_32F (resize.cpp: the coefficient setup of resize(),
 * HResizeLinear / VResizeLinear), or the 2x INTER_AREA fast path it switches to. */
void orc_resize_hp(const float *src, int sw, int sh, float *dst, int dw, int dh,
                   double scale_x, double scale_y, int area_fast) {
  if (sw == dw && sh == dh) {   /* resize(): dsize == ssize -> copyTo */
    memcpy(dst, src, sizeof(float) * (size_t)sw * sh);
    return;
  }
  if (area_fast) {   /* resizeAreaFast, scale 2: ((a + b) + c) + d, times 0.25f */
#pragma omp parallel for schedule(static)
    for (int dy = 0; dy < dh; ++dy)
      for (int dx = 0; dx < dw; ++dx) {
        const float *S = src + IDX(2 * dx, 2 * dy, sw);
        dst[IDX(dx, dy, dw)] = (S[0] + S[1] + S[sw] + S[sw + 1]) * 0.25f;
      }
    return;
  }
#pragma omp parallel for schedule(static)
  for (int dy = 0; dy < dh; ++dy) {
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    const float b0 = 1.f - fy, b1 = fy;
    const int r0 = imin(imax(sy, 0), sh - 1), r1 = imin(imax(sy + 1, 0), sh - 1);
    for (int dx = 0; dx < dw; ++dx) {
      float fx = (float)((dx + 0.5) * scale_x - 0.5);
      int sx = (int)floorf(fx);
      fx -= (float)sx;
      if (sx < 0) fx = 0.f, sx = 0;
      const int single = sx + 1 >= sw;
      if (sx >= sw - 1) fx = 0.f, sx = sw - 1;
      const float a0 = 1.f - fx, a1 = fx;
      const float *S0 = src + IDX(0, r0, sw), *S1 = src + IDX(0, r1, sw);
      const float t0 = single ? S0[sx] * 1.0f : S0[sx] * a0 + S0[sx + 1] * a1;
      const float t1 = single ? S1[sx] * 1.0f : S1[sx] * a0 + S1[sx + 1] * a1;
      dst[IDX(dx, dy, dw)] = t0 * b0 + t1 * b1;
    }
  }
}

/* imgproc interpolateCubic (a = -0.75) at x = i / 32 (initInterTab1D) */
static void cubic_tab(float tab[32][4]) {
  const float A = -0.75f;
  for (int i = 0; i < 32; ++i) {
    const float x = (float)i * (1.f / 32);
    tab[i][0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
    tab[i][1] = ((A + 2) * x - (A + 3)) * x * x + 1;
    tab[i][2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
    tab[i][3] = 1.f - tab[i][0] - tab[i][1] - tab[i][2];
  }
}

/* cvRound of a float map coordinate times INTER_TAB_SIZE: nearest-even, the x86
 * "integer indefinite" INT_MIN outside the int range (and for NaN) */
static inline int round_map(float v) {
  if (!(v > -2147483648.f && v < 2147483648.f)) return INT_MIN;
  return (int)lrintf(v);
}
static inline int sat_short(int v) { return v < -32768 ? -32768 : v > 32767 ? 32767 : v; }

/* remapBicubic<float> with BORDER_CONSTANT 0 at one px for one plane */
static inline float remap_px(const float *S, int w, int h, int sx, int sy, const float *wt) {
  if ((unsigned)sx < (unsigned)imax(w - 3, 0) && (unsigned)sy < (unsigned)imax(h - 3, 0)) {
    const float *r = S + IDX(sx, sy, w);
    float sum = r[0] * wt[0] + r[1] * wt[1] + r[2] * wt[2] + r[3] * wt[3];
    r += w;
    sum += r[0] * wt[4] + r[1] * wt[5] + r[2] * wt[6] + r[3] * wt[7];
    r += w;
    sum += r[0] * wt[8] + r[1] * wt[9] + r[2] * wt[10] + r[3] * wt[11];
    r += w;
    sum += r[0] * wt[12] + r[1] * wt[13] + r[2] * wt[14] + r[3] * wt[15];
    return sum;
  }
  if (sx >= w || sx + 4 <= 0 || sy >= h || sy + 4 <= 0) return 0.0f;
  float sum = 0.0f * 1.0f;
  for (int i = 0; i < 4; ++i) {
    const int yi = sy + i;
    if (yi < 0 || yi >= h) continue;
    for (int j = 0; j < 4; ++j) {
      const int xj = sx + j;
      if (xj < 0 || xj >= w) continue;
      sum += (S[IDX(xj, yi, w)] - 0.0f) * wt[i * 4 + j];
    }
  }
  return sum;
}

void orc_remap_cubic(const float *I0, const float *I1, const float *I1x, const float *I1y,
                     const float *u1, const float *u2, int w, int h, float *I1wx,
                     float *I1wy, float *grad, float *rho_c) {
  float tab[32][4];
  cubic_tab(tab);
#pragma omp parallel for schedule(static)
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const size_t i = IDX(x, y, w);
      /* buildFlowMap: map = x + u (float) */
      const float X = (float)x + u1[i], Y = (float)y + u2[i];
      const int ix = round_map(X * 32.f), iy = round_map(Y * 32.f);
      const int sx = sat_short(ix >> 5) - 1, sy = sat_short(iy >> 5) - 1;
      const int fx = ix & 31, fy = iy & 31;
      float wt[16];
      for (int k1 = 0; k1 < 4; ++k1)
        for (int k2 = 0; k2 < 4; ++k2) wt[k1 * 4 + k2] = tab[fy][k1] * tab[fx][k2];
      const float I1w = remap_px(I1, w, h, sx, sy, wt);
      const float wx = remap_px(I1x, w, h, sx, sy, wt);
      const float wy = remap_px(I1y, w, h, sx, sy, wt);
      /* calcGradRho */
      const float Ix2 = wx * wx;
      const float Iy2 = wy * wy;
      I1wx[i] = wx;
      I1wy[i] = wy;
      grad[i] = Ix2 + Iy2;
      rho_c[i] = I1w - wx * u1[i] - wy * u2[i] - I0[i];
    }
}

static inline float divergence(const float *v1, const float *v2, int y, int x, int w) {
  if (x > 0 && y > 0) {
    const float v1x = v1[IDX(x, y, w)] - v1[IDX(x - 1, y, w)];
    const float v2y = v2[IDX(x, y, w)] - v2[IDX(x, y - 1, w)];
    return v1x + v2y;
  }
  if (y > 0) return v1[IDX(0, y, w)] + v2[IDX(0, y, w)] - v2[IDX(0, y - 1, w)];
  if (x > 0) return v1[IDX(x, 0, w)] - v1[IDX(x - 1, 0, w)] + v2[IDX(x, 0, w)];
  return v1[0] + v2[0];
}

/* estimateV + divergence + estimateU of one inner iteration; returns the residual */
static double estimate_u_cpu(const float *I1wx, const float *I1wy, const float *grad,
                             const float *rho_c, const float *p11, const float *p12,
                             const float *p21, const float *p22, const float *p31,
                             const float *p32, float *u1, float *u2, float *u3, int w, int h,
                             float l_t, float theta, float gamma) {
  double *rows = (double *)calloc((size_t)h, sizeof(double));
#pragma omp parallel for schedule(static)
  for (int y = 0; y < h; ++y) {
    double rsum = 0.0;
    for (int x = 0; x < w; ++x) {
      const size_t i = IDX(x, y, w);
      const float I1wxv = I1wx[i], I1wyv = I1wy[i], gradv = grad[i];
      const float u1o = u1[i], u2o = u2[i];
      const float u3o = gamma != 0.0f ? u3[i] : 0.0f;
      /* CPU association: rho_c + (I1wx*u1 + I1wy*u2) [+ gamma*u3] */
      float rho = rho_c[i] + (I1wxv * u1o + I1wyv * u2o);
      if (gamma != 0.0f) rho = rho + gamma * u3o;
      float d1 = 0.0f, d2 = 0.0f, d3 = 0.0f;
      if (rho < -l_t * gradv) {
        d1 = l_t * I1wxv;
        d2 = l_t * I1wyv;
        if (gamma != 0.0f) d3 = l_t * gamma;
      } else if (rho > l_t * gradv) {
        d1 = -l_t * I1wxv;
        d2 = -l_t * I1wyv;
        if (gamma != 0.0f) d3 = -l_t * gamma;
      } else if (gradv > FLT_EPSILON) {
        const float fi = -rho / gradv;
        d1 = fi * I1wxv;
        d2 = fi * I1wyv;
        if (gamma != 0.0f) d3 = fi * gamma;
      }
      const float v1 = u1o + d1, v2 = u2o + d2, v3 = u3o + d3;
      const float u1n = v1 + theta * divergence(p11, p12, y, x, w);
      const float u2n = v2 + theta * divergence(p21, p22, y, x, w);
      u1[i] = u1n;
      u2[i] = u2n;
      if (gamma != 0.0f) u3[i] = v3 + theta * divergence(p31, p32, y, x, w);
      const float n1 = (u1o - u1n) * (u1o - u1n);
      const float n2 = (u2o - u2n) * (u2o - u2n);
      rsum += (double)(n1 + n2);
    }
    rows[y] = rsum;
  }
  double total = 0.0;
  for (int y = 0; y < h; ++y) total += rows[y];
  free(rows);
  return total;
}

static inline float hypot_cpu(float a, float b) {
  return (float)sqrt((double)a * a + (double)b * b);
}

static void estimate_dual_cpu(const float *u1, const float *u2, const float *u3, float *p11,
                              float *p12, float *p21, float *p22, float *p31, float *p32, int w,
                              int h, float taut, float gamma) {
#pragma omp parallel for schedule(static)
  for (int y = 0; y < h; ++y) {
    const int yn = imin(y + 1, h - 1);
    for (int x = 0; x < w; ++x) {
      const int xn = imin(x + 1, w - 1);
      const size_t i = IDX(x, y, w);
      const float u1x = u1[IDX(xn, y, w)] - u1[i];
      const float u1y = u1[IDX(x, yn, w)] - u1[i];
      const float u2x = u2[IDX(xn, y, w)] - u2[i];
      const float u2y = u2[IDX(x, yn, w)] - u2[i];
      const float ng1 = 1.0f + taut * hypot_cpu(u1x, u1y);
      const float ng2 = 1.0f + taut * hypot_cpu(u2x, u2y);
      p11[i] = (p11[i] + taut * u1x) / ng1;
      p12[i] = (p12[i] + taut * u1y) / ng1;
      p21[i] = (p21[i] + taut * u2x) / ng2;
      p22[i] = (p22[i] + taut * u2y) / ng2;
      if (gamma != 0.0f) {
        const float u3x = u3[IDX(xn, y, w)] - u3[i];
        const float u3y = u3[IDX(x, yn, w)] - u3[i];
        const float ng3 = 1.0f + taut * hypot_cpu(u3x, u3y);
        p31[i] = (p31[i] + taut * u3x) / ng3;
        p32[i] = (p32[i] + taut * u3y) / ng3;
      }
    }
  }
}

/* resize(): exact 2x downscale of INTER_LINEAR takes the INTER_AREA fast path */
static int area_fast_of(double scale_x, double scale_y) {
  const int ix = (int)lrint(scale_x), iy = (int)lrint(scale_y);
  return fabs(scale_x - ix) < DBL_EPSILON && fabs(scale_y - iy) < DBL_EPSILON && ix == 2 &&
         iy == 2;
}

int orc_tvl1_calc_dualtvl1(const tvl1_params *prm, const uint8_t *I0, size_t pitch0,
                           const uint8_t *I1, size_t pitch1, int w, int h, float *u, float *v,
                           size_t flow_pitch, tvl1_stats *stats) {
  return orc_tvl1_calc_dualtvl1_in(prm, I0, pitch0, I1, pitch1, 0, w, h, u, v, flow_pitch, stats);
}

int orc_tvl1_calc_dualtvl1_in(const tvl1_params *prm, const void *I0, size_t pitch0,
                              const void *I1, size_t pitch1, int f32, int w, int h, float *u,
                              float *v, size_t flow_pitch, tvl1_stats *stats) {
  if (prm->nscales <= 0 || prm->warps < 0 || prm->inner_iterations < 0 ||
      prm->outer_iterations < 0)
    return TVL1_EINVAL;
  if (w <= 0 || h <= 0) return TVL1_ESIZE;
  if (pitch0 < (size_t)w || pitch1 < (size_t)w || flow_pitch < sizeof(float) * (size_t)w)
    return TVL1_EINVAL;
  if (prm->median_filtering > 1 && prm->median_filtering != 3 && prm->median_filtering != 5)
    return TVL1_EINVAL;

  const int nsc = prm->nscales < TVL1_MAX_LEVELS ? prm->nscales : TVL1_MAX_LEVELS;
  int ws[TVL1_MAX_LEVELS], hs[TVL1_MAX_LEVELS];
  const int L = orc_pyramid_sizes(w, h, nsc, prm->scale_step, ws, hs);
  const int use_gamma = prm->gamma != 0.0;
  const size_t N0 = (size_t)w * h;

  float *I0s[TVL1_MAX_LEVELS], *I1s[TVL1_MAX_LEVELS], *U1[TVL1_MAX_LEVELS],
      *U2[TVL1_MAX_LEVELS], *U3[TVL1_MAX_LEVELS];
  for (int s = 0; s < L; ++s) {
    const size_t N = (size_t)ws[s] * hs[s];
    I0s[s] = (float *)malloc(N * sizeof(float));
    I1s[s] = (float *)malloc(N * sizeof(float));
    U1[s] = (float *)calloc(N, sizeof(float));
    U2[s] = (float *)calloc(N, sizeof(float));
    U3[s] = use_gamma ? (float *)calloc(N, sizeof(float)) : NULL;
  }
  float *pl[12];
  for (int k = 0; k < 12; ++k) pl[k] = (float *)malloc(N0 * sizeof(float));
  float *I1x = pl[0], *I1y = pl[1], *I1wx = pl[2], *I1wy = pl[3], *grad = pl[4],
        *rho_c = pl[5], *p11 = pl[6], *p12 = pl[7], *p21 = pl[8], *p22 = pl[9],
        *p31 = pl[10], *p32 = pl[11], *tmp = NULL;
  if (prm->median_filtering > 1) tmp = (float *)malloc(N0 * sizeof(float));

  int64_t level_iters[TVL1_MAX_LEVELS];
  memset(level_iters, 0, sizeof(level_iters));

  /* calc(): convertTo(CV_32F), then resize(.., Size(), scaleStep, scaleStep) per level */
  orc_convert_in(I0, pitch0, f32, w, h, I0s[0]);
  orc_convert_in(I1, pitch1, f32, w, h, I1s[0]);
  const double dscale = 1. / prm->scale_step;
  const int afast = area_fast_of(dscale, dscale);
  for (int s = 1; s < L; ++s) {
    orc_resize_hp(I0s[s - 1], ws[s - 1], hs[s - 1], I0s[s], ws[s], hs[s], dscale, dscale, afast);
    orc_resize_hp(I1s[s - 1], ws[s - 1], hs[s - 1], I1s[s], ws[s], hs[s], dscale, dscale, afast);
  }

  const float l_t = (float)(prm->lambda * prm->theta);
  const float taut = (float)(prm->tau / prm->theta);
  const float theta_f = (float)prm->theta;
  const float gamma_f = (float)prm->gamma;
  const float upmul = (float)(1.0 / prm->scale_step);

  for (int s = L - 1; s >= 0; --s) {
    const int lw = ws[s], lh = hs[s];
    const size_t N = (size_t)lw * lh;
    const float scaledEps = (float)(prm->epsilon * prm->epsilon * (double)(lw * lh));
    orc_centered_gradient(I1s[s], lw, lh, I1x, I1y);
    for (int k = 6; k < 12; ++k) memset(pl[k], 0, N * sizeof(float));
    for (int wp = 0; wp < prm->warps; ++wp) {
      orc_remap_cubic(I0s[s], I1s[s], I1x, I1y, U1[s], U2[s], lw, lh, I1wx, I1wy, grad, rho_c);
      float error = FLT_MAX;
      int n = 0;
      for (int no = 0; error > scaledEps && no < prm->outer_iterations; ++no) {
        if (tmp) {
          orc_median(U1[s], lw, lh, prm->median_filtering, tmp);
          memcpy(U1[s], tmp, N * sizeof(float));
          orc_median(U2[s], lw, lh, prm->median_filtering, tmp);
          memcpy(U2[s], tmp, N * sizeof(float));
        }
        for (int ni = 0; error > scaledEps && ni < prm->inner_iterations; ++ni) {
          error = (float)estimate_u_cpu(I1wx, I1wy, grad, rho_c, p11, p12, p21, p22, p31, p32,
                                        U1[s], U2[s], U3[s], lw, lh, l_t, theta_f, gamma_f);
          estimate_dual_cpu(U1[s], U2[s], U3[s], p11, p12, p21, p22, p31, p32, lw, lh, taut,
                            gamma_f);
          ++n;
        }
      }
      level_iters[s] += n;
      if (stats && stats->warp_iterations &&
          s * prm->warps + wp < stats->warp_iterations_capacity)
        stats->warp_iterations[s * prm->warps + wp] = n;
    }
    if (s == 0) break;
    /* resize(u, .., I0s[s-1].size()) then multiply by 1/scaleStep (u3 not scaled) */
    const int dw = ws[s - 1], dh = hs[s - 1];
    const double sxu = 1. / ((double)dw / lw), syu = 1. / ((double)dh / lh);
    const int uf = area_fast_of(sxu, syu);
    orc_resize_hp(U1[s], lw, lh, U1[s - 1], dw, dh, sxu, syu, uf);
    orc_resize_hp(U2[s], lw, lh, U2[s - 1], dw, dh, sxu, syu, uf);
    if (use_gamma) orc_resize_hp(U3[s], lw, lh, U3[s - 1], dw, dh, sxu, syu, uf);
    for (size_t i = 0; i < (size_t)dw * dh; ++i) {
      U1[s - 1][i] = U1[s - 1][i] * upmul;
      U2[s - 1][i] = U2[s - 1][i] * upmul;
    }
  }

  for (int y = 0; y < h; ++y) {
    memcpy((char *)u + (size_t)y * flow_pitch, U1[0] + (size_t)y * w, sizeof(float) * w);
    memcpy((char *)v + (size_t)y * flow_pitch, U2[0] + (size_t)y * w, sizeof(float) * w);
  }
  if (stats) {
    stats->levels = L;
    int64_t tot = 0;
    for (int s = 0; s < TVL1_MAX_LEVELS; ++s) {
      stats->level_width[s] = s < L ? ws[s] : 0;
      stats->level_height[s] = s < L ? hs[s] : 0;
      stats->level_iterations[s] = s < L ? level_iters[s] : 0;
      tot += s < L ? level_iters[s] : 0;
    }
    stats->iterations_total = tot;
    stats->checks_total = tot;   /* every inner iteration evaluates the residual */
    stats->algorithmic_bytes = orc_survey_bytes(L, ws, hs, prm->warps, level_iters);
  }
  for (int s = 0; s < L; ++s) {
    free(I0s[s]);
    free(I1s[s]);
    free(U1[s]);
    free(U2[s]);
    free(U3[s]);
  }
  for (int k = 0; k < 12; ++k) free(pl[k]);
  free(tmp);
  return TVL1_OK;
}
