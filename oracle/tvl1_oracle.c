/*
 * tvl1_oracle.c — TEST INFRASTRUCTURE ONLY (see tvl1_oracle.h).
 *
 * A plain-C, float32 restatement of the solver the reference calls at
 * /root/reference/src/optflow.cpp:516-520:
 *     cv::cuda::OpticalFlowDual_TVL1::create(tau, lambda, theta, nscales, warps,
 *                                            epsilon, iterations, scaleStep, gamma)
 *         ->calc(frame0, frame1, output);
 * OpenCV 3.4.1 + opencv_contrib 3.4.1 (pinned at singularity/optflow.def:22-23,
 * built with CUDA_FAST_MATH, :33-34) is NOT vendored and NOT present in this
 * image.  Its published algorithm is restated here from SURVEY.md Appendix A
 * (upstream files cudaoptflow/src/tvl1flow.cpp, cudaoptflow/src/cuda/tvl1flow.cu,
 * cudawarping/src/resize.cpp, cudawarping/src/cuda/resize.cu).  Section tags
 * [A.n] below refer to that appendix.
 *
 * PARITY UNPINNED: the reference has no tests, fixtures or golden outputs
 * (SURVEY 4, 8c); this file is checked by known-answer tests and pins the
 * committed fixtures under tests/golden/ that it generated.
 *
 * Numerics: IEEE float32, no FMA contraction (built with -ffp-contract=off),
 * expression order as in the upstream kernels, residual sums in double.  The
 * reference build used fast math (approximate division/hypot, FMA): its own
 * outputs differ from any IEEE restatement at the ulp level (A.7).
 *
 * fma mode (tvl1_params.fast_math = 2): the same algorithm with every a*b + c that nvcc's
 * default -fmad=true contracts written as one fmaf (IEEE division and sqrt kept), so the
 * distance between the two arithmetics -- and the tolerance parity must hold to -- can be
 * measured.  The rule, NVPTX's DAG combine with aggressive FMA fusion: an
 * add or subtract with a multiply operand becomes one fma, the LEFT operand's product when
 * both are products (a*b + c*d -> fma(a, b, c*d)); a - b*c -> fma(-b, c, a).  Each site is
 * marked FMA below.  fast_math = 1 (approximate division / sqrt) has no exact C form: the
 * oracle solves it in IEEE and the engine is held to the tolerance bar.
 */
#include "tvl1_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define IDX(x, y, w) ((size_t)(y) * (size_t)(w) + (size_t)(x))

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }

int orc_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

void orc_set_num_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}

/* [A.1] I0f = float(I0): GpuMat::convertTo(CV_32F, 1.0) for CV_8U inputs. */
void orc_convert_u8(const uint8_t *src, size_t pitch, int w, int h, float *dst) {
#pragma omp parallel for schedule(static)
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) dst[IDX(x, y, w)] = (float)src[(size_t)y * pitch + x];
}

/* [A.1] for CV_32FC1 inputs: convertTo(CV_32F, 255.0) = src * 255 + 0 (pitch in bytes). */
void orc_convert_f32(const float *src, size_t pitch, int w, int h, float *dst) {
#pragma omp parallel for schedule(static)
  for (int y = 0; y < h; ++y) {
    const float *row = (const float *)((const char *)src + (size_t)y * pitch);
    for (int x = 0; x < w; ++x) dst[IDX(x, y, w)] = row[x] * 255.0f + 0.0f;
  }
}

/* the level-0 frames of a solve from u8 (pitch in px) or f32 (pitch in bytes) inputs */
void orc_convert_in(const void *src, size_t pitch, int f32, int w, int h, float *dst) {
  if (f32)
    orc_convert_f32((const float *)src, pitch, w, h, dst);
  else
    orc_convert_u8((const uint8_t *)src, pitch, w, h, dst);
}

/* [A.2] cuda::resize INTER_LINEAR (resize.cu resize_linear / LinearFilter):
 * corner-aligned source coordinate src = dst * f, taps floor/+1, the +1 tap
 * clamped to the last column/row (BrdReplicate / texture clamp). */
static void resize_linear(const float *src, int sw, int sh, float *dst, int dw, int dh,
                          float fx, float fy, int fma_mode) {
  if (sw == dw && sh == dh) { /* resize.cpp: dsize == src.size() -> copyTo */
    memcpy(dst, src, sizeof(float) * (size_t)sw * sh);
    return;
  }
#pragma omp parallel for schedule(static)
  for (int dy = 0; dy < dh; ++dy) {
    const float dyf = (float)dy;
    const float src_y = dyf * fy;
    const int y1 = (int)floorf(src_y);
    const int y2 = y1 + 1;
    const int y2r = imin(y2, sh - 1);
    for (int dx = 0; dx < dw; ++dx) {
      const float dxf = (float)dx;
      const float src_x = dxf * fx;
      const int x1 = (int)floorf(src_x);
      const int x2 = x1 + 1;
      const int x2r = imin(x2, sw - 1);
      const float t00 = src[IDX(x1, y1, sw)], t01 = src[IDX(x2r, y1, sw)];
      const float t10 = src[IDX(x1, y2r, sw)], t11 = src[IDX(x2r, y2r, sw)];
      float out = 0.0f;
      if (fma_mode) {
        /* FMA: x2 - dst_x*fx -> fma(-dst_x, fx, x2), dst_x*fx - x1 -> fma(dst_x, fx, -x1)
         * (the floor takes the rounded product); out + src*w -> fma(src, w, out) */
        const float ax = fmaf(-dxf, fx, (float)x2), bx = fmaf(dxf, fx, -(float)x1);
        const float ay = fmaf(-dyf, fy, (float)y2), by = fmaf(dyf, fy, -(float)y1);
        out = fmaf(t00, ax * ay, out);
        out = fmaf(t01, bx * ay, out);
        out = fmaf(t10, ax * by, out);
        out = fmaf(t11, bx * by, out);
      } else {
        out = out + t00 * (((float)x2 - src_x) * ((float)y2 - src_y));
        out = out + t01 * ((src_x - (float)x1) * ((float)y2 - src_y));
        out = out + t10 * (((float)x2 - src_x) * (src_y - (float)y1));
        out = out + t11 * ((src_x - (float)x1) * (src_y - (float)y1));
      }
      dst[IDX(dx, dy, dw)] = out;
    }
  }
}

void orc_resize_linear(const float *src, int sw, int sh, float *dst, int dw, int dh,
                       float fx, float fy) {
  resize_linear(src, sw, sh, dst, dw, dh, fx, fy, 0);
}

/* [A.2] dst size = saturate_cast<int>(cols * scaleStep) (cvRound, half-to-even);
 * a level with a side < 16 ends the pyramid and is discarded (nscales_ = s). */
int orc_pyramid_sizes(int w, int h, int nscales, double scale_step, int *ws, int *hs) {
  int L = nscales;
  ws[0] = w;
  hs[0] = h;
  for (int s = 1; s < nscales; ++s) {
    const int nw = (int)lrint((double)ws[s - 1] * scale_step);
    const int nh = (int)lrint((double)hs[s - 1] * scale_step);
    if (nw < 16 || nh < 16) {
      L = s;
      break;
    }
    ws[s] = nw;
    hs[s] = nh;
  }
  return L;
}

/* [A.3] centeredGradient: 0.5f * (I[min(x+1,W-1)] - I[max(x-1,0)]), same in y. */
void orc_centered_gradient(const float *I, int w, int h, float *Ix, float *Iy) {
#pragma omp parallel for schedule(static)
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      Ix[IDX(x, y, w)] = 0.5f * (I[IDX(imin(x + 1, w - 1), y, w)] - I[IDX(imax(x - 1, 0), y, w)]);
      Iy[IDX(x, y, w)] = 0.5f * (I[IDX(x, imin(y + 1, h - 1), w)] - I[IDX(x, imax(y - 1, 0), w)]);
    }
}

/* [A.3] Keys cubic kernel, a = -0.5 (tvl1flow.cu `cubic`). */
static inline float cubic(float x, int fma_mode) {
  x = fabsf(x);
  if (fma_mode) { /* FMA: x*x*t + 1 -> fma(x*x, t, 1), t = 1.5x - 2.5 -> fma(1.5, x, -2.5) */
    if (x <= 1.0f) return fmaf(x * x, fmaf(1.5f, x, -2.5f), 1.0f);
    if (x < 2.0f) return fmaf(x, fmaf(x, fmaf(-0.5f, x, 2.5f), -4.0f), 2.0f);
    return 0.0f;
  }
  if (x <= 1.0f) return x * x * (1.5f * x - 2.5f) + 1.0f;
  if (x < 2.0f) return x * (x * (-0.5f * x + 2.5f) - 4.0f) + 2.0f;
  return 0.0f;
}

/* [A.3] warpBackward: 4x4(5x5) cubic gather of I1, I1x, I1y at (x+u1, y+u2) with
 * texture clamp, weight-normalised; grad = I1wx^2 + I1wy^2;
 * rho_c = I1w - I1wx*u1 - I1wy*u2 - I0. */
static void warp_backward(const float *I0, const float *I1, const float *I1x, const float *I1y,
                          const float *u1, const float *u2, int w, int h, float *I1wx,
                          float *I1wy, float *grad, float *rho_c, int fma_mode) {
#pragma omp parallel for schedule(static)
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const size_t i = IDX(x, y, w);
      const float u1v = u1[i];
      const float u2v = u2[i];
      const float wx = (float)x + u1v;
      const float wy = (float)y + u2v;
      const int xmin = (int)ceilf(wx - 2.0f);
      const int xmax = (int)floorf(wx + 2.0f);
      const int ymin = (int)ceilf(wy - 2.0f);
      const int ymax = (int)floorf(wy + 2.0f);
      float sum = 0.0f, sumx = 0.0f, sumy = 0.0f, wsum = 0.0f;
      for (int cy = ymin; cy <= ymax; ++cy) {
        const int ry = imin(imax(cy, 0), h - 1);
        for (int cx = xmin; cx <= xmax; ++cx) {
          const int rx = imin(imax(cx, 0), w - 1);
          const float wgt = cubic(wx - (float)cx, fma_mode) * cubic(wy - (float)cy, fma_mode);
          const size_t j = IDX(rx, ry, w);
          if (fma_mode) { /* FMA: sum + w*I -> fma(w, I, sum) */
            sum = fmaf(wgt, I1[j], sum);
            sumx = fmaf(wgt, I1x[j], sumx);
            sumy = fmaf(wgt, I1y[j], sumy);
          } else {
            sum = sum + wgt * I1[j];
            sumx = sumx + wgt * I1x[j];
            sumy = sumy + wgt * I1y[j];
          }
          wsum = wsum + wgt;
        }
      }
      const float coeff = 1.0f / wsum;
      const float I1wv = sum * coeff;
      const float I1wxv = sumx * coeff;
      const float I1wyv = sumy * coeff;
      I1wx[i] = I1wxv;
      I1wy[i] = I1wyv;
      const float Ix2 = I1wxv * I1wxv;
      const float Iy2 = I1wyv * I1wyv;
      if (fma_mode) { /* FMA: Ix2 + Iy2 -> fma(I1wx, I1wx, Iy2); the two products of rho_c
                       * fused into the running difference */
        grad[i] = fmaf(I1wxv, I1wxv, Iy2);
        rho_c[i] = fmaf(-I1wyv, u2v, fmaf(-I1wxv, u1v, I1wv)) - I0[i];
      } else {
        grad[i] = Ix2 + Iy2;
        rho_c[i] = I1wv - I1wxv * u1v - I1wyv * u2v - I0[i];
      }
    }
}

void orc_warp_backward(const float *I0, const float *I1, const float *I1x, const float *I1y,
                       const float *u1, const float *u2, int w, int h, float *I1wx,
                       float *I1wy, float *grad, float *rho_c) {
  warp_backward(I0, I1, I1x, I1y, u1, u2, w, h, I1wx, I1wy, grad, rho_c, 0);
}

/* [A.3] backward-difference divergence with OpenCV's special row/column 0 forms
 * (the x==0, y>0 form associates differently from the interior form). */
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

/* Parity report only: how the residual is accumulated,
 * and a trace of every check's error / scaledEps.  OpenCV 3.4.1's cuda::sum of the CV_32F
 * diff buffer (procOneScale, behind /root/reference/src/optflow.cpp:518-519) reduces in an
 * order this restatement cannot know [OCV], so the report measures how far each stopping
 * decision sits from its threshold and reruns the schedule under a deliberately different
 * accumulation.
 *   mode 0 (default, the engine's): each row summed left to right in double, rows in order;
 *   mode 1: each row summed left to right in float, the row sums added in float from the
 *           last row to the first -- a lossy, differently ordered accumulation.
 * Process-global, not thread-safe: test infrastructure. */
static int g_resid_mode = 0;
static double *g_trace = NULL;
static int g_trace_cap = 0, g_trace_n = 0;

void orc_set_residual_mode(int mode) { g_resid_mode = mode; }

/* records of 4 doubles: level, warp, n, error / scaledEps; NULL turns the trace off */
void orc_set_check_trace(double *buf, int cap_records) {
  g_trace = buf;
  g_trace_cap = buf ? cap_records : 0;
  g_trace_n = 0;
}

int orc_check_trace_count(void) { return g_trace_n; }

static void trace_check(int level, int warp, int n, double ratio) {
  if (g_trace && g_trace_n < g_trace_cap) {
    double *r = g_trace + 4 * (size_t)g_trace_n;
    r[0] = level, r[1] = warp, r[2] = n, r[3] = ratio;
  }
  if (g_trace) ++g_trace_n;
}

/* [A.3] estimateU: TH thresholding + u = v + theta * div(p). */
static double estimate_u(const float *I1wx, const float *I1wy, const float *grad,
                         const float *rho_c, const float *p11, const float *p12,
                         const float *p21, const float *p22, const float *p31,
                         const float *p32, float *u1, float *u2, float *u3, int w, int h,
                         float l_t, float theta, float gamma, int calc_error, int fma_mode) {
  double *rows = calc_error ? (double *)calloc((size_t)h, sizeof(double)) : NULL;
  const int fmode = calc_error && g_resid_mode == 1;
  float *frows = fmode ? (float *)calloc((size_t)h, sizeof(float)) : NULL;
#pragma omp parallel for schedule(static)
  for (int y = 0; y < h; ++y) {
    double rsum = 0.0;
    float fsum = 0.0f;
    for (int x = 0; x < w; ++x) {
      const size_t i = IDX(x, y, w);
      const float I1wxv = I1wx[i];
      const float I1wyv = I1wy[i];
      const float gradv = grad[i];
      const float u1o = u1[i];
      const float u2o = u2[i];
      const float u3o = gamma != 0.0f ? u3[i] : 0.0f;
      /* rho = rho_c + (I1wx*u1 + I1wy*u2 + gamma*u3) -- gamma*u3 inside the
       * parentheses (with gamma = 0 either association gives the same bits) */
      /* FMA: rho_c + fma(gamma, u3, fma(I1wx, u1, I1wy*u2)) (u3 = 0 when gamma = 0: the fma
       * still turns a -0 sum into +0) */
      const float rho = fma_mode ? rho_c[i] + fmaf(gamma, u3o, fmaf(I1wxv, u1o, I1wyv * u2o))
                                 : rho_c[i] + (I1wxv * u1o + I1wyv * u2o + gamma * u3o);
      float d1 = 0.0f, d2 = 0.0f, d3 = 0.0f;
      if (rho < -l_t * gradv) {
        d1 = l_t * I1wxv;
        d2 = l_t * I1wyv;
        if (gamma != 0.0f) d3 = l_t * gamma;       /* +-l_t*gamma */
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
      const float v1 = u1o + d1;
      const float v2 = u2o + d2;
      const float v3 = u3o + d3;
      const float div1 = divergence(p11, p12, y, x, w);
      const float div2 = divergence(p21, p22, y, x, w);
      const float div3 = gamma != 0.0f ? divergence(p31, p32, y, x, w) : 0.0f;
      /* FMA: v + theta*div -> fma(theta, div, v) */
      const float u1n = fma_mode ? fmaf(theta, div1, v1) : v1 + theta * div1;
      const float u2n = fma_mode ? fmaf(theta, div2, v2) : v2 + theta * div2;
      u1[i] = u1n;
      u2[i] = u2n;
      if (gamma != 0.0f) u3[i] = fma_mode ? fmaf(theta, div3, v3) : v3 + theta * div3;
      if (calc_error) {
        const float e1 = u1o - u1n, e2 = u2o - u2n;
        /* FMA: n1 + n2 -> fma(e1, e1, e2*e2) */
        const float term = fma_mode ? fmaf(e1, e1, e2 * e2) : e1 * e1 + e2 * e2;
        rsum += (double)term;
        if (fmode) fsum += term;
      }
    }
    if (rows) rows[y] = rsum;
    if (frows) frows[y] = fsum;
  }
  double total = 0.0;
  if (rows) {
    for (int y = 0; y < h; ++y) total += rows[y];
    free(rows);
  }
  if (frows) {
    float ft = 0.0f;
    for (int y = h - 1; y >= 0; --y) ft += frows[y];
    free(frows);
    total = (double)ft;
  }
  return total;
}

double orc_estimate_u(const float *I1wx, const float *I1wy, const float *grad,
                      const float *rho_c, const float *p11, const float *p12,
                      const float *p21, const float *p22, const float *p31,
                      const float *p32, float *u1, float *u2, float *u3, int w, int h,
                      float l_t, float theta, float gamma, int calc_error) {
  return estimate_u(I1wx, I1wy, grad, rho_c, p11, p12, p21, p22, p31, p32, u1, u2, u3, w, h,
                    l_t, theta, gamma, calc_error, 0);
}

/* hypotf restated as sqrt(a*a + b*b) (FMA: fma(a, a, b*b)); CUDA's library hypotf is not
 * available here */
static inline float hypot_f(float a, float b, int fma_mode) {
  return fma_mode ? sqrtf(fmaf(a, a, b * b)) : sqrtf(a * a + b * b);
}

/* one projection component: p' = (p + taut*du) / ng (FMA: fma(taut, du, p)) */
static inline float proj(float p, float du, float taut, float ng, int fma_mode) {
  return (fma_mode ? fmaf(taut, du, p) : p + taut * du) / ng;
}

/* [A.3] estimateDualVariables: forward differences (0 at last col/row),
 * ng = 1 + taut*|grad u| (FMA: fma(taut, g, 1)), p = (p + taut*grad u) / ng. */
static void estimate_dual(const float *u1, const float *u2, const float *u3, float *p11,
                          float *p12, float *p21, float *p22, float *p31, float *p32, int w,
                          int h, float taut, float gamma, int fma_mode) {
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
      const float g1 = hypot_f(u1x, u1y, fma_mode);
      const float g2 = hypot_f(u2x, u2y, fma_mode);
      const float ng1 = fma_mode ? fmaf(taut, g1, 1.0f) : 1.0f + taut * g1;
      const float ng2 = fma_mode ? fmaf(taut, g2, 1.0f) : 1.0f + taut * g2;
      p11[i] = proj(p11[i], u1x, taut, ng1, fma_mode);
      p12[i] = proj(p12[i], u1y, taut, ng1, fma_mode);
      p21[i] = proj(p21[i], u2x, taut, ng2, fma_mode);
      p22[i] = proj(p22[i], u2y, taut, ng2, fma_mode);
      if (gamma != 0.0f) {
        const float u3x = u3[IDX(xn, y, w)] - u3[i];
        const float u3y = u3[IDX(x, yn, w)] - u3[i];
        const float g3 = hypot_f(u3x, u3y, fma_mode);
        const float ng3 = fma_mode ? fmaf(taut, g3, 1.0f) : 1.0f + taut * g3;
        p31[i] = proj(p31[i], u3x, taut, ng3, fma_mode);
        p32[i] = proj(p32[i], u3y, taut, ng3, fma_mode);
      }
    }
  }
}

void orc_estimate_dual(const float *u1, const float *u2, const float *u3, float *p11,
                       float *p12, float *p21, float *p22, float *p31, float *p32, int w,
                       int h, float taut, float gamma) {
  estimate_dual(u1, u2, u3, p11, p12, p21, p22, p31, p32, w, h, taut, gamma, 0);
}

/* Build-only median filter: cv::medianBlur on CV_32F
 * (ksize 3 or 5), BORDER_REPLICATE.  Not in the reference's CUDA path. */
void orc_median(const float *src, int w, int h, int k, float *dst) {
  const int r = k / 2;
#pragma omp parallel for schedule(static)
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      float v[25];
      int n = 0;
      for (int dy = -r; dy <= r; ++dy)
        for (int dx = -r; dx <= r; ++dx)
          v[n++] = src[IDX(imin(imax(x + dx, 0), w - 1), imin(imax(y + dy, 0), h - 1), w)];
      for (int a = 1; a < n; ++a) { /* insertion sort: exact, order-independent result */
        const float t = v[a];
        int b = a - 1;
        while (b >= 0 && v[b] > t) {
          v[b + 1] = v[b];
          --b;
        }
        v[b + 1] = t;
      }
      dst[IDX(x, y, w)] = v[n / 2];
    }
}

/* solve_wrapper post-ops (optflow.cpp:411-473): map = flow + (x, y) when mode>=1,
 * mode 2 subtracts the grid again (features branch, identity alignment); then zero
 * both fields where I1 <= 1 (threshold THRESH_BINARY_INV + setTo). */
void orc_postprocess(float *u, float *v, size_t flow_pitch, const uint8_t *I1, size_t pitch1,
                     int w, int h, int mode) {
  for (int y = 0; y < h; ++y) {
    float *ur = (float *)((char *)u + (size_t)y * flow_pitch);
    float *vr = (float *)((char *)v + (size_t)y * flow_pitch);
    for (int x = 0; x < w; ++x) {
      if (mode >= 1) {
        ur[x] = ur[x] + (float)x;
        vr[x] = vr[x] + (float)y;
      }
      if (mode == 2) {
        ur[x] = ur[x] - (float)x;
        vr[x] = vr[x] - (float)y;
      }
      if (I1[(size_t)y * pitch1 + x] <= 1) {
        ur[x] = 0.0f;
        vr[x] = 0.0f;
      }
    }
  }
}

/* SURVEY 8(d) byte model, per level with executed iteration counts. */
double orc_survey_bytes(int L, const int *ws, const int *hs, int warps,
                           const int64_t *iters) {
  double B = 0.0;
  for (int l = 0; l < L; ++l) {
    const double N = (double)ws[l] * hs[l];
    B += N * (12.0 + 16.0 + 40.0 * warps + 64.0 * (double)iters[l]);
    if (l >= 1) B += N * 8.0;
    if (l < L - 1) B += N * 8.0;
  }
  const double N0 = (double)ws[0] * hs[0];
  B += N0 * (2.0 + 8.0) + N0 * 8.0;
  return B;
}

typedef struct {
  float *I0, *I1, *u1, *u2, *u3;
} level_bufs;

/* [A.1]-[A.4] calc / calcImpl / procOneScale; u8 inputs (pitch in px) or f32 (bytes). */
static int calc_in(const tvl1_params *prm, const void *I0, size_t pitch0, const void *I1,
                   size_t pitch1, int f32, int w, int h, float *u, float *v,
                   size_t flow_pitch, tvl1_stats *stats) {
  if (!prm || !I0 || !I1 || !u || !v) return TVL1_EINVAL;
  if (w <= 0 || h <= 0) return TVL1_ESIZE;
  const size_t in_bytes = f32 ? sizeof(float) * (size_t)w : (size_t)w;
  if (pitch0 < in_bytes || pitch1 < in_bytes || flow_pitch < sizeof(float) * (size_t)w)
    return TVL1_EINVAL;
  if (prm->profile == 1)
    return orc_tvl1_calc_dualtvl1_in(prm, I0, pitch0, I1, pitch1, f32, w, h, u, v, flow_pitch,
                                     stats);
  if (prm->profile != 0) return TVL1_EINVAL;
  if (prm->nscales <= 0 || prm->warps < 0 || prm->iterations < 0) return TVL1_EINVAL;
  if (prm->median_filtering > 1 && prm->median_filtering != 3 && prm->median_filtering != 5)
    return TVL1_EINVAL;

  const int nsc = prm->nscales < TVL1_MAX_LEVELS ? prm->nscales : TVL1_MAX_LEVELS;
  int ws[TVL1_MAX_LEVELS], hs[TVL1_MAX_LEVELS];
  const int L = orc_pyramid_sizes(w, h, nsc, prm->scale_step, ws, hs);
  const int use_gamma = prm->gamma != 0.0;
  /* fma mode for the gamma = 0 path with 0 <= tau/theta < inf (the engine's streaming
   * kernels; other parameter sets run IEEE there too) */
  const float taut_f = (float)(prm->tau / prm->theta);
  const int fma_mode = prm->fast_math == 2 && !use_gamma && taut_f >= 0.0f && taut_f <= FLT_MAX;

  level_bufs lv[TVL1_MAX_LEVELS];
  memset(lv, 0, sizeof(lv));
  const size_t N0 = (size_t)w * h;
  for (int s = 0; s < L; ++s) {
    const size_t N = (size_t)ws[s] * hs[s];
    lv[s].I0 = (float *)malloc(N * sizeof(float));
    lv[s].I1 = (float *)malloc(N * sizeof(float));
    lv[s].u1 = (float *)calloc(N, sizeof(float));
    lv[s].u2 = (float *)calloc(N, sizeof(float));
    lv[s].u3 = use_gamma ? (float *)calloc(N, sizeof(float)) : NULL;
  }
  float *I1x = (float *)malloc(N0 * sizeof(float));
  float *I1y = (float *)malloc(N0 * sizeof(float));
  float *I1wx = (float *)malloc(N0 * sizeof(float));
  float *I1wy = (float *)malloc(N0 * sizeof(float));
  float *grad = (float *)malloc(N0 * sizeof(float));
  float *rho_c = (float *)malloc(N0 * sizeof(float));
  float *p11 = (float *)malloc(N0 * sizeof(float));
  float *p12 = (float *)malloc(N0 * sizeof(float));
  float *p21 = (float *)malloc(N0 * sizeof(float));
  float *p22 = (float *)malloc(N0 * sizeof(float));
  float *p31 = use_gamma ? (float *)malloc(N0 * sizeof(float)) : NULL;
  float *p32 = use_gamma ? (float *)malloc(N0 * sizeof(float)) : NULL;
  float *tmp = prm->median_filtering > 1 ? (float *)malloc(N0 * sizeof(float)) : NULL;

  int64_t level_iters[TVL1_MAX_LEVELS];
  memset(level_iters, 0, sizeof(level_iters));
  int64_t checks = 0;

  /* [A.1] convertTo + [A.2] pyramid (fx passed to the kernel = float(1/scaleStep)) */
  orc_convert_in(I0, pitch0, f32, w, h, lv[0].I0);
  orc_convert_in(I1, pitch1, f32, w, h, lv[0].I1);
  const float fdown = (float)(1.0 / prm->scale_step);
  for (int s = 1; s < L; ++s) {
    resize_linear(lv[s - 1].I0, ws[s - 1], hs[s - 1], lv[s].I0, ws[s], hs[s], fdown, fdown, fma_mode);
    resize_linear(lv[s - 1].I1, ws[s - 1], hs[s - 1], lv[s].I1, ws[s], hs[s], fdown, fdown, fma_mode);
  }

  const float l_t = (float)(prm->lambda * prm->theta);
  const float taut = (float)(prm->tau / prm->theta);
  const float theta_f = (float)prm->theta;
  const float gamma_f = (float)prm->gamma;
  const float upmul = (float)(1.0 / prm->scale_step);

  for (int s = L - 1; s >= 0; --s) {
    const int lw = ws[s], lh = hs[s];
    const size_t N = (size_t)lw * lh;
    const double scaledEps = prm->epsilon * prm->epsilon * (double)N;
    orc_centered_gradient(lv[s].I1, lw, lh, I1x, I1y);
    memset(p11, 0, N * sizeof(float));
    memset(p12, 0, N * sizeof(float));
    memset(p21, 0, N * sizeof(float));
    memset(p22, 0, N * sizeof(float));
    if (use_gamma) {
      memset(p31, 0, N * sizeof(float));
      memset(p32, 0, N * sizeof(float));
    }
    for (int wp = 0; wp < prm->warps; ++wp) {
      if (tmp) {
        orc_median(lv[s].u1, lw, lh, prm->median_filtering, tmp);
        memcpy(lv[s].u1, tmp, N * sizeof(float));
        orc_median(lv[s].u2, lw, lh, prm->median_filtering, tmp);
        memcpy(lv[s].u2, tmp, N * sizeof(float));
      }
      warp_backward(lv[s].I0, lv[s].I1, I1x, I1y, lv[s].u1, lv[s].u2, lw, lh, I1wx, I1wy, grad,
                    rho_c, fma_mode);
      double error = DBL_MAX;
      double prevError = 0.0;
      int n;
      for (n = 0; error > scaledEps && n < prm->iterations; ++n) {
        const int calcError = (prm->epsilon > 0) && (n & 1) && (prevError < scaledEps);
        const double e = estimate_u(I1wx, I1wy, grad, rho_c, p11, p12, p21, p22, p31, p32,
                                    lv[s].u1, lv[s].u2, lv[s].u3, lw, lh, l_t, theta_f, gamma_f,
                                    calcError, fma_mode);
        if (calcError) {
          error = e;
          prevError = error;
          ++checks;
          trace_check(s, wp, n, error / scaledEps);
        } else {
          error = DBL_MAX;
          prevError -= scaledEps;
        }
        estimate_dual(lv[s].u1, lv[s].u2, lv[s].u3, p11, p12, p21, p22, p31, p32, lw, lh, taut,
                      gamma_f, fma_mode);
      }
      level_iters[s] += n;
      if (stats && stats->warp_iterations &&
          s * prm->warps + wp < stats->warp_iterations_capacity)
        stats->warp_iterations[s * prm->warps + wp] = n;
    }
    if (s == 0) break;
    /* [A.3] upsample: resize to the finer size (fx = float(1/(dW/sW))), then
     * multiply u1,u2 by float(1/scaleStep).  u3 is resized but not scaled. */
    const int dw = ws[s - 1], dh = hs[s - 1];
    const float fxu = (float)(1.0 / ((double)dw / lw));
    const float fyu = (float)(1.0 / ((double)dh / lh));
    resize_linear(lv[s].u1, lw, lh, lv[s - 1].u1, dw, dh, fxu, fyu, fma_mode);
    resize_linear(lv[s].u2, lw, lh, lv[s - 1].u2, dw, dh, fxu, fyu, fma_mode);
    if (use_gamma) resize_linear(lv[s].u3, lw, lh, lv[s - 1].u3, dw, dh, fxu, fyu, fma_mode);
    const size_t Nd = (size_t)dw * dh;
    for (size_t i = 0; i < Nd; ++i) {
      lv[s - 1].u1[i] = lv[s - 1].u1[i] * upmul;
      lv[s - 1].u2[i] = lv[s - 1].u2[i] * upmul;
    }
  }

  /* [A.4] flow = (u1[0], u2[0]) */
  for (int y = 0; y < h; ++y) {
    memcpy((char *)u + (size_t)y * flow_pitch, lv[0].u1 + (size_t)y * w, sizeof(float) * w);
    memcpy((char *)v + (size_t)y * flow_pitch, lv[0].u2 + (size_t)y * w, sizeof(float) * w);
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
    stats->checks_total = checks;
    stats->algorithmic_bytes = orc_survey_bytes(L, ws, hs, prm->warps, level_iters);
  }

  for (int s = 0; s < L; ++s) {
    free(lv[s].I0);
    free(lv[s].I1);
    free(lv[s].u1);
    free(lv[s].u2);
    free(lv[s].u3);
  }
  free(I1x); free(I1y); free(I1wx); free(I1wy); free(grad); free(rho_c);
  free(p11); free(p12); free(p21); free(p22); free(p31); free(p32); free(tmp);
  return TVL1_OK;
}

int orc_tvl1_calc(const tvl1_params *prm, const uint8_t *I0, size_t pitch0,
                  const uint8_t *I1, size_t pitch1, int w, int h, float *u, float *v,
                  size_t flow_pitch, tvl1_stats *stats) {
  return calc_in(prm, I0, pitch0, I1, pitch1, 0, w, h, u, v, flow_pitch, stats);
}

/* tvl1_calc_f32 on host buffers (pitches in bytes) */
int orc_tvl1_calc_f32(const tvl1_params *prm, const float *I0, size_t pitch0, const float *I1,
                      size_t pitch1, int w, int h, float *u, float *v, size_t flow_pitch,
                      tvl1_stats *stats) {
  return calc_in(prm, I0, pitch0, I1, pitch1, 1, w, h, u, v, flow_pitch, stats);
}
