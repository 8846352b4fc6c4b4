/*
 * tvl1_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's solver path: the
 * OpenCV 3.4.1 `cv::cuda::OpticalFlowDual_TVL1` called at
 * /root/reference/src/optflow.cpp:516-520 plus the solve_wrapper post-ops
 * (optflow.cpp:445-473).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library; the product path never does.
 *
 * PARITY UNPINNED: the reference ships no tests, fixtures or golden vectors and
 * OpenCV 3.4.1 (a third-party dependency pinned at singularity/optflow.def:22-23)
 * is absent from this image, so this restatement is pinned only by the
 * known-answer tests in tests/ and by fixtures it generated itself.
 */
#ifndef TVL1_ORACLE_H
#define TVL1_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/tvl1.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- stage functions (packed row-major buffers, pitch == width) ---- */

/* K1 GpuMat::convertTo(CV_32F, 1.0) */
void orc_convert_u8(const uint8_t *src, size_t pitch, int w, int h, float *dst);

/* K2/K9 cuda::resize INTER_LINEAR, corner-aligned (fx, fy = src/dst step as float) */
void orc_resize_linear(const float *src, int sw, int sh, float *dst, int dw, int dh,
                       float fx, float fy);

/* pyramid sizes exactly as calcImpl builds them; returns effective level count */
int orc_pyramid_sizes(int w, int h, int nscales, double scale_step, int *ws, int *hs);

/* K3 centeredGradient */
void orc_centered_gradient(const float *I, int w, int h, float *Ix, float *Iy);

/* K5 warpBackward (I1w is not produced: nothing downstream reads it) */
void orc_warp_backward(const float *I0, const float *I1, const float *I1x, const float *I1y,
                       const float *u1, const float *u2, int w, int h,
                       float *I1wx, float *I1wy, float *grad, float *rho_c);

/* K6 estimateU (in place on u1,u2[,u3]); returns sum(diff) in double when calc_error */
double orc_estimate_u(const float *I1wx, const float *I1wy, const float *grad,
                      const float *rho_c, const float *p11, const float *p12,
                      const float *p21, const float *p22, const float *p31,
                      const float *p32, float *u1, float *u2, float *u3, int w, int h,
                      float l_t, float theta, float gamma, int calc_error);

/* K8 estimateDualVariables (in place on p) */
void orc_estimate_dual(const float *u1, const float *u2, const float *u3, float *p11,
                       float *p12, float *p21, float *p22, float *p31, float *p32, int w,
                       int h, float taut, float gamma);

/* build-only median filter (cv::medianBlur semantics, BORDER_REPLICATE, k = 3 or 5) */
void orc_median(const float *src, int w, int h, int k, float *dst);

/* ---- profile 1: OpenCV's CPU cv::DualTVL1OpticalFlow schedule ---- */

/* cv::resize INTER_LINEAR on CV_32F (half-pixel centres, separable float weights);
 * scale = source px per destination px (double, as resize derives it); area_fast =
 * the exact-2x INTER_AREA fast path resize switches to */
void orc_resize_hp(const float *src, int sw, int sh, float *dst, int dw, int dh,
                   double scale_x, double scale_y, int area_fast);

/* remap(I1 / I1x / I1y, x + u1, y + u2, INTER_CUBIC, BORDER_CONSTANT 0) + calcGradRho */
void orc_remap_cubic(const float *I0, const float *I1, const float *I1x, const float *I1y,
                     const float *u1, const float *u2, int w, int h, float *I1wx,
                     float *I1wy, float *grad, float *rho_c);

int orc_tvl1_calc_dualtvl1(const tvl1_params *params, const uint8_t *I0, size_t pitch0,
                           const uint8_t *I1, size_t pitch1, int w, int h, float *u, float *v,
                           size_t flow_pitch, tvl1_stats *stats);
/* the same on u8 (pitch in px, f32 = 0) or f32 inputs (pitch in bytes, f32 = 1) */
int orc_tvl1_calc_dualtvl1_in(const tvl1_params *params, const void *I0, size_t pitch0,
                              const void *I1, size_t pitch1, int f32, int w, int h, float *u,
                              float *v, size_t flow_pitch, tvl1_stats *stats);
/* [A.1] level-0 frames: float(u8), or f32 * 255 + 0 (convertTo(CV_32F, 255)) */
void orc_convert_in(const void *src, size_t pitch, int f32, int w, int h, float *dst);

/* ---- whole solve: same contract as tvl1_calc_host (include/tvl1.h) ---- */
int orc_tvl1_calc(const tvl1_params *params, const uint8_t *I0, size_t pitch0,
                  const uint8_t *I1, size_t pitch1, int w, int h, float *u, float *v,
                  size_t flow_pitch, tvl1_stats *stats);
/* ... and tvl1_calc_f32's contract (f32 frames, pitches in bytes) */
int orc_tvl1_calc_f32(const tvl1_params *params, const float *I0, size_t pitch0,
                      const float *I1, size_t pitch1, int w, int h, float *u, float *v,
                      size_t flow_pitch, tvl1_stats *stats);

/* solve_wrapper post-ops (optflow.cpp:445-473) on host buffers */
void orc_postprocess(float *u, float *v, size_t flow_pitch, const uint8_t *I1, size_t pitch1,
                     int w, int h, int mode);

/* ---- feature pre-alignment: this build's pipeline restated
 * (tvl1_oracle_align.c; the contracts of tvl1_orb_detect, tvl1_match_knn2,
 * tvl1_find_alignment, tvl1_warp_affine_u8 and tvl1_postprocess_affine in include/tvl1.h) */
/* keypoints (5 floats each: x, y, octave, 0 (angle not restated), response) and 32-byte
 * descriptors of up to cap keypoints; returns how many were found (-1 on no memory) */
int orc_orb_detect(const uint8_t *img, size_t pitch, int w, int h, const tvl1_align_params *ap,
                   float *kp, uint8_t *desc, int cap);
void orc_match_knn2(const uint8_t *query, int nq, const uint8_t *train, int nt, int32_t *idx,
                    int32_t *dist);
/* 1 when a model was found; src / dst: n (x, y) pairs in double */
int orc_find_homography(const double *src_xy, const double *dst_xy, int n, int method,
                        double thresh, double H[9], uint8_t *mask);
int orc_find_alignment(const uint8_t *frame1, size_t pitch1, int w1, int h1,
                       const uint8_t *frame0, size_t pitch0, int w0, int h0,
                       const tvl1_align_params *ap, float affine[6], int *n_good,
                       int *outcome);
void orc_warp_affine_u8(const uint8_t *src, size_t sp, int sw, int sh, uint8_t *dst, size_t dp,
                        int dw, int dh, const float affine[6]);
void orc_postprocess_affine(float *u, float *v, size_t flow_pitch, const uint8_t *I1,
                            size_t pitch1, int w, int h, int flow_output, const float affine[6]);

/* number of OpenMP threads the oracle uses (1 when built without OpenMP) */
/* parity report only: residual accumulation order and a per-check trace of
 * error / scaledEps (records of 4 doubles: level, warp, n, ratio) */
void orc_set_residual_mode(int mode);
void orc_set_check_trace(double *buf, int cap_records);
int orc_check_trace_count(void);
int orc_num_threads(void);
void orc_set_num_threads(int n);

#ifdef __cplusplus
}
#endif
#endif
