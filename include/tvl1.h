/*
 * tvl1.h — C-ABI boundary of the MI355X-native dense TV-L1 optical-flow engine.
 *
 * This header is the drop-in replacement for the reference's single solver
 * call site:
 *
 *   reference  src/optflow.h:31 / src/optflow.cpp:516-520
 *     void TVL1_solve(cv::cuda::GpuMat& frame0, cv::cuda::GpuMat& frame1,
 *                     cv::cuda::GpuMat& output, const Json::Value& args);
 *   which does
 *     cv::cuda::OpticalFlowDual_TVL1::create(tau, lambda, theta, nscales, warps,
 *                                            epsilon, iterations, scaleStep, gamma)
 *       ->calc(frame0, frame1, output);                 (OpenCV 3.4.1, not vendored)
 *
 * Mapping (one row per reference concept):
 *   OpticalFlowDual_TVL1::create(...)       -> tvl1_create(&ctx, device, &params)
 *   solver->calc(I0, I1, flow) on GpuMats   -> tvl1_calc(ctx, dI0, pitch0, dI1, pitch1, w, h,
 *                                                       du, dv, flow_pitch, &stats, stream)
 *   cuda::split(flow) (optflow.cpp:404)     -> outputs are already planar (u, v)
 *   solver destruction                      -> tvl1_destroy(ctx)
 *   cv::Exception (CV_Assert)               -> tvl1_status return code + tvl1_last_error(ctx)
 *   post-ops optflow.cpp:445-473            -> tvl1_postprocess(...) (map grid add + I1<=1 mask)
 *   generate_TV_args defaults :500-514      -> tvl1_params_default(&params)
 *
 * Conventions
 *   - Plain pointers and sizes only; no HIP, torch or OpenCV types.  `stream` is a
 *     hipStream_t passed as void* (NULL = the default stream).
 *   - All pitches are in BYTES (OpenCV GpuMat::step convention).
 *   - Inputs are 8-bit unsigned grayscale (CV_8UC1, IMREAD_GRAYSCALE, optflow.cpp:106);
 *     outputs are planar float32 u (x displacement) and v (y displacement) such
 *     that I1(x+u, y+v) ~= I0(x, y)  (flow points from frame0=p to frame1=q).
 *   - Errors never throw across the ABI: every entry point returns tvl1_status.
 *   - A ctx is not thread-safe.  Distinct ctxs (one per device per host thread)
 *     are independent.  tvl1_calc is asynchronous w.r.t. the host only where the
 *     stats say so: the convergence test reads the residual on the host exactly
 *     where OpenCV does (a device->host read on "check" iterations), so the call
 *     returns after the solve has been fully enqueued; outputs are valid after a
 *     stream synchronize (tvl1_calc_host synchronizes for you).
 */
#ifndef FIBSEM_OPTFLOW_AMD_TVL1_H
#define FIBSEM_OPTFLOW_AMD_TVL1_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TVL1_ABI_VERSION 9
#define TVL1_MAX_LEVELS 32

typedef enum tvl1_status {
  TVL1_OK = 0,
  TVL1_EINVAL = 1, /* bad argument (null pointer, nscales <= 0, bad pitch ...)  */
  TVL1_ESIZE = 2,  /* size mismatch / image smaller than 1x1 / too large       */
  TVL1_EHIP = 3,   /* a HIP runtime call failed (message in tvl1_last_error)    */
  TVL1_ENOMEM = 4, /* device or host allocation failed                          */
  TVL1_ENODEV = 5  /* no usable gfx950 device / extension not built             */
} tvl1_status;

/* The nine cv::cuda::OpticalFlowDual_TVL1::create() arguments (optflow.cpp:518)
 * plus the two build-only additions listed in SURVEY Appendix B. */
typedef struct tvl1_params {
  double tau;          /* 0.25  optflow.cpp:503 */
  double lambda;       /* 0.05  optflow.cpp:504 */
  double theta;        /* 0.3   optflow.cpp:505 */
  int32_t nscales;     /* 10    optflow.cpp:506 */
  int32_t warps;       /* 5     optflow.cpp:507 */
  double epsilon;      /* 0.01  optflow.cpp:508 */
  int32_t iterations;  /* 300   optflow.cpp:509 */
  double scale_step;   /* 0.8   optflow.cpp:510 */
  double gamma;        /* 0.0   optflow.cpp:511 */
  int32_t use_initial_flow; /* read at optflow.cpp:512 but NOT passed to create() (:518): ignored, as in the reference */
  int32_t median_filtering; /* build-only: 1 = off (reference behaviour); 3 or 5 = median of u,v before each warp */
  int32_t fast_math;   /* build-only arithmetic mode:
                          0 = IEEE float32, no contraction: bit-identical to oracle/ (default);
                          1 = the reference build's CUDA_FAST_MATH semantics (singularity/optflow.def:33-34):
                              a*b + c contracted as nvcc does, approximate division and sqrt.  Held to
                              the tolerance of DESIGN.md 2 against oracle/, not to bit identity;
                          2 = nvcc's default -fmad=true contraction alone, IEEE division and sqrt:
                              bit-identical to oracle/'s fma mode.
                          gamma != 0 and tau/theta < 0 solves stay IEEE. */
  int32_t profile;     /* build-only: 0 = cv::cuda::OpticalFlowDual_TVL1,
                          the reference's path (default); 1 = the schedule of OpenCV's CPU
                          cv::DualTVL1OpticalFlow: half-pixel pyramid/upsample, remap INTER_CUBIC
                          (a = -0.75, 1/32 px map, BORDER_CONSTANT), outer iterations each starting
                          with medianFiltering, inner iterations each checking the residual.
                          `iterations` is unused there; fast_math is ignored. */
  int32_t inner_iterations; /* profile 1: innerIterations (cv::DualTVL1OpticalFlow default 30) */
  int32_t outer_iterations; /* profile 1: outerIterations (default 10) */
} tvl1_params;

/* Per-call statistics.  Valid after tvl1_calc returns (host-side counters). */
typedef struct tvl1_stats {
  int32_t levels;                           /* effective pyramid depth (OpenCV mutates nscales_) */
  int32_t level_width[TVL1_MAX_LEVELS];
  int32_t level_height[TVL1_MAX_LEVELS];
  int64_t level_iterations[TVL1_MAX_LEVELS]; /* executed iterations summed over warps */
  int64_t iterations_total;
  int64_t checks_total;                     /* iterations that evaluated the residual (cuda::sum) */
  double algorithmic_bytes;                 /* SURVEY 8(d) byte model with executed counts */
  /* Optional caller-owned buffer: executed iterations per (level, warp), indexed
   * [level * warps + warp], level 0 = finest.  Left untouched when NULL. */
  int32_t *warp_iterations;
  int32_t warp_iterations_capacity;         /* number of int32 slots in warp_iterations */
  int32_t speculation_misses;               /* tvl1_calc: launches enqueued behind a residual check
                                             * that ran empty (a wrong guess);
                                             * tvl1_calc_batch: warps whose constants were not
                                             * stored but needed (re-gathered) */
  /* Filled only when profiling is enabled (tvl1_set_profiling): HIP-event time,
   * launch count and algorithmic bytes per kernel class, on the solve's stream.
   * Class 0 = fused primal-dual iteration (K6+K8+K7 partials), 1 = warpBackward
   * (K5), 2 = everything else (convert, pyramid, gradient, upsample, output), 3 = a batch's
   * coarsest level solved on chip in one launch (warps, iterations and stopping rule; bound
   * on chip, so it stays out of class 0's HBM roofline). */
  double kernel_ms[4];
  int64_t kernel_launches[4];
  double kernel_bytes[4];      /* SURVEY 8(d) algorithmic bytes (64 B/px per iteration for class 0) */
  double kernel_hbm_bytes[4];  /* compulsory HBM bytes of THIS implementation's tiling */
} tvl1_stats;

typedef struct tvl1_ctx tvl1_ctx;

/* Fill params with the reference defaults of generate_TV_args (optflow.cpp:500-514). */
void tvl1_params_default(tvl1_params *params);

/* Create a solver bound to HIP device `device` (ordinal).  Replaces
 * OpticalFlowDual_TVL1::create (optflow.cpp:518).  Scratch grows on demand. */
tvl1_status tvl1_create(tvl1_ctx **out, int device, const tvl1_params *params);

/* Replace the solver parameters of an existing ctx (the reference re-creates the
 * solver per call, optflow.cpp:518; this avoids re-allocating scratch). */
tvl1_status tvl1_set_params(tvl1_ctx *ctx, const tvl1_params *params);

/* Solve I0 -> I1 on DEVICE memory.  Replaces solver->calc(frame0, frame1, flow)
 * (optflow.cpp:519) followed by cuda::split (optflow.cpp:404).
 *   I0, I1 : device u8 images, row pitch pitch0/pitch1 bytes (ROI views allowed)
 *   u, v   : device f32 outputs, row pitch flow_pitch bytes
 *   stats  : may be NULL
 *   stream : hipStream_t as void*, NULL = default stream            */
tvl1_status tvl1_calc(tvl1_ctx *ctx,
                      const uint8_t *I0, size_t pitch0,
                      const uint8_t *I1, size_t pitch1,
                      int32_t width, int32_t height,
                      float *u, float *v, size_t flow_pitch,
                      tvl1_stats *stats, void *stream);

/* CV_32FC1 frames: calc converts f32 inputs with convertTo(CV_32F, 255), so
 * pixel values are expected in [0, 1]; everything else as tvl1_calc.  Device pointers,
 * pitches in bytes (>= 4 * width, multiples of 4). */
tvl1_status tvl1_calc_f32(tvl1_ctx *ctx, const float *I0, size_t pitch0, const float *I1,
                          size_t pitch1, int32_t width, int32_t height, float *u, float *v,
                          size_t flow_pitch, tvl1_stats *stats, void *stream);

/* Batched solve (build addition for the production workload, SURVEY 3.2: two 3072x100
 * ROI strips per slice pair, each a solve of ~400 tiny launches): n pairs of one size,
 * pair b at I0 + b*pair_stride0, I1 + b*pair_stride1 (bytes; 0 = the same frame for every
 * pair; device pointers, as in
 * tvl1_calc), flow of pair b at u / v + b*flow_pair_stride.  Up to 256 pairs share every
 * kernel launch; each pair's flow and per-warp iteration counts are those of tvl1_calc
 * (bit-identical; with fast_math = 1 within the same tolerance as tvl1_calc's).  stats: NULL
 * or an array of n.  gamma != 0 and profile 1 solve the pairs one by one.  Asynchronous on
 * `stream` like tvl1_calc, but the host waits at residual checks. */
tvl1_status tvl1_calc_batch(tvl1_ctx *ctx, int32_t n,
                            const uint8_t *I0, size_t pitch0, size_t pair_stride0,
                            const uint8_t *I1, size_t pitch1, size_t pair_stride1,
                            int32_t width, int32_t height,
                            float *u, float *v, size_t flow_pitch, size_t flow_pair_stride,
                            tvl1_stats *stats, void *stream);

/* ---- Feature pre-alignment (features.cpp:46-167, optflow.cpp:366-377) ----
 * find_alignment(frame1, frame0): ORB keypoints and descriptors on the GPU, brute-force
 * Hamming 2-NN + ratio test, RANSAC / LMEDS homography on the host; affine = its top 2x3
 * (maps frame1 coordinates onto frame0), or the identity when <= 10 matches survive the
 * ratio test (outcome 1) or the homography is missing or zooms by more than 20 % (outcome
 * 2).  SURF (features = 2) is served by the ORB path.  Parity with OpenCV unpinned (see
 * fibsem-optflow_amd/csrc/tvl1_align.hpp).  Inputs are device pointers; synchronous. */
typedef struct tvl1_align_params {
  int32_t nfeatures;           /* 5000 features.cpp:22 */
  float scale_factor;          /* 1.2  :23 */
  int32_t nlevels;             /* 8    :24 */
  int32_t edge_threshold;      /* 31   :25 */
  int32_t first_level;         /* 0    :26 */
  int32_t wta_k;               /* 2    :27 (only 2 is supported) */
  int32_t patch_size;          /* 31   :28 (only 31 is supported) */
  int32_t fast_threshold;      /* 20   :29 */
  int32_t blur_for_descriptor; /* 0    :30 */
  float ratio;                 /* 0.8  :109 */
  int32_t method;              /* homo: 8 = RANSAC (default, :133), 4 = LMEDS */
  double ransac_threshold;     /* ransac: 5 (:133) */
} tvl1_align_params;

void tvl1_align_params_default(tvl1_align_params *p);

tvl1_status tvl1_find_alignment(tvl1_ctx *ctx,
                                const uint8_t *frame1, size_t pitch1, int32_t w1, int32_t h1,
                                const uint8_t *frame0, size_t pitch0, int32_t w0, int32_t h0,
                                const tvl1_align_params *params, float affine[6],
                                int32_t *n_good, int32_t *outcome, void *stream);

/* The two stages of tvl1_find_alignment as calls of their own (ABI 7):
 *
 * cv::cuda::ORB::detectAndCompute(frame, noArray(), keypoints, descriptors)
 * (features.cpp:56-61) of one device u8 frame: the keypoints tvl1_find_alignment uses, levels
 * in order, best response first within a level.  kp: 5 floats per keypoint -- x, y (level-0
 * px, cv::KeyPoint::pt), octave (the pyramid level), angle (degrees in [0, 360)), response;
 * desc: 32 bytes per keypoint (rBRIEF, 256 bits, bit j of byte k = test 8k + j).  Host
 * outputs for up to cap keypoints; *n = how many were found (may exceed cap: the first cap
 * are written).  Synchronous on stream. */
tvl1_status tvl1_orb_detect(tvl1_ctx *ctx, const uint8_t *frame, size_t pitch, int32_t w,
                            int32_t h, const tvl1_align_params *params, float *kp,
                            uint8_t *desc, int32_t cap, int32_t *n, void *stream);

/* cv::cuda::DescriptorMatcher::createBFMatcher(NORM_HAMMING)->knnMatch(query, train, k = 2)
 * (features.cpp:97-104) on host descriptor lists (32 bytes each), on the GPU: for query i,
 * idx[2i], idx[2i+1] = the nearest and second-nearest train index (ties: the lower index;
 * -1, with distance 2^30, where the train set has no such descriptor), dist[2i], dist[2i+1]
 * = their Hamming distances.  Synchronous on stream. */
tvl1_status tvl1_match_knn2(tvl1_ctx *ctx, const uint8_t *query, int32_t nq,
                            const uint8_t *train, int32_t nt, int32_t *idx, int32_t *dist,
                            void *stream);

/* cv::findHomography(src, dst, method, ransacReprojThreshold) on host point lists
 * (features.cpp:131-133; the model tvl1_find_alignment fits): method 8 = RANSAC, 4 = LMEDS,
 * 0 = all points; a normalised DLT refit on the inliers, then 10 Levenberg-Marquardt steps
 * on their reprojection error.  src / dst: n (x, y) pairs; H: row-major 3x3, H[8] = 1;
 * inlier_mask: n bytes or NULL.  Host only (no GPU work, ctx not needed).  TVL1_EINVAL for
 * n < 4 or a bad method; TVL1_ESIZE when no model is found (all hypotheses degenerate). */
tvl1_status tvl1_find_homography(const float *src_xy, const float *dst_xy, int32_t n,
                                 int32_t method, double ransac_threshold, double H[9],
                                 uint8_t *inlier_mask);

/* cv::cuda::warpAffine(src, dst, M, dsize, INTER_LINEAR, BORDER_CONSTANT, 0) on u8
 * (optflow.cpp:370): dst(x, y) = src(M^-1 (x, y)).  Device pointers, async on stream. */
tvl1_status tvl1_warp_affine_u8(tvl1_ctx *ctx, const uint8_t *src, size_t src_pitch,
                                int32_t sw, int32_t sh, uint8_t *dst, size_t dst_pitch,
                                int32_t dw, int32_t dh, const float affine[6], void *stream);

/* solve_wrapper's features branch with the alignment's affine (optflow.cpp:411-443,
 * 468-473): map = flow + grid, warpAffine(map, M), then flow = map' - grid (flow_output 1)
 * or map' (0), and 0 where I1 <= 1.  Device pointers, async on stream. */
tvl1_status tvl1_postprocess_affine(tvl1_ctx *ctx, float *u, float *v, size_t flow_pitch,
                                    const uint8_t *I1, size_t pitch1, int32_t width,
                                    int32_t height, int32_t flow_output, const float affine[6],
                                    void *stream);

/* Same on HOST memory: upload, solve, download, synchronize.
 * (GpuMat::upload optflow.cpp:315-316 ... download :475-476) */
tvl1_status tvl1_calc_host(tvl1_ctx *ctx,
                           const uint8_t *I0, size_t pitch0,
                           const uint8_t *I1, size_t pitch1,
                           int32_t width, int32_t height,
                           float *u, float *v, size_t flow_pitch,
                           tvl1_stats *stats);

/* Output post-processing of solve_wrapper (optflow.cpp:411-473), in place on
 * device u, v:  mode 0 = "flow" (unchanged), 1 = "map" (u += x, v += y),
 * 2 = features branch with output_type "flow" under an identity alignment
 * (u = (u + x) - x, optflow.cpp:429-437); then u = v = 0 wherever I1 <= 1
 * (cuda::threshold THRESH_BINARY_INV + setTo). */
tvl1_status tvl1_postprocess(tvl1_ctx *ctx, float *u, float *v, size_t flow_pitch,
                             const uint8_t *I1, size_t pitch1,
                             int32_t width, int32_t height, int32_t mode, void *stream);

/* tvl1_postprocess on n same-size pairs of a batch in one launch (ABI 8; the CLI's batched
 * strip jobs, solve_wrapper optflow.cpp:411-473 per ROI): pair b's flow at u / v +
 * b*flow_pair_stride, its frame1 at I1 + b*pair_stride1 (bytes).  Device pointers, async. */
tvl1_status tvl1_postprocess_batch(tvl1_ctx *ctx, int32_t n, float *u, float *v,
                                   size_t flow_pitch, size_t flow_pair_stride,
                                   const uint8_t *I1, size_t pitch1, size_t pair_stride1,
                                   int32_t width, int32_t height, int32_t mode, void *stream);

/* The flow values of a few chosen px (ABI 8; plane_elems since ABI 9): out_u[i] =
 * u[offsets[i]], out_v[i] = v[offsets[i]], offsets in floats from the device pointers u / v
 * (host array of n).  Every offset must lie in [0, plane_elems), the number of floats
 * addressable from u and from v (for a batch: pairs x pair stride); any other offset is
 * TVL1_EINVAL before anything is launched.  The point-match output draws npoints px per ROI
 * (random_points, optflow.cpp:522-572) and needs only their flow, not the whole field.
 * Host outputs; synchronous on stream. */
tvl1_status tvl1_gather_flow(tvl1_ctx *ctx, const float *u, const float *v, int64_t plane_elems,
                             const int64_t *offsets, int32_t n, float *out_u, float *out_v,
                             void *stream);

/* The ctx's own non-blocking HIP stream (hipStream_t as void*): callers that keep
 * several pairs in flight on one device give each ctx its own stream this way. */
void *tvl1_stream(tvl1_ctx *ctx);

/* Enable (1) / disable (0) per-kernel-class HIP-event timing into tvl1_stats. */
tvl1_status tvl1_set_profiling(tvl1_ctx *ctx, int32_t enable);

/* Destroy a ctx and free its device scratch. */
void tvl1_destroy(tvl1_ctx *ctx);

/* Last error message of ctx (or of the last failed tvl1_create when ctx==NULL). */
const char *tvl1_last_error(const tvl1_ctx *ctx);

/* ABI version (TVL1_ABI_VERSION) — lets an FFI binding check what it loaded. */
int32_t tvl1_abi_version(void);

/* Number of visible HIP devices (0 when no GPU); never initialises a context. */
int32_t tvl1_device_count(void);

#ifdef __cplusplus
}
#endif

#endif /* FIBSEM_OPTFLOW_AMD_TVL1_H */
