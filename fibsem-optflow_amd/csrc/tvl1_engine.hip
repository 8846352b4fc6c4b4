// tvl1_engine.hip — host side of the MI355X TV-L1 engine + the C-ABI of include/tvl1.h.
//
// Replaces the reference's solver boundary /root/reference/src/optflow.cpp:516-520
// (TVL1_solve -> cv::cuda::OpticalFlowDual_TVL1::create(...)->calc(...)).  The
// host loop below restates OpenCV 3.4.1 calcImpl/procOneScale
// and launches the gfx950 kernels of tvl1_kernels.hpp.  There is no CPU path:
// every stage runs on the device; the only device->host traffic inside a solve is
// the residual of "check" iterations, read exactly where OpenCV reads it.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <atomic>
#include <chrono>

#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tvl1.h"
#include "tvl1_kernels.hpp"
#include "tvl1_batch.hpp"
#include "tvl1_align.hpp"

// the iteration passes are compiled in tvl1_passes.hip (another instruction scheduler)
namespace tvl1k {
#define TVL1_PASS_INSTANCE(...) extern template __global__ void __VA_ARGS__;
#include "tvl1_passes.inc"
#undef TVL1_PASS_INSTANCE
}  // namespace tvl1k

using namespace tvl1k;

namespace {

thread_local std::string g_create_error;

constexpr int kStripRows = 32;   // rows per wave strip in k_iterate
constexpr int kTbMax = 4;        // max iterations fused per pass in k_iterate_tb
constexpr int kRollMinSeg = 8;   // smallest k_iterate_roll segment (rows)
#ifndef TVL1_WI_M
#define TVL1_WI_M 6
#endif
// k_warp_iter's window margin (px): flows within about +-(M - 1) px gather from its LDS
// window ring, larger ones from HBM (the same taps)
constexpr int kWiMargin = TVL1_WI_M;
// Batched passes on levels at most this wide use 64-px bands, kb_iterate_roll<K, 1> (95
// VGPRs, 5 wavefronts per SIMD, against 3 for the LDS-staged <4, 2>): the production strips'
// levels of 515-1573 x 17-51 px give a batch too few 128-px bands to fill the SIMDs, so twice
// the wavefronts with half the work each finish sooner.  Measured on the strip workload (with
// the register-ring <4, 2>): cut-off 1700 +2.4 %, 1100 +1.2 %, 2500 +1.8 %, every level -3 %;
// with the LDS-staged one 1700 and 1100 +1.3 %, 2500 +0.2 %.
constexpr int kBatchPx1W = 1700;

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
// IterArgs::taut_small: the projection's ng = 1 + taut*g ignores g below 2^-48 when |taut|
// <= 2^20, so sqrt_nn may skip its (0, 2^-96) form (tvl1_kernels.hpp, sqrt_nn); NaN: false
inline int taut_small(float taut) { return std::fabs(taut) <= 0x1p20f ? 1 : 0; }

struct Geometry {
  int W = 0, H = 0, L = 0;
  int ws[TVL1_MAX_LEVELS], hs[TVL1_MAX_LEVELS], ps[TVL1_MAX_LEVELS];
  bool gamma = false;
};

}  // namespace

struct tvl1_ctx {
  int device = 0;
  tvl1_params prm{};
  std::string err;
  hipStream_t own_stream = nullptr;

  // arena
  char *arena = nullptr;
  size_t arena_bytes = 0;
  Geometry geo;
  bool geo_valid = false;

  float *I0s[TVL1_MAX_LEVELS] = {};
  float *I1s[TVL1_MAX_LEVELS] = {};
  float4 *G = nullptr;
  float *U[2][3] = {};   // u1, u2, u3
  float *Pd[2][6] = {};  // p11, p12, p21, p22, p31, p32
  float *C[2][3] = {};   // two sets of warp constants I1wx, I1wy, rho_c (speculation)
  uint8_t *in0 = nullptr, *in1 = nullptr;   // staging for tvl1_calc_host
  float *outu = nullptr, *outv = nullptr;
  double *partials = nullptr;
  int partials_cap = 0;
  double *pinned = nullptr;      // host-pinned residual landing slot (coherent, mapped)
  double *pinned_dev = nullptr;  // its device address: k_reduce stores the residual there
  hipEvent_t ev_check[2] = {};   // recorded after each residual check (by sequence parity)
  unsigned long long *gate = nullptr;   // device word: the speculation gate
  int spec = 1;                   // TVL1_SPEC: 0 no launches enqueued behind a check, 1 when the
                                  // solve is alone on its device (this process), 2 always
  int spec_trace = 0;             // TVL1_SPEC_TRACE=1: one stderr line per check and guess
  unsigned long long check_seq = 0;  // sequence number of the last residual check
  int poll = 1;                      // TVL1_POLL: wait for a residual by polling its
                                     // sequence number in host memory (0: event sync)
  hipEvent_t ev_order = nullptr;  // orders work on the caller's stream after a zero fill
  hipEvent_t ev_switch = nullptr; // orders a call on a new stream after the previous stream
  hipStream_t last_stream = nullptr;   // the stream the ctx's last call enqueued on
  bool last_stream_valid = false;
  struct Retired {                // an arena outgrown while possibly in use (arena_alloc)
    char *p;
    std::vector<hipEvent_t> done;   // recorded on every stream the ctx has worked on
  };
  std::vector<Retired> retired;
  std::vector<hipStream_t> streams;   // streams the ctx's work was enqueued on (note_stream)
  // dispatch: the defaults are the measured best; the environment knobs are
  // for tests (named in tests/test_gpu_parity.py) and diagnostics
  int roll_seg = 0;          // TVL1_ROLL_SEG: k_iterate_roll rows per segment (0 = auto)
  long roll_px4_min = 5000000;   // TVL1_ROLL_PX4_MIN: 2-iteration passes take 4 px per lane on
                                 // levels of at least this many px (2 px below: more waves)
  int roll_slots[kRollMax + 1][2][5] = {};   // resident k_iterate_roll<G, K, PX> wavefronts
  int fill = 100;            // TVL1_FILL: % of the resident slots a single-pair streaming launch
                             // is sized for while the solve is alone on its device, and
  int fill_shared = 60;      // TVL1_FILL_SHARED: ... while other solves of this process share
                             // the device (their blocks take the rest; DESIGN 9: 3 in flight
                             // +1.8 % at 60 %, and a pair alone keeps its 100 % latency)
                             // is sized for (segment rows)
  long roll_long_min = 0;    // >= 3-iteration passes stream (k_iterate_roll) on levels of at
                             // least this many 56 x 32 tiles, else k_iterate_tb
  int warp_ring_slots = 0;   // resident k_warp_ring<6, 2> blocks per device
  size_t buf_limit = ((size_t)1 << 31) - 4096;   // TVL1_BUF_LIMIT: plane bytes the
                             // buffer-addressed kernels take (tests force the fallbacks)
  int fuse = 1;              // TVL1_FUSE=0: no k_warp_iter (warp + first pass as two kernels)
  int tb4 = 1;               // TVL1_TB4=0: blocked passes (gamma = 0) in 64 x 32 regions
                             // (k_iterate_tb) instead of 64 x 48 (k_iterate_tb4)
  long fuse_min = 4000000;   // TVL1_FUSE_MIN: k_warp_iter on levels of >= this many px; smaller
                             // levels: k_warp_ring + the pass (as fast, and their warps mostly
                             // run past the first check).  4 M since the two-consumer form
                             // (C2's 4.2 Mpx level 4: one pair alone -3.7 %, in flight +0.3 %)
  int witer_slots = 0;       // resident k_warp_iter<6, -, 128, 1, wi_nc> blocks per device
  int mid = 1;               // TVL1_MID=0: no mid-check passes (k_iterate_roll_mid, DESIGN.md
                             // §4.1 of r6): two 2-iteration passes of a converging warp as one
                             // (C2 in flight +2.5 %, profiles/r6/final_mid/)
  double mid_min = 1.1;      // TVL1_MID_MIN: ... when the check before them read at least this
                             // many eps^2 W H (the first of the two checks then rarely stops)
  int mid_slots = 0;         // resident k_iterate_roll_mid wavefronts
  int wi_nc = 2;             // TVL1_WI_NC: k_warp_iter consumer wavefronts (2: one per
                             // iteration of the pass; 1: both on one wave)
  // batch arena (tvl1_calc_batch): per logical plane, kBatchMax pairs' copies
  char *barena = nullptr;
  size_t barena_bytes = 0;
  int bW = 0, bH = 0, bL = 0, bn = 0;   // geometry it is laid out for
  int bws[TVL1_MAX_LEVELS] = {}, bhs[TVL1_MAX_LEVELS] = {};   // ... and its level sizes
  float *bI0s[TVL1_MAX_LEVELS] = {}, *bI1s[TVL1_MAX_LEVELS] = {};
  size_t bips[TVL1_MAX_LEVELS] = {};    // pair stride of level s image planes (floats)
  float *bU[2][2] = {}, *bP[2][4] = {}, *bC[3] = {};
  size_t bps = 0;                       // pair stride of the level-0-sized planes (floats)
  double *bpartials = nullptr;
  int batch_fuse = 1;                   // TVL1_BATCH_FUSE=0: no fused warp + first pass
  int batch_group = 1;                  // TVL1_BATCH_GROUP=0: r3's lock-step passes (the
                                        // shortest pass any pair allows, for all)
  int batch_store_pred = 1;             // TVL1_BATCH_STORE=1: kb_warp_iter always stores the
                                        // warp constants (r3); default: only predicted pairs
  int batch_px1_w = kBatchPx1W;         // TVL1_BATCH_PX1_W: batched passes on levels at most
                                        // this wide run 64-px bands (1 px per lane)
  int kb1_slots[kRollMax + 1] = {};     // resident kb_iterate_roll<K, 1> wavefronts
  int batch_seg_min = 128;              // TVL1_BATCH_SEG_MIN: batched passes never split a
                                        // level into segments shorter than min(rows, this)
                                        // (0: roll_segment alone)
  int probe_lds = 0;                    // TVL1_PROBE_ROLL_LDS: dynamic LDS per k_iterate_roll
                                        // block (occupancy probe only; with the LDS-staged
                                        // passes' 40 KiB, at most 120 KiB)
  int probe_wi_lds = 0;                 // TVL1_PROBE_WI_LDS: the same for k_warp_iter (< 64 KiB)
  char *gather_scratch = nullptr;       // tvl1_gather_flow's offsets and values
  size_t gather_bytes = 0;
  int batch_small = 1;                  // TVL1_BATCH_SMALL=0: the coarsest level of a batch
                                        // streams like the others (no kb_small_level)
  char *small_scratch = nullptr;        // kb_small_level's per-warp iteration counts
  size_t small_bytes = 0;
  float *map_scratch = nullptr;         // tvl1_postprocess_affine's staged map planes
  size_t map_bytes = 0;
  char *align_scratch = nullptr;        // tvl1_find_alignment's pyramid, keys, descriptors
  size_t align_bytes = 0;
  int4 *align_pat = nullptr;            // the rBRIEF pair pattern (device, set once)
  int bnblk = 0;                        // partials per pair
  int check = 0;             // TVL1_CHECK=1: synchronise + check after every launch (diagnostics)

  // optional per-kernel-class HIP-event timing (tvl1_set_profiling)
  bool profiling = false;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  struct Mark {
    int cls;
    size_t a, b;
    double bytes;      // SURVEY 8(d) algorithmic bytes
    double hbm_bytes;  // compulsory bytes of this implementation
  };
  std::vector<Mark> marks;
};

static size_t prof_begin(tvl1_ctx *c, hipStream_t st) {
  if (!c->profiling) return 0;
  if (c->ev_used + 2 > c->ev_pool.size()) {
    for (int i = 0; i < 64; ++i) {
      hipEvent_t e;
      // timing-only events: no system-scope fence (cache writeback + invalidate) at each
      // record, which slowed the kernel after it and inflated the per-launch times ~6 %
      // against the rocprofv3 kernel trace (r3)
      if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) break;
      c->ev_pool.push_back(e);
    }
  }
  if (c->ev_used + 2 > c->ev_pool.size()) return 0;
  const size_t a = c->ev_used++;
  (void)hipEventRecord(c->ev_pool[a], st);
  return a + 1;  // 0 = not recording
}

static void prof_end(tvl1_ctx *c, hipStream_t st, size_t tok, int cls, double bytes,
                     double hbm_bytes = -1.0) {
  if (!c->profiling || tok == 0) return;
  const size_t b = c->ev_used++;
  (void)hipEventRecord(c->ev_pool[b], st);
  c->marks.push_back({cls, tok - 1, b, bytes, hbm_bytes < 0 ? bytes : hbm_bytes});
}

static tvl1_status set_err(tvl1_ctx *c, tvl1_status st, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c)
    c->err = buf;
  else
    g_create_error = buf;
  return st;
}

#define HIP_TRY(ctx, expr)                                                              \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return set_err((ctx), TVL1_EHIP, "%s failed: %s (%s:%d)", #expr,                 \
                     hipGetErrorString(e_), __FILE__, __LINE__);                        \
  } while (0)

static tvl1_status check_params(tvl1_ctx *c, const tvl1_params *p) {
  if (!p) return set_err(c, TVL1_EINVAL, "params is NULL");
  // CV_Assert(nscales_ > 0) in calcImpl
  if (p->nscales <= 0) return set_err(c, TVL1_EINVAL, "nscales must be > 0 (got %d)", p->nscales);
  if (p->warps < 0) return set_err(c, TVL1_EINVAL, "warps must be >= 0");
  if (p->iterations < 0) return set_err(c, TVL1_EINVAL, "iterations must be >= 0");
  if (!(p->theta != 0.0)) return set_err(c, TVL1_EINVAL, "theta must be non-zero (tau/theta)");
  if (!(p->scale_step > 0.0 && p->scale_step <= 1.0))
    return set_err(c, TVL1_EINVAL, "scaleStep must be in (0, 1]");
  if (p->median_filtering > 1 && p->median_filtering != 3 && p->median_filtering != 5)
    return set_err(c, TVL1_EINVAL, "medianFiltering must be 1 (off), 3 or 5");
  if (p->fast_math < 0 || p->fast_math > 2)
    return set_err(c, TVL1_EINVAL, "fastMath must be 0 (IEEE), 1 (fast) or 2 (fma) (got %d)",
                   p->fast_math);
  if (p->profile != 0 && p->profile != 1)
    return set_err(c, TVL1_EINVAL, "profile must be 0 (CUDA OpticalFlowDual_TVL1) or 1 (CPU DualTVL1) (got %d)",
                   p->profile);
  if (p->inner_iterations < 0 || p->outer_iterations < 0)
    return set_err(c, TVL1_EINVAL, "innerIterations / outerIterations must be >= 0");
  return TVL1_OK;
}

// Pyramid sizes exactly as calcImpl: round-half-even(cols*step), stop < 16.
static int pyramid_sizes(int w, int h, int nscales, double step, int *ws, int *hs) {
  int L = nscales < TVL1_MAX_LEVELS ? nscales : TVL1_MAX_LEVELS;
  ws[0] = w;
  hs[0] = h;
  for (int s = 1; s < L; ++s) {
    const int nw = (int)std::lrint((double)ws[s - 1] * step);
    const int nh = (int)std::lrint((double)hs[s - 1] * step);
    if (nw < 16 || nh < 16) return s;
    ws[s] = nw;
    hs[s] = nh;
  }
  return L;
}

// Arithmetic mode of a solve (kIEEE / kFast / kFma, tvl1_kernels.hpp): tvl1_params.fast_math
// for the gamma = 0 path with 0 <= tau/theta < inf; gamma != 0 and taut < 0 solves run the
// IEEE kernels.
static int math_of(const tvl1_params &p) {
  const float taut = (float)(p.tau / p.theta);
  const bool exact_div = !(taut >= 0.0f && taut <= FLT_MAX);
  return p.gamma != 0.0 || exact_div ? kIEEE : p.fast_math;
}

// Rows per k_iterate_roll segment.  Every wavefront runs (rows + 2K) steps, so the pass
// takes about rounds x (rows + 2K) step times, rounds = ceil(wavefronts / resident slots):
// pick the split into segments that minimises that (a partial last round idles most of
// the device; short segments repeat the 2K-row halo).
static int roll_segment(int bands, int lh, int k, int slots) {
  if (slots <= 0) slots = 4096;
  int best = lh;
  long best_cost = -1;
  for (int R = 1; R <= 4; ++R) {
    const int segs = std::max(1, R * slots / bands);
    const int seg = std::max(kRollMinSeg, (lh + segs - 1) / segs);
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

static int iterate_blocks(int W, int H) {
  const int segs = (W + kSegPx - 1) / kSegPx;
  const int strips = (H + kStripRows - 1) / kStripRows;
  const int waves = segs * strips;
  return (waves + 3) / 4;
}

// (Re)allocate one of the ctx's scratch arenas, zero-filled, for work on stream `use`.
// The old allocation may still be read by work the ctx enqueued (tvl1_calc is
// asynchronous).  It is retired, not freed at once: events recorded on the ctx's recent
// streams (note_stream keeps the last 8) mark its last use, and reap_retired releases it
// once they are done, or waits for the oldest when more than kRetiredMax are held, or at
// tvl1_destroy.  What makes the release safe is hipFree itself: on ROCm it synchronises the
// whole device before it frees, so a retired arena is never freed under a kernel that
// still reads it, whatever stream that kernel is on.  The price is that a reap stalls every
// other context's pairs in flight for that moment; it happens only when an arena was
// outgrown (geometry growth, at most twice held), never in the steady state of a job whose
// sizes repeat.  The arenas are only ever grown: a smaller layout re-lays the existing
// allocation (ensure_geometry, ensure_batch), ordered across streams by order_streams.  The
// work on `use` is ordered after the zero fill by an event, not by a host wait.  (The stream-ordered
// allocator, hipMallocAsync / hipFreeAsync, would release in stream order too, but it
// deadlocked against a concurrent hipStreamDestroy on this ROCm, so it is not used.)
// Remember a stream the ctx enqueues work on, so a retired arena can be released once every
// such stream has passed the point of its retirement.
static void note_stream(tvl1_ctx *c, hipStream_t s) {
  for (size_t i = 0; i < c->streams.size(); ++i)
    if (c->streams[i] == s) {   // most recent last
      c->streams.erase(c->streams.begin() + i);
      break;
    }
  c->streams.push_back(s);
  if (c->streams.size() > 8) c->streams.erase(c->streams.begin());
}

static void free_retired(tvl1_ctx::Retired &r) {
  (void)hipFree(r.p);
  for (hipEvent_t e : r.done) (void)hipEventDestroy(e);
  r.done.clear();
}

// Release the retired arenas whose work has finished (every event done); with `wait`, the
// oldest ones are waited for too until at most kRetiredMax remain.  A caller that alternates
// geometries therefore holds a bounded number of old arenas.
static constexpr size_t kRetiredMax = 2;
static void reap_retired(tvl1_ctx *c, bool wait) {
  size_t keep = 0;
  for (size_t i = 0; i < c->retired.size(); ++i) {
    tvl1_ctx::Retired &r = c->retired[i];
    bool done = true;
    const bool must = wait && c->retired.size() - i > kRetiredMax;
    for (hipEvent_t e : r.done) {
      if (must) (void)hipEventSynchronize(e);
      else if (hipEventQuery(e) != hipSuccess) done = false;
    }
    (void)hipGetLastError();   // hipErrorNotReady is not an error
    if (done) free_retired(r);
    else c->retired[keep++] = r;
  }
  c->retired.resize(keep);
}

// A ctx's arenas are reused (and re-laid in place) by every call, so a call on a stream
// other than the previous call's must not start before that stream's work on them is done
// (a batch re-laid for a new geometry on stream B while stream A's kb_output still
// reads the old layout).  One event record + stream wait per switch of streams; a ctx that
// stays on one stream pays nothing.  A stream the caller has destroyed since has nothing
// left on it: its record fails and is ignored.
static void order_streams(tvl1_ctx *c, hipStream_t st) {
  if (c->last_stream_valid && c->last_stream != st) {
    if (hipEventRecord(c->ev_switch, c->last_stream) == hipSuccess)
      (void)hipStreamWaitEvent(st, c->ev_switch, 0);
    (void)hipGetLastError();
  }
  c->last_stream = st;
  c->last_stream_valid = true;
}

static tvl1_status arena_alloc(tvl1_ctx *c, char **arena, size_t *have, size_t bytes,
                               hipStream_t use) {
  note_stream(c, use);
  if (*arena) {
    tvl1_ctx::Retired r{*arena, {}};
    note_stream(c, c->own_stream);
    for (hipStream_t s : c->streams) {
      hipEvent_t e = nullptr;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        continue;
      }
      if (hipEventRecord(e, s) != hipSuccess) {   // a destroyed stream: nothing left on it
        (void)hipGetLastError();
        (void)hipEventDestroy(e);
        continue;
      }
      r.done.push_back(e);
    }
    c->retired.push_back(r);
    *arena = nullptr;
    *have = 0;
    reap_retired(c, true);
  }
  hipError_t e = hipMalloc((void **)arena, bytes);
  if (e != hipSuccess && !c->retired.empty()) {
    // out of memory with outgrown arenas held: release them (hipFree waits for the device;
    // a rare path, better than failing) and try once more
    (void)hipGetLastError();
    for (auto &r : c->retired) free_retired(r);
    c->retired.clear();
    e = hipMalloc((void **)arena, bytes);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();   // not sticky: the caller may retry smaller
    *arena = nullptr;
    return set_err(c, TVL1_ENOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
  }
  *have = bytes;
  // zero once so pitch padding starts finite (hipMemsetAsync on the ctx's stream: a plain
  // hipMemset runs on the legacy null stream, unordered with non-blocking streams)
  HIP_TRY(c, hipMemsetAsync(*arena, 0, bytes, c->own_stream));
  if (use != c->own_stream) {
    HIP_TRY(c, hipEventRecord(c->ev_order, c->own_stream));
    HIP_TRY(c, hipStreamWaitEvent(use, c->ev_order, 0));
  }
  return TVL1_OK;
}

// Carve the arena for a geometry; grows (never shrinks) the device allocation.  The
// calls's work goes to stream st.
static tvl1_status ensure_geometry(tvl1_ctx *c, int W, int H, hipStream_t st) {
  order_streams(c, st);
  note_stream(c, st);
  if (!c->retired.empty()) reap_retired(c, false);
  Geometry g;
  g.W = W;
  g.H = H;
  g.gamma = c->prm.gamma != 0.0;
  g.L = pyramid_sizes(W, H, c->prm.nscales, c->prm.scale_step, g.ws, g.hs);
  for (int s = 0; s < g.L; ++s) g.ps[s] = (int)align_up((size_t)g.ws[s], 64);
  if (c->geo_valid && g.W == c->geo.W && g.H == c->geo.H && g.L == c->geo.L &&
      g.gamma == c->geo.gamma && !memcmp(g.ws, c->geo.ws, sizeof(int) * g.L) &&
      !memcmp(g.hs, c->geo.hs, sizeof(int) * g.L))
    return TVL1_OK;

  const size_t P0 = (size_t)g.ps[0];
  const size_t plane = P0 * (size_t)H * sizeof(float);
  size_t bytes = 0;
  for (int s = 0; s < g.L; ++s) bytes += 2 * (size_t)g.ps[s] * g.hs[s] * sizeof(float);
  bytes += 4 * plane;                       // G (float4)
  bytes += 2 * 3 * plane;                   // U[2][3]
  bytes += 2 * 6 * plane;                   // Pd[2][6]
  bytes += 2 * 3 * plane;                   // C[2]
  bytes += 2 * align_up(P0 * H, 256);       // in0, in1 (u8)
  bytes += 2 * plane;                       // outu, outv
  // residual partials: k_iterate_tb worst case (RH 32 at 4 iterations: 56 x 24 px per
  // block), k_iterate_roll worst case (56-px bands, segments of kRollMinSeg rows)
  const int tb_blocks = ((W + 55) / 56) * ((H + 23) / 24);
  const int roll_waves = ((W + 55) / 56) * ((H + kRollMinSeg - 1) / kRollMinSeg);
  const int nblk = std::max(std::max(iterate_blocks(W, H), tb_blocks), roll_waves) + 64;
  bytes += align_up((size_t)nblk * sizeof(double), 256);
  bytes += 4096;                            // alignment slack

  if (bytes > c->arena_bytes) {
    c->geo_valid = false;
    const tvl1_status r = arena_alloc(c, &c->arena, &c->arena_bytes, bytes, st);
    if (r != TVL1_OK) return r;
  }
  char *p = c->arena;
  auto take = [&](size_t n) {
    char *r = p;
    p += align_up(n, 256);
    return r;
  };
  for (int s = 0; s < TVL1_MAX_LEVELS; ++s) c->I0s[s] = c->I1s[s] = nullptr;
  for (int s = 0; s < g.L; ++s) {
    const size_t n = (size_t)g.ps[s] * g.hs[s] * sizeof(float);
    c->I0s[s] = (float *)take(n);
    c->I1s[s] = (float *)take(n);
  }
  c->G = (float4 *)take(4 * plane);
  for (int b = 0; b < 2; ++b)
    for (int k = 0; k < 3; ++k) c->U[b][k] = (float *)take(plane);
  for (int b = 0; b < 2; ++b)
    for (int k = 0; k < 6; ++k) c->Pd[b][k] = (float *)take(plane);
  for (int b = 0; b < 2; ++b)
    for (int k = 0; k < 3; ++k) c->C[b][k] = (float *)take(plane);
  c->in0 = (uint8_t *)take(P0 * H);
  c->in1 = (uint8_t *)take(P0 * H);
  c->outu = (float *)take(plane);
  c->outv = (float *)take(plane);
  c->partials = (double *)take((size_t)nblk * sizeof(double));
  c->partials_cap = nblk;
  c->geo = g;
  c->geo_valid = true;
  return TVL1_OK;
}

// Diagnostics (TVL1_CHECK=1): after every launch, synchronise and report which
// kernel at which level / warp / iteration failed.
#define DIAG(ctx, st, what, lev, warp, it)                                                   \
  do {                                                                                     \
    if ((ctx)->check) {                                                                    \
      hipError_t e_ = hipStreamSynchronize(st);                                            \
      if (e_ == hipSuccess) e_ = hipGetLastError();                                        \
      if (e_ != hipSuccess)                                                                \
        return set_err((ctx), TVL1_EHIP, "%s failed at level %d warp %d n %d: %s", what,    \
                       (int)(lev), (int)(warp), (int)(it), hipGetErrorString(e_));         \
    }                                                                                      \
  } while (0)

// Launch the kernel instance of a runtime arithmetic mode (tvl1_params.fast_math):
// LAUNCH(FM) expands to the launch of the FM instantiation.
#define MATH_SWITCH(m, LAUNCH) \
  if ((m) == kFast) {          \
    LAUNCH(kFast)              \
  } else if ((m) == kFma) {    \
    LAUNCH(kFma)               \
  } else {                     \
    LAUNCH(kIEEE)              \
  }

static inline dim3 grid2(int w, int h, int z = 1) {
  return dim3((unsigned)((w + 63) / 64), (unsigned)((h + 3) / 4), (unsigned)z);
}
static const dim3 kBlk2(64, 4, 1);

// SURVEY 8(d) byte model with executed iteration counts (reported in stats).
static double survey_bytes(const Geometry &g, int warps, const int64_t *iters) {
  double B = 0.0;
  for (int l = 0; l < g.L; ++l) {
    const double N = (double)g.ws[l] * g.hs[l];
    B += N * (12.0 + 16.0 + 40.0 * warps + 64.0 * (double)iters[l]);
    if (l >= 1) B += N * 8.0;
    if (l < g.L - 1) B += N * 8.0;
  }
  const double N0 = (double)g.ws[0] * g.hs[0];
  B += N0 * (2.0 + 8.0) + N0 * 8.0;
  return B;
}

// calcImpl + procOneScale on device inputs already in the arena
// or caller memory.  Result left in caller's u, v.
//
// Host schedule.  procOneScale's inner loop
//     for (n = 0; error > eps^2*W*H && n < iterations; ++n)
//         calcError = eps > 0 && (n & 1) && prevError < eps^2*W*H
// is known on the host for every iteration up to and including the next check,
// so those iterations run as ONE temporally blocked pass (<= kTbMax iterations);
// the residual of the check is then read exactly where OpenCV reads it.
//
// One residual check: k_reduce sums the per-block partials in a fixed order into coherent
// host memory, and the host reads it once the kernel is done -- by polling the check's
// sequence number, which k_reduce stores after the residual (a few us sooner than an event
// wait), or with c->poll = 0 by an event.  The poll gives up on a stream error.
//
// Checks are split in two so that work can be enqueued behind a check before the host reads
// it (speculation): launch_check enqueues k_reduce (residual slot and event by the
// parity of its sequence number, so the next check cannot overwrite a residual the host has
// not read yet), wait_check reads it.
// (first: the partials start there: a mid-check pass's first check, k_iterate_roll_mid)
static tvl1_status launch_check(tvl1_ctx *c, hipStream_t st, int nparts, const CheckGate &g,
                                unsigned long long *seq_out, int first = 0) {
  unsigned long long *seq_dev = (unsigned long long *)(c->pinned_dev + 1);
  const unsigned long long seq = ++c->check_seq;
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(kBlock), 0, st, c->partials + first, nparts,
                     c->pinned_dev + ((seq & 1) ? 2 : 0), c->poll ? seq_dev : nullptr, seq, g);
  HIP_TRY(c, hipGetLastError());
  if (!c->poll) HIP_TRY(c, hipEventRecord(c->ev_check[seq & 1], st));
  *seq_out = seq;
  return TVL1_OK;
}

static tvl1_status wait_check(tvl1_ctx *c, hipStream_t st, unsigned long long seq, double *out) {
  unsigned long long *seq_host = (unsigned long long *)(c->pinned + 1);
  if (!c->poll) {
    HIP_TRY(c, hipEventSynchronize(c->ev_check[seq & 1]));
  } else {
    // a later (speculative) check may already have stored its own, larger number
    for (unsigned spins = 1;; ++spins) {
      if (__atomic_load_n(seq_host, __ATOMIC_ACQUIRE) >= seq) break;
      if ((spins & 4095) == 0) {   // now and then: has the stream failed or finished?
        const hipError_t e = hipStreamQuery(st);
        if (e != hipSuccess && e != hipErrorNotReady)
          return set_err(c, TVL1_EHIP, "residual check: %s", hipGetErrorString(e));
        if (e == hipSuccess && __atomic_load_n(seq_host, __ATOMIC_ACQUIRE) < seq)
          return set_err(c, TVL1_EHIP, "residual check: stream idle without the residual");
      }
      // spin briefly, then give the core away between reads (a caller may run many
      // contexts and other host work, e.g. the CLI's decode threads)
      if (spins < 2048)
        __builtin_ia32_pause();
      else
        sched_yield();
    }
  }
  *out = *(volatile double *)(c->pinned + ((seq & 1) ? 2 : 0));
  return TVL1_OK;
}

static tvl1_status read_residual(tvl1_ctx *c, hipStream_t st, int nparts, double *out) {
  CheckGate g{};
  unsigned long long seq = 0;
  const tvl1_status r = launch_check(c, st, nparts, g, &seq);
  if (r != TVL1_OK) return r;
  return wait_check(c, st, seq, out);
}

// resize(): an exact 2x downscale of INTER_LINEAR takes the INTER_AREA fast path
static int area_fast_of(double sx, double sy) {
  const int ix = (int)std::lrint(sx), iy = (int)std::lrint(sy);
  return std::fabs(sx - ix) < DBL_EPSILON && std::fabs(sy - iy) < DBL_EPSILON && ix == 2 && iy == 2;
}

// Profile 1 (tvl1_params.profile): the schedule of OpenCV's CPU
// cv::DualTVL1OpticalFlow::calc / procOneScale, restated in oracle/tvl1_oracle_dualtvl1.c.
// Per warp: remap (k_remap_cubic), then up to outerIterations rounds, each starting with
// medianFiltering, of up to innerIterations primal-dual iterations, every one of which
// evaluates the residual (one k_iterate launch + k_reduce + one host read each).  This is
// a compatibility mode, not the benchmark path: it keeps OpenCV's per-iteration check.
// The two input frames of a solve: u8 (tvl1_calc) or f32 (tvl1_calc_f32), device pointers,
// row pitches in bytes.
struct Frames {
  const void *I0, *I1;
  size_t pitch0, pitch1;
  bool f32;
};

// [A.1] I0f = convertTo(CV_32F, u8 ? 1 : 255) into the level-0 planes
static void convert_frames(tvl1_ctx *c, const Frames &in, int W, int H, hipStream_t st) {
  if (in.f32)
    hipLaunchKernelGGL(k_convert_f32, grid2(W, H, 2), kBlk2, 0, st, (const float *)in.I0,
                       in.pitch0, (const float *)in.I1, in.pitch1, c->I0s[0], c->I1s[0], W, H,
                       c->geo.ps[0]);
  else
    hipLaunchKernelGGL(k_convert_u8, grid2(W, H, 2), kBlk2, 0, st, (const uint8_t *)in.I0,
                       in.pitch0, (const uint8_t *)in.I1, in.pitch1, c->I0s[0], c->I1s[0], W, H,
                       c->geo.ps[0]);
}

static tvl1_status solve_dualtvl1(tvl1_ctx *c, const Frames &in, int W, int H, float *u,
                                  float *v, size_t fpitch, tvl1_stats *stats, hipStream_t st) {
  const tvl1_params &prm = c->prm;
  const Geometry &g = c->geo;
  const int L = g.L;
  const bool gam = g.gamma;
  const bool median = prm.median_filtering > 1;
  convert_frames(c, in, W, H, st);
  const double dscale = 1. / prm.scale_step;
  const int afast = area_fast_of(dscale, dscale);
  for (int s = 1; s < L; ++s)
    hipLaunchKernelGGL(k_resize_hp, grid2(g.ws[s], g.hs[s], 2), kBlk2, 0, st, c->I0s[s - 1],
                       c->I1s[s - 1], nullptr, g.ws[s - 1], g.hs[s - 1], g.ps[s - 1], c->I0s[s],
                       c->I1s[s], nullptr, g.ws[s], g.hs[s], g.ps[s], dscale, dscale, afast, 0,
                       1.0f);
  HIP_TRY(c, hipGetLastError());
  int ui = 0, pi = 0;
  {
    const size_t n = (size_t)g.ps[L - 1] * g.hs[L - 1] * sizeof(float);
    for (int k = 0; k < (gam ? 3 : 2); ++k) HIP_TRY(c, hipMemsetAsync(c->U[ui][k], 0, n, st));
  }
  const float l_t = (float)(prm.lambda * prm.theta);
  const float taut = (float)(prm.tau / prm.theta);
  const bool exact_div = !(taut >= 0.0f && taut <= FLT_MAX);
  const float upmul = (float)(1.0 / prm.scale_step);
  int64_t level_iters[TVL1_MAX_LEVELS] = {};
  for (int s = L - 1; s >= 0; --s) {
    const int lw = g.ws[s], lh = g.hs[s], P = g.ps[s];
    const float scaledEps = (float)(prm.epsilon * prm.epsilon * (double)(lw * lh));
    hipLaunchKernelGGL(k_gradient, grid2(lw, lh), kBlk2, 0, st, c->I1s[s], lw, lh, P, c->G);
    IterArgs a{};
    a.W = lw;
    a.H = lh;
    a.P = P;
    a.segs = (lw + kSegPx - 1) / kSegPx;
    a.strip_rows = kStripRows;
    a.l_t = l_t;
    a.theta = (float)prm.theta;
    a.gamma = (float)prm.gamma;
    a.taut = taut;
    a.taut_small = taut_small(taut);
    a.partials = c->partials;
    a.calc_err = 1;
    a.I1wx = c->C[0][0];
    a.I1wy = c->C[0][1];
    a.rho = c->C[0][2];
    const int nblk = iterate_blocks(lw, lh);
    bool p_zero = true;
    for (int wp = 0; wp < prm.warps; ++wp) {
      hipLaunchKernelGGL(k_remap_cubic, grid2(lw, lh), kBlk2, 0, st, c->I0s[s], c->G,
                         c->U[ui][0], c->U[ui][1], lw, lh, P, c->C[0][0], c->C[0][1],
                         c->C[0][2]);
      float error = FLT_MAX;
      int n = 0;
      for (int no = 0; error > scaledEps && no < prm.outer_iterations; ++no) {
        if (median) {
          hipLaunchKernelGGL(k_median, grid2(lw, lh, 2), kBlk2, 0, st, c->U[ui][0], c->U[ui][1],
                             lw, lh, P, prm.median_filtering, c->U[ui ^ 1][0], c->U[ui ^ 1][1]);
          if (gam)
            HIP_TRY(c, hipMemcpyAsync(c->U[ui ^ 1][2], c->U[ui][2], (size_t)P * lh * sizeof(float),
                                      hipMemcpyDeviceToDevice, st));
          ui ^= 1;
        }
        for (int ni = 0; error > scaledEps && ni < prm.inner_iterations; ++ni) {
          a.u1s = c->U[ui][0]; a.u2s = c->U[ui][1]; a.u3s = c->U[ui][2];
          a.u1d = c->U[ui ^ 1][0]; a.u2d = c->U[ui ^ 1][1]; a.u3d = c->U[ui ^ 1][2];
          a.p11s = c->Pd[pi][0]; a.p12s = c->Pd[pi][1]; a.p21s = c->Pd[pi][2];
          a.p22s = c->Pd[pi][3]; a.p31s = c->Pd[pi][4]; a.p32s = c->Pd[pi][5];
          a.p11d = c->Pd[pi ^ 1][0]; a.p12d = c->Pd[pi ^ 1][1]; a.p21d = c->Pd[pi ^ 1][2];
          a.p22d = c->Pd[pi ^ 1][3]; a.p31d = c->Pd[pi ^ 1][4]; a.p32d = c->Pd[pi ^ 1][5];
          a.p_zero = p_zero ? 1 : 0;
          if (gam && exact_div)
            hipLaunchKernelGGL((k_iterate<true, true, true>), dim3(nblk), dim3(kBlock), 0, st, a);
          else if (exact_div)
            hipLaunchKernelGGL((k_iterate<false, true, true>), dim3(nblk), dim3(kBlock), 0, st, a);
          else if (gam)
            hipLaunchKernelGGL((k_iterate<true, false, true>), dim3(nblk), dim3(kBlock), 0, st, a);
          else
            hipLaunchKernelGGL((k_iterate<false, false, true>), dim3(nblk), dim3(kBlock), 0, st, a);
          double e = 0.0;
          {
            const tvl1_status r = read_residual(c, st, nblk, &e);
            if (r != TVL1_OK) return r;
          }
          error = (float)e;
          p_zero = false;
          ui ^= 1;
          pi ^= 1;
          ++n;
        }
      }
      level_iters[s] += n;
      if (stats && stats->warp_iterations && s * prm.warps + wp < stats->warp_iterations_capacity)
        stats->warp_iterations[s * prm.warps + wp] = n;
    }
    HIP_TRY(c, hipGetLastError());
    if (s == 0) break;
    // resize(u, .., I0s[s-1].size()), then multiply u1, u2 (not u3) by 1/scaleStep
    const int dw = g.ws[s - 1], dh = g.hs[s - 1];
    const double sxu = 1. / ((double)dw / lw), syu = 1. / ((double)dh / lh);
    hipLaunchKernelGGL(k_resize_hp, grid2(dw, dh, gam ? 3 : 2), kBlk2, 0, st, c->U[ui][0],
                       c->U[ui][1], c->U[ui][2], lw, lh, P, c->U[ui ^ 1][0], c->U[ui ^ 1][1],
                       c->U[ui ^ 1][2], dw, dh, g.ps[s - 1], sxu, syu, area_fast_of(sxu, syu), 2,
                       upmul);
    ui ^= 1;
  }
  hipLaunchKernelGGL(k_output, grid2(W, H), kBlk2, 0, st, c->U[ui][0], c->U[ui][1], W, H,
                     g.ps[0], u, v, fpitch);
  HIP_TRY(c, hipGetLastError());
  if (stats) {
    stats->levels = L;
    int64_t tot = 0;
    for (int s = 0; s < TVL1_MAX_LEVELS; ++s) {
      stats->level_width[s] = s < L ? g.ws[s] : 0;
      stats->level_height[s] = s < L ? g.hs[s] : 0;
      stats->level_iterations[s] = s < L ? level_iters[s] : 0;
      tot += s < L ? level_iters[s] : 0;
    }
    stats->iterations_total = tot;
    stats->checks_total = tot;
    stats->speculation_misses = 0;
    stats->algorithmic_bytes = survey_bytes(g, prm.warps, level_iters);
    for (int k = 0; k < 4; ++k) {
      stats->kernel_ms[k] = 0.0;
      stats->kernel_launches[k] = 0;
      stats->kernel_bytes[k] = 0.0;
      stats->kernel_hbm_bytes[k] = 0.0;
    }
  }
  return TVL1_OK;
}

// Solves in progress per device in this process.  Speculation pays only for a
// solve alone on its device: with other pairs in flight their kernels already fill the
// check round trips, and a wrong guess would cost them GPU time.
static std::atomic<int> g_solving[64];
struct SolveCount {
  int d;
  explicit SolveCount(int dev) : d(dev & 63) { g_solving[d].fetch_add(1, std::memory_order_relaxed); }
  ~SolveCount() { g_solving[d].fetch_sub(1, std::memory_order_relaxed); }
};

static tvl1_status solve(tvl1_ctx *c, const Frames &in, int W, int H, float *u, float *v,
                         size_t fpitch, tvl1_stats *stats, hipStream_t st) {
  const tvl1_params &prm = c->prm;
  if (prm.profile == 1) return solve_dualtvl1(c, in, W, H, u, v, fpitch, stats, st);
  const SolveCount active(c->device);
  const Geometry &g = c->geo;
  const int L = g.L;
  const bool gam = g.gamma;
  const bool median = prm.median_filtering > 1;
  if (c->profiling) {
    c->ev_used = 0;
    c->marks.clear();
  }

  // [A.1] convertTo + [A.2] pyramid, kernel step = float(1/scaleStep)
  size_t tk = prof_begin(c, st);
  convert_frames(c, in, W, H, st);
  const float fdown = (float)(1.0 / prm.scale_step);
  const bool contract_pyr = contracts(math_of(prm));
  for (int s = 1; s < L; ++s) {
    if (contract_pyr)
      hipLaunchKernelGGL(k_resize_down2<true>, grid2(g.ws[s], g.hs[s], 2), kBlk2, 0, st,
                         c->I0s[s - 1], c->I1s[s - 1], g.ws[s - 1], g.hs[s - 1], g.ps[s - 1],
                         c->I0s[s], c->I1s[s], g.ws[s], g.hs[s], g.ps[s], fdown, fdown);
    else
      hipLaunchKernelGGL(k_resize_down2<false>, grid2(g.ws[s], g.hs[s], 2), kBlk2, 0, st,
                         c->I0s[s - 1], c->I1s[s - 1], g.ws[s - 1], g.hs[s - 1], g.ps[s - 1],
                         c->I0s[s], c->I1s[s], g.ws[s], g.hs[s], g.ps[s], fdown, fdown);
  }
  {
    double b = (double)W * H * (2 + 8);
    for (int s = 1; s < L; ++s) b += (double)g.ws[s] * g.hs[s] * 8 + (double)g.ws[s - 1] * g.hs[s - 1] * 8;
    prof_end(c, st, tk, 2, b);
  }
  HIP_TRY(c, hipGetLastError());

  int ui = 0, pi = 0;  // ping-pong indices of the u and p buffer sets
  int cb = 0;          // constants buffer (I1wx, I1wy, rho) of the current warp
  {                    // u = 0 at the coarsest level (no initial flow)
    const int s = L - 1;
    const size_t n = (size_t)g.ps[s] * g.hs[s] * sizeof(float);
    HIP_TRY(c, hipMemsetAsync(c->U[ui][0], 0, n, st));
    HIP_TRY(c, hipMemsetAsync(c->U[ui][1], 0, n, st));
    if (gam) HIP_TRY(c, hipMemsetAsync(c->U[ui][2], 0, n, st));
  }

  const float l_t = (float)(prm.lambda * prm.theta);
  const float taut = (float)(prm.tau / prm.theta);
  // The projection's shared-reciprocal division (dual_px) needs ng = 1 + taut*|grad u| >= 1;
  // other parameters take the one-iteration kernel with plain IEEE divisions.
  const bool exact_div = !(taut >= 0.0f && taut <= FLT_MAX);
  // arithmetic mode of the gamma = 0 kernels (kIEEE / kFast / kFma, tvl1_kernels.hpp);
  // gamma != 0 and taut < 0 solves run IEEE
  const int math = math_of(prm);
  const float theta_f = (float)prm.theta;
  const float gamma_f = (float)prm.gamma;
  const float upmul = (float)(1.0 / prm.scale_step);

  int64_t level_iters[TVL1_MAX_LEVELS] = {};
  int64_t checks = 0;
  int32_t spec_misses = 0;   // speculative launches that ran empty
  int mid_passes = 0, mid_taken = 0;   // mid-check passes; of those, ended on the mid state
  // share of the resident slots a streaming launch is sized for: all of them for a solve
  // alone on its device, fill_shared while other solves are in progress (their blocks fill
  // the rest instead of waiting for this launch's last round).  Segmentation never changes
  // a result (tests/test_gpu_parity.py TVL1_ROLL_SEG cases)
  auto fill_now = [&]() {
    return g_solving[c->device & 63].load(std::memory_order_relaxed) > 1 ? c->fill_shared : c->fill;
  };

  // ---- launch helpers
  // The streaming kernels (k_iterate_roll, k_warp_ring, k_warp_iter) take 32-bit buffer
  // byte offsets, and the iteration passes address a whole plane group (RollBufs: up to 6
  // planes at the level-0 plane stride) through one descriptor: a level whose largest group
  // reaches c->buf_limit bytes uses the 64-bit-addressed kernels (k_warp_img, k_iterate_tb).
  const size_t pstride = (size_t)g.ps[0] * g.H * sizeof(float);   // arena plane stride
  auto group_bytes = [&](int s, int planes) {
    return (size_t)(planes - 1) * pstride + (size_t)g.ps[s] * g.hs[s] * sizeof(float);
  };
  auto buffer_ok = [&](int s) { return group_bytes(s, gam ? 6 : 4) < c->buf_limit; };
  // the planes of a pass as RollBufs groups (the arena keeps each set's planes contiguous)
  auto roll_bufs = [&](int s, int uset, int pset, int cbuf) {
    RollBufs b;
    b.c = c->C[cbuf][0];
    b.us = c->U[uset][0];
    b.ud = c->U[uset ^ 1][0];
    b.ps = c->Pd[pset][0];
    b.pd = c->Pd[pset ^ 1][0];
    b.pstride = (unsigned)pstride;
    b.cb = (unsigned)group_bytes(s, 3);
    b.ub = (unsigned)group_bytes(s, gam ? 3 : 2);
    b.pb = (unsigned)group_bytes(s, gam ? 6 : 4);
    return b;
  };
  auto gather = [&](int s, int uset, int cbuf, int wp) -> tvl1_status {  // K5 warpBackward
    const int lw = g.ws[s], lh = g.hs[s], P = g.ps[s];
    size_t t0 = prof_begin(c, st);
    if (!buffer_ok(s)) {
      const int tx = (lw + kWarpTW - 1) / kWarpTW, ty = (lh + kWarpTH - 1) / kWarpTH;
#define WARP_IMG(FM)                                                                           \
  hipLaunchKernelGGL(k_warp_img<FM>, dim3(tx * ty), dim3(256), 0, st, c->I0s[s], c->I1s[s],    \
                     c->U[uset][0], c->U[uset][1], lw, lh, P, tx, c->C[cbuf][0], c->C[cbuf][1], \
                     c->C[cbuf][2]);
      MATH_SWITCH(math, WARP_IMG)
#undef WARP_IMG
    } else {
      WarpRingArgs wa;
      wa.I0 = c->I0s[s];
      wa.I1 = c->I1s[s];
      wa.u1 = c->U[uset][0];
      wa.u2 = c->U[uset][1];
      wa.I1wx = c->C[cbuf][0];
      wa.I1wy = c->C[cbuf][1];
      wa.rho = c->C[cbuf][2];
      wa.W = lw;
      wa.H = lh;
      wa.P = P;
      wa.bands = (lw + 63) / 64;
      wa.seg_rows = c->roll_seg > 0 ? std::max(c->roll_seg, kRollMinSeg)
                                    : roll_segment(wa.bands, lh, 6, c->warp_ring_slots * fill_now() / 100);
      wa.waves = wa.bands * ((lh + wa.seg_rows - 1) / wa.seg_rows);
#define WARP_RING(FM) \
  hipLaunchKernelGGL((k_warp_ring<6, 2, FM>), dim3(wa.waves), dim3(128), 0, st, wa);
      MATH_SWITCH(math, WARP_RING)
#undef WARP_RING
    }
    // algorithmic: 40 B/px per warp; compulsory here ~28 B/px (I1 x 1 + 2M/64)
    prof_end(c, st, t0, 1, (double)lw * lh * 40.0, (double)lw * lh * 28.0);
    DIAG(c, st, "warp kernel", s, wp, -1);
    return TVL1_OK;
  };
  auto upsample = [&](int s, int uset) -> tvl1_status {  // level s -> s-1 into U[uset^1]
    const int lw = g.ws[s], lh = g.hs[s];
    const int dw = g.ws[s - 1], dh = g.hs[s - 1];
    const float fxu = (float)(1.0 / ((double)dw / lw));
    const float fyu = (float)(1.0 / ((double)dh / lh));
    size_t t0 = prof_begin(c, st);
    if (contracts(math))
      hipLaunchKernelGGL(k_upsample<true>, grid2(dw, dh, gam ? 3 : 2), kBlk2, 0, st, c->U[uset][0],
                         c->U[uset][1], c->U[uset][2], lw, lh, g.ps[s], c->U[uset ^ 1][0],
                         c->U[uset ^ 1][1], c->U[uset ^ 1][2], dw, dh, g.ps[s - 1], fxu, fyu, upmul);
    else
      hipLaunchKernelGGL(k_upsample<false>, grid2(dw, dh, gam ? 3 : 2), kBlk2, 0, st, c->U[uset][0],
                         c->U[uset][1], c->U[uset][2], lw, lh, g.ps[s], c->U[uset ^ 1][0],
                         c->U[uset ^ 1][1], c->U[uset ^ 1][2], dw, dh, g.ps[s - 1], fxu, fyu, upmul);
    prof_end(c, st, t0, 2, (double)lw * lh * 8.0 + (double)dw * dh * 8.0);
    DIAG(c, st, "k_upsample", s, -1, -1);
    return TVL1_OK;
  };
#define TRY(expr)                      \
  do {                                 \
    tvl1_status r_ = (expr);           \
    if (r_ != TVL1_OK) return r_;      \
  } while (0)

  double w0_hint = 50.0;   // speculation: residual / (eps^2 W H) at a level's first check
  for (int s = L - 1; s >= 0; --s) {
    const int lw = g.ws[s], lh = g.hs[s], P = g.ps[s];
    const double Nl = (double)lw * lh;
    const double scaledEps = prm.epsilon * prm.epsilon * (double)lw * (double)lh;
    bool p_zero = true;  // p = 0 at the start of every level (setTo(0) in procOneScale)

    IterArgs a{};
    a.W = lw;
    a.H = lh;
    a.P = P;
    a.segs = (lw + kSegPx - 1) / kSegPx;
    a.strip_rows = kStripRows;
    a.l_t = l_t;
    a.theta = theta_f;
    a.gamma = gamma_f;
    a.taut = taut;
    a.taut_small = taut_small(taut);
    a.partials = c->partials;
    const int nblk = iterate_blocks(lw, lh);
    // Pass kernels: 2-iteration passes (HBM-bound) stream through k_iterate_roll's x-only
    // halo; passes of >= 3 iterations are VALU-bound, where the streaming kernel wins only
    // while the level has enough rows for one round of >= 32-row segments (short segments
    // repeat the 2K-row halo) and k_iterate_tb (64 x 32 regions, 2 px/lane) wins below.
    // Planes beyond 32-bit buffer offsets take k_iterate_tb for every pass.
    const bool roll_ok = buffer_ok(s);
    const bool roll_long = roll_ok && (long)((lw + 55) / 56) * ((lh + 31) / 32) >= c->roll_long_min;

    // one iteration pass of k iterations (ending in a check if calc_end) from the buffer sets
    // (ui, pi) with the constants of set cb; witer: the warp's first pass as k_warp_iter
    // (storing the constants if store_c).  gate: a speculative launch
    auto launch_pass = [&](int k, bool calc_end, bool witer, bool store_c, int ui, int pi, int cb,
                           bool p_zero, const unsigned long long *gate, unsigned long long gseq,
                           int wp, int n, int &blocks_out, bool midp = false) -> tvl1_status {
        a.u1s = c->U[ui][0]; a.u2s = c->U[ui][1]; a.u3s = c->U[ui][2];
        a.u1d = c->U[ui ^ 1][0]; a.u2d = c->U[ui ^ 1][1]; a.u3d = c->U[ui ^ 1][2];
        a.p11s = c->Pd[pi][0]; a.p12s = c->Pd[pi][1]; a.p21s = c->Pd[pi][2];
        a.p22s = c->Pd[pi][3]; a.p31s = c->Pd[pi][4]; a.p32s = c->Pd[pi][5];
        a.p11d = c->Pd[pi ^ 1][0]; a.p12d = c->Pd[pi ^ 1][1]; a.p21d = c->Pd[pi ^ 1][2];
        a.p22d = c->Pd[pi ^ 1][3]; a.p31d = c->Pd[pi ^ 1][4]; a.p32d = c->Pd[pi ^ 1][5];
        a.calc_err = calc_end ? 1 : 0;
        a.p_zero = p_zero ? 1 : 0;
        a.I1wx = c->C[cb][0];
        a.I1wy = c->C[cb][1];
        a.rho = c->C[cb][2];
        a.gate = gate;
        a.gate_seq = gseq;
        int blocks = nblk;
        const size_t tkp = prof_begin(c, st);
        double hbm;
        const int nu = gam ? 3 : 2, np = gam ? 6 : 4;
        const double ld_planes = 3 + nu + (p_zero ? 0 : np), st_planes = nu + np;
        double alg_extra = 0.0;   // the fused warpBackward's algorithmic bytes
        if (witer) {
          WarpIterArgs w;
          w.ra.b = roll_bufs(s, ui, pi, cb);
          w.ra.it = a;
          w.ra.it.I1wx = c->C[cb][0];
          w.ra.it.I1wy = c->C[cb][1];
          w.ra.it.rho = c->C[cb][2];
          w.I0 = c->I0s[s];
          w.I1 = c->I1s[s];
          // the constants go to HBM only when the warp may run further passes: always for
          // a level's first warp, else when the previous warp did not stop at its first
          // check (a wrong guess recomputes them with the warp kernel after the check)
          w.store_c = store_c ? 1 : 0;
          constexpr int M = kWiMargin, BW = 128;
          w.ra.bands = (lw + BW - 5) / (BW - 4);
          const int seg = c->roll_seg > 0 ? std::max(c->roll_seg, kRollMinSeg)
                                          : roll_segment(w.ra.bands, lh, 2 + M, c->witer_slots * fill_now() / 100);
          w.ra.seg_rows = seg;
          const int segs = (lh + seg - 1) / seg;
          w.ra.waves = w.ra.bands * segs;
          blocks = w.ra.waves;
          if (blocks > c->partials_cap)
            return set_err(c, TVL1_EHIP, "internal: %d blocks > partials capacity %d", blocks,
                           c->partials_cap);
#define WITER(FM)                                                                           \
  if (c->wi_nc == 2)                                                                       \
    hipLaunchKernelGGL((k_warp_iter<M, FM, BW, 1, 2>), dim3(w.ra.waves), dim3(128 + BW),    \
                       c->probe_wi_lds, st, w);                                             \
  else                                                                                     \
    hipLaunchKernelGGL((k_warp_iter<M, FM, BW, 1, 1>), dim3(w.ra.waves), dim3(64 + BW), 0, st, w);
          MATH_SWITCH(math, WITER)
#undef WITER
          // compulsory: p, u, I0 and the I1 window (x 1 + 2M/BW) per band column and row;
          // u, p (+ the constants) stored
          double rows = 0.0;
          for (int sg = 0; sg < segs; ++sg) {
            const int ys = sg * seg, ye = std::min(ys + seg, lh);
            rows += std::min(ye - 1 + 2, lh - 1) - std::max(ys - 2, 0) + 1;
          }
          hbm = (double)w.ra.bands * BW * rows * 4.0 *
                    ((p_zero ? 3 : 7) + (double)wi_ww<M, BW>() / BW) +
                Nl * 4.0 * (6.0 + (w.store_c ? 3.0 : 0.0));
          alg_extra = Nl * 40.0;   // 40 B/px per warp
        } else if (exact_div) {   // taut < 0 or not finite: one iteration per launch, IEEE
          if (gam)
            hipLaunchKernelGGL((k_iterate<true, true>), dim3(nblk), dim3(kBlock), 0, st, a);
          else
            hipLaunchKernelGGL((k_iterate<false, true>), dim3(nblk), dim3(kBlock), 0, st, a);
          hbm = Nl * 4.0 * (ld_planes + st_planes) * k;
        } else if (roll_ok && (k <= 2 || roll_long)) {
          RollArgs ra;
          ra.b = roll_bufs(s, ui, pi, cb);
          ra.it = a;
          const int px = k <= 2 && (long)lw * lh >= c->roll_px4_min ? 4 : 2;
          const int halo = (k + px - 1) / px * px;   // roll_halo<K, PX>
          const int out_w = 64 * px - 2 * halo;
          ra.bands = (lw + out_w - 1) / out_w;
          const int slots = midp ? c->mid_slots : c->roll_slots[k][gam][px];
          const int seg = c->roll_seg > 0 ? std::max(c->roll_seg, kRollMinSeg)
                                           : roll_segment(ra.bands, lh, k, slots * fill_now() / 100);
          ra.seg_rows = seg;
          const int segs = (lh + seg - 1) / seg;
          ra.waves = ra.bands * segs;
          blocks = ra.waves;  // one residual partial per wavefront (two for the mid pass)
          if ((midp ? 2 : 1) * blocks > c->partials_cap)
            return set_err(c, TVL1_EHIP, "internal: %d wavefronts > partials capacity %d", blocks,
                           c->partials_cap);
          if (midp && (k != 4 || px != 2 || gam || !calc_end))
            return set_err(c, TVL1_EHIP, "internal: mid-check pass of k = %d, px = %d", k, px);
          const dim3 grid((ra.waves + 3) / 4);
#define ROLL_G(K, PX) \
  hipLaunchKernelGGL((k_iterate_roll<true, K, PX>), grid, dim3(256), 0, st, ra);
#define ROLL_M(FM, K, PX)                                                                  \
  if (c->probe_lds > 0)                                                                    \
    (void)hipFuncSetAttribute((const void *)k_iterate_roll<false, K, PX, FM>,              \
                              hipFuncAttributeMaxDynamicSharedMemorySize, c->probe_lds);   \
  hipLaunchKernelGGL((k_iterate_roll<false, K, PX, FM>), grid, dim3(256), c->probe_lds, st, ra);
#define ROLL(K, PX)                     \
  if (gam) {                            \
    ROLL_G(K, PX)                       \
  } else if (math == kFast) {           \
    ROLL_M(kFast, K, PX)                \
  } else if (math == kFma) {            \
    ROLL_M(kFma, K, PX)                 \
  } else {                              \
    ROLL_M(kIEEE, K, PX)                \
  }
#define MID_M(FM) hipLaunchKernelGGL((k_iterate_roll_mid<FM>), grid, dim3(256), 0, st, ra);
          if (midp) {
            MATH_SWITCH(math, MID_M)
          } else if (px == 4) {   // k <= 2
            if (k == 1) {
              ROLL(1, 4)
            } else {
              ROLL(2, 4)
            }
          } else {
            switch (k) {
              case 1: ROLL(1, 2) break;
              case 2: ROLL(2, 2) break;
              case 3: ROLL(3, 2) break;
              default: ROLL(4, 2) break;
            }
          }
#undef MID_M
#undef ROLL
#undef ROLL_M
#undef ROLL_G
          // compulsory: every band lane loads its column over the segment's rows + halo
          double rows = 0.0;
          for (int sg = 0; sg < segs; ++sg) {
            const int ys = sg * seg, ye = std::min(ys + seg, lh);
            rows += std::min(ye - 1 + k, lh - 1) - std::max(ys - k, 0) + 1;
          }
          hbm = (double)ra.bands * 64.0 * px * rows * 4.0 * ld_planes + Nl * 4.0 * st_planes;
        } else if (c->tb4 && !gam) {   // 64 x 48 regions, 3 rows x 2 px per thread
          TBArgs t;
          t.it = a;
          t.niter = k;
          t.tiles_x = (lw + 55) / 56;
          constexpr int nr = kTb4RowsPerThread;
          t.out_h = kTb4Groups * nr - 2 * k;
          blocks = t.tiles_x * ((lh + t.out_h - 1) / t.out_h);
          if (blocks > c->partials_cap)
            return set_err(c, TVL1_EHIP, "internal: %d blocks > partials capacity %d", blocks,
                           c->partials_cap);
#define TB4_M(FM) \
  hipLaunchKernelGGL((k_iterate_tb4<FM>), dim3(blocks), dim3(32 * kTb4Groups), 0, st, t);
          MATH_SWITCH(math, TB4_M)
#undef TB4_M
          hbm = (double)blocks * 64.0 * (kTb4Groups * nr) * 4.0 * ld_planes + Nl * 4.0 * st_planes;
        } else {   // 64 x 32 regions, 2 px per lane
          TBArgs t;
          t.it = a;
          t.niter = k;
          t.tiles_x = (lw + 55) / 56;
          constexpr int rh = 32;
          t.out_h = rh - 2 * k;
          blocks = t.tiles_x * ((lh + t.out_h - 1) / t.out_h);
          if (blocks > c->partials_cap)
            return set_err(c, TVL1_EHIP, "internal: %d blocks > partials capacity %d", blocks,
                           c->partials_cap);
#define TB(G, FM) \
  hipLaunchKernelGGL((k_iterate_tb<G, rh, 1, 2, FM>), dim3(blocks), dim3(32 * rh), 0, st, t);
#define TB_M(FM) TB(false, FM)
          if (gam) {
            TB(true, kIEEE)
          } else {
            MATH_SWITCH(math, TB_M)
          }
#undef TB_M
#undef TB
          // compulsory for this tiling: every staged region cell loads I1wx, I1wy, rho,
          // u (+p unless p == 0), every px stores u and p once per pass
          hbm = (double)blocks * 64.0 * rh * 4.0 * ld_planes + Nl * 4.0 * st_planes;
        }
        // algorithmic: 64 B/px per executed iteration (+ 40 B/px for a
        // fused warpBackward)
        prof_end(c, st, tkp, 0, Nl * 64.0 * k + alg_extra, hbm);
        DIAG(c, st, "iteration pass", s, wp, n);
        blocks_out = blocks;
        return TVL1_OK;
    };

    // warpBackward fused into the warp's first pass (2 iterations ending in the first
    // check) when that pass would stream through k_iterate_roll anyway
    const bool fuse = c->fuse && !gam && !exact_div && roll_ok && prm.epsilon > 0 &&
                      prm.iterations >= 2 && (long)lw * lh >= c->fuse_min;
    const int kmax = exact_div ? 1 : roll_ok ? kRollMax : kTbMax;
    // the mid-check pass (k_iterate_roll_mid) where a 4-iteration pass streams
    const bool mid_ok = !gam && !exact_div && roll_long && prm.epsilon > 0 && kRollMax >= 4;
    // Speculation: behind each residual check the host enqueues the launch it
    // expects to follow, gated on the device by the check's own evaluation of the stopping
    // rule, and only then waits for the residual.  A right guess hides the host round trip;
    // a wrong one costs an empty launch, and the host enqueues the right work as before.
    const bool spec_ok = c->spec && !exact_div && roll_ok && prm.epsilon > 0;
    const bool spec_stop_ok = spec_ok && !median && prm.iterations >= 2;
    // Guesses.  A warp's residual (in units of eps^2 W H) after its first check falls steadily,
    // so: the action the level's previous warp took at the same iteration count; else the
    // next residual extrapolated from the last two (the check after a long run of unchecked
    // iterations comes where the schedule's linear model crosses 1: guess a stop); a level's
    // first warp starts where the previous level's did.
    struct Hist {
      double r0 = -1.0, r1 = -1.0;   // the warp's last two residuals / (eps^2 W H); < 0: none
      int n0 = -1, n_last = -1;      // iteration counts at those checks
    };
    // the residual expected at the check after one at n (the warp's history up to that check)
    auto extrapolate = [&](const Hist &h, int n, int wp) {
      if (h.r1 < 0) return wp == 0 ? w0_hint : 1.5;
      if (n - h.n_last > 2) return 0.9;   // a long unchecked run ends near the model's crossing
      if (h.r0 >= 0 && h.n_last - h.n0 == 2) return h.r1 * (h.r1 / h.r0);   // steady decay
      return h.n_last == 2 ? h.r1 * 0.6 : h.r1 * 0.93;   // after a warp's first check: a drop
    };
    // (remembered up to 4096 iterations: a huge `iterations` must not size a huge table)
    const size_t nact = (size_t)std::min(prm.iterations, 4096) + 1;
    std::vector<int> act_prev(nact, -2), act_cur(nact, -2);
    auto act_of = [&](double e, int n) {   // 0: stop, else k << 1 | calc_end
      if (!(e > scaledEps && n < prm.iterations)) return 0;
      bool ce;
      double pe;
      return sched_after(e, scaledEps, n, prm.iterations, kmax, 1, &ce, &pe) << 1 | (ce ? 1 : 0);
    };
    // what to predict after a check at iteration count n of warp wp: pk = 0 the warp stops
    // (its successor's first pass follows), pk > 0 it continues with (pk, pcalc), -1 nothing
    auto predict0 = [&](int wp, int n, bool nostore, int last_n, const Hist &h,
                        const std::vector<int> *prevw, int &pk, int &pcalc) {
      pk = -1;
      pcalc = 0;
      if (!spec_ok) return;
      if (c->spec == 1 && g_solving[c->device & 63].load(std::memory_order_relaxed) > 1) return;
      const bool can_stop = spec_stop_ok && wp + 1 < prm.warps;
      const bool can_cont = !nostore && n < prm.iterations;
      if (can_stop && (n >= prm.iterations || (n == 2 && last_n == 2))) {
        pk = 0;
        return;
      }
      const int ap = prevw && wp >= 2 && n < (int)prevw->size() ? (*prevw)[n] : -2;
      if (ap == 0 && can_stop) {
        pk = 0;
        return;
      }
      if (ap > 0 && can_cont) {
        pk = ap >> 1;
        pcalc = ap & 1;
        return;
      }
      const double r = extrapolate(h, n, wp);
      if (r <= 1.0 && can_stop) {
        pk = 0;
      } else if (can_cont) {
        const int a = act_of(std::max(r, 1.0 + 1e-9) * scaledEps, n);
        pk = a >> 1;
        pcalc = a & 1;
      } else if (can_stop) {
        pk = 0;
      }
    };
    // a predicted 2-iteration continuation after a warp's first check is left to the host,
    // which may run it as a mid-check pass (less GPU work than the pass enqueued ahead)
    auto predict = [&](int wp, int n, bool nostore, int last_n, const Hist &h,
                       const std::vector<int> *prevw, int &pk, int &pcalc) {
      predict0(wp, n, nostore, last_n, h, prevw, pk, pcalc);
      if (c->mid && mid_ok && pk == 2 && pcalc && n > 2) pk = -1;
    };
    auto gate_of = [&](int wp, int n, int pk, int pcalc, unsigned long long gin_seq, bool gated) {
      CheckGate gt{};
      if (gated) {
        gt.in = c->gate;
        gt.in_seq = gin_seq;
      }
      if (pk >= 0) {
        gt.out = c->gate;
        gt.thr = scaledEps;
        gt.n = n;
        gt.iters = prm.iterations;
        gt.kmax = kmax;
        gt.eps_pos = 1;
        gt.pk = pk;
        gt.pcalc = pcalc;
      }
      (void)wp;
      return gt;
    };

    int last_warp_n = -1;   // iterations of the level's previous warp
    // a warp whose first pass (and check) the previous warp enqueued speculatively
    bool pre = false;
    bool pre_nostore = false;
    unsigned long long pre_seq = 0;
    int pre_pk = -1, pre_pcalc = 0;
    for (int wp = 0; wp < prm.warps; ++wp) {
      bool fused_nostore = false;   // k_warp_iter ran without storing the constants
      double error = DBL_MAX;
      double prevError = 0.0;
      int n = 0;
      // a check enqueued but not yet read: its sequence number and prediction
      bool pending = false;
      unsigned long long pend_seq = 0;
      int pend_pk = -1, pend_pcalc = 0;
      Hist h;
      if (pre) {
        n = 2;
        fused_nostore = pre_nostore;
        pending = true;
        pend_seq = pre_seq;
        pend_pk = pre_pk;
        pend_pcalc = pre_pcalc;
        pre = false;
      } else {
        if (median) {
          hipLaunchKernelGGL(k_median, grid2(lw, lh, 2), kBlk2, 0, st, c->U[ui][0], c->U[ui][1],
                             lw, lh, P, prm.median_filtering, c->U[ui ^ 1][0], c->U[ui ^ 1][1]);
          if (gam) {
            const size_t n = (size_t)P * lh * sizeof(float);
            HIP_TRY(c, hipMemcpyAsync(c->U[ui ^ 1][2], c->U[ui][2], n, hipMemcpyDeviceToDevice, st));
          }
          ui ^= 1;
        }
        if (!fuse) TRY(gather(s, ui, cb, wp));
      }
      a.I1wx = c->C[cb][0];
      a.I1wy = c->C[cb][1];
      a.rho = c->C[cb][2];
      bool next_pre = false;   // this warp stopped where predicted: the next warp has begun
      while (pending || (error > scaledEps && n < prm.iterations)) {
        if (!pending) {
          bool calc_end = false;
          double prev_sim = prevError;
          const int k = sched_after(prevError, scaledEps, n, prm.iterations, kmax,
                                    prm.epsilon > 0, &calc_end, &prev_sim);
          // A converging warp (a check every second iteration, the error just above eps^2 W H)
          // runs its next two 2-iteration passes as one k_iterate_roll_mid pass: both checks'
          // residuals and the state after 4 iterations in the usual set.  The host reads the
          // first check as procOneScale does; if the warp stops there (or its schedule is not
          // a second 2-iteration pass) a 2-iteration pass from the same input set, which the
          // mid-check pass leaves as it was, recomputes the state at that check (DESIGN.md
          // §4.1 of r6).  Not for a warp's first check (n = 2: its error drops the
          // most), nor where the 4-iteration pass does not stream.
          if (c->mid && mid_ok && k == 2 && calc_end && n > 2 && n + 4 <= prm.iterations &&
              prevError >= c->mid_min * scaledEps) {
            int blocks = 0;
            TRY(launch_pass(4, true, false, false, ui, pi, cb, p_zero, nullptr, 0, wp, n, blocks, true));
            unsigned long long seq_mid = 0, seq_end = 0;
            TRY(launch_check(c, st, blocks, CheckGate{}, &seq_mid, blocks));
            TRY(launch_check(c, st, blocks, CheckGate{}, &seq_end));
            auto note = [&](double e, int nn) {   // the bookkeeping of a check read below
              ++checks;
              h.r0 = h.r1;
              h.n0 = h.n_last;
              h.r1 = e / scaledEps;
              h.n_last = nn;
              if ((size_t)nn < nact) act_cur[nn] = act_of(e, nn);
            };
            double e_mid = 0.0;
            TRY(wait_check(c, st, seq_mid, &e_mid));
            n += 2;
            note(e_mid, n);
            ++mid_passes;
            bool ce2 = false;
            double prev2 = 0.0;
            const bool stop = !(e_mid > scaledEps && n < prm.iterations);
            if (!stop &&
                sched_after(e_mid, scaledEps, n, prm.iterations, kmax, 1, &ce2, &prev2) == 2 && ce2) {
              double e_end = 0.0;   // the second check: the next pass's own
              TRY(wait_check(c, st, seq_end, &e_end));
              n += 2;
              note(e_end, n);
              error = e_end;
              prevError = e_end;
            } else {   // the state at the first check: its 2 iterations again, no residual
              ++mid_taken;
              TRY(launch_pass(2, false, false, false, ui, pi, cb, false, nullptr, 0, wp, n - 2, blocks));
              error = e_mid;
              prevError = e_mid;
            }
            p_zero = false;
            ui ^= 1;
            pi ^= 1;
            continue;
          }
          const bool witer = fuse && n == 0 && k == 2 && calc_end;
          // the constants go to HBM only when the warp may run further passes: always for
          // a level's first warp, else when the previous warp did not stop at its first
          // check (a wrong guess recomputes them with the warp kernel after the check)
          const bool store_c = wp == 0 || last_warp_n != 2;
          int blocks = 0;
          TRY(launch_pass(k, calc_end, witer, store_c, ui, pi, cb, p_zero, nullptr, 0, wp, n, blocks));
          if (witer) fused_nostore = !store_c;
          p_zero = false;
          ui ^= 1;
          pi ^= 1;
          n += k;
          if (!calc_end) {
            error = DBL_MAX;
            prevError = prev_sim;
            continue;
          }
          predict(wp, n, fused_nostore, last_warp_n, h, &act_prev, pend_pk, pend_pcalc);
          TRY(launch_check(c, st, blocks, gate_of(wp, n, pend_pk, pend_pcalc, 0, false), &pend_seq));
        }
        pending = false;
        // the predicted launch(es) behind the check, gated on it
        const int sp_pk = pend_pk, sp_pcalc = pend_pcalc;
        const size_t marks0 = c->marks.size(), ev0 = c->ev_used;
        const unsigned long long seq0 = c->check_seq;
        unsigned long long sp_seq = 0;   // the speculative launch's own check
        int sp_pk2 = -1, sp_pcalc2 = 0;
        bool sp_nostore = false;
        if (sp_pk == 0) {   // the next warp's first pass and check
          const int w2 = wp + 1, cb2 = cb ^ 1;
          const bool store2 = n != 2;   // k_warp_iter's store rule, if this warp stops here
          int blocks = 0;
          // the gather is not gated (a gate check costs k_warp_ring 34 VGPRs): after a wrong
          // guess it has only filled the constants set the next warp recomputes anyway
          if (!fuse) TRY(gather(s, ui, cb2, w2));
          TRY(launch_pass(2, true, fuse, store2, ui, pi, cb2, false, c->gate, pend_seq, w2, 0, blocks));
          sp_nostore = fuse && !store2;
          if ((size_t)n < nact) act_cur[n] = 0;   // (as guessed; recorded after the read)
          predict(w2, 2, sp_nostore, n, Hist{}, &act_cur, sp_pk2, sp_pcalc2);
          TRY(launch_check(c, st, blocks, gate_of(w2, 2, sp_pk2, sp_pcalc2, pend_seq, true), &sp_seq));
        } else if (sp_pk > 0) {   // this warp's next pass
          int blocks = 0;
          TRY(launch_pass(sp_pk, sp_pcalc != 0, false, false, ui, pi, cb, false, c->gate, pend_seq,
                          wp, n, blocks));
          if (sp_pcalc) {
            Hist h2;   // with check j's residual extrapolated
            h2.r0 = h.r1;
            h2.n0 = h.n_last;
            h2.r1 = h.r1 < 0 ? -1.0 : extrapolate(h, n, wp);
            h2.n_last = n;
            predict(wp, n + sp_pk, false, last_warp_n, h2, &act_prev, sp_pk2, sp_pcalc2);
            TRY(launch_check(c, st, blocks, gate_of(wp, n + sp_pk, sp_pk2, sp_pcalc2, pend_seq, true),
                             &sp_seq));
          }
        }
        TRY(wait_check(c, st, pend_seq, &error));   // the cuda::sum -> host read
        prevError = error;
        ++checks;
        const bool ends = !(error > scaledEps && n < prm.iterations);
        if (wp == 0 && h.r1 < 0) w0_hint = error / scaledEps;
        h.r0 = h.r1;
        h.n0 = h.n_last;
        h.r1 = error / scaledEps;
        h.n_last = n;
        if ((size_t)n < nact) act_cur[n] = act_of(error, n);
        bool right = false;
        double sp_prev = 0.0;
        if (sp_pk == 0) {
          right = ends;
        } else if (sp_pk > 0 && !ends) {
          bool ce;
          right = sched_after(error, scaledEps, n, prm.iterations, kmax, 1, &ce, &sp_prev) == sp_pk &&
                  (int)ce == sp_pcalc;
        }
        if (c->spec_trace)
          fprintf(stderr, "spec level %d warp %d n %d E/thr %.3f guess %d/%d %s\n", s, wp, n,
                  error / scaledEps, sp_pk, sp_pcalc, sp_pk < 0 ? "-" : right ? "hit" : "miss");
        if (sp_pk >= 0 && !right) {   // the gated launches ran empty: forget them
          ++spec_misses;
          c->marks.resize(marks0);
          c->ev_used = ev0;
          c->check_seq = seq0;
        }
        if (right && sp_pk == 0) {   // the next warp's first pass is done, its check pending
          ui ^= 1;
          pi ^= 1;
          p_zero = false;
          next_pre = true;
          pre_nostore = sp_nostore;
          pre_seq = sp_seq;
          pre_pk = sp_pk2;
          pre_pcalc = sp_pcalc2;
          break;
        }
        if (right) {   // the warp's next pass is done
          p_zero = false;
          ui ^= 1;
          pi ^= 1;
          n += sp_pk;
          if (sp_pcalc) {
            pending = true;
            pend_seq = sp_seq;
            pend_pk = sp_pk2;
            pend_pcalc = sp_pcalc2;
          } else {
            error = DBL_MAX;
            prevError = sp_prev;
          }
          continue;
        }
        // k_warp_iter guessed that this warp stops here; it continues: compute its
        // constants (from its input u, the set the pass just read) before the next pass
        if (fused_nostore && !ends) TRY(gather(s, ui ^ 1, cb, wp));
        fused_nostore = false;
      }
      level_iters[s] += n;
      last_warp_n = n;
      if (stats && stats->warp_iterations && s * prm.warps + wp < stats->warp_iterations_capacity)
        stats->warp_iterations[s * prm.warps + wp] = n;
      cb ^= 1;  // every warp gets the other constants buffer
      pre = next_pre;
      act_prev.swap(act_cur);
      std::fill(act_cur.begin(), act_cur.end(), -2);
    }
    HIP_TRY(c, hipGetLastError());
    if (s == 0) break;
    TRY(upsample(s, ui));  // zoom the flow to level s-1, scale by 1/scaleStep
    ui ^= 1;
  }
#undef TRY
  tk = prof_begin(c, st);
  hipLaunchKernelGGL(k_output, grid2(W, H), kBlk2, 0, st, c->U[ui][0], c->U[ui][1], W, H,
                     g.ps[0], u, v, fpitch);
  prof_end(c, st, tk, 2, (double)W * H * 16.0);
  HIP_TRY(c, hipGetLastError());

  if (stats) {
    for (int k = 0; k < 4; ++k) {
      stats->kernel_ms[k] = 0.0;
      stats->kernel_launches[k] = 0;
      stats->kernel_bytes[k] = 0.0;
      stats->kernel_hbm_bytes[k] = 0.0;
    }
  }
  if (c->profiling && !c->marks.empty()) {
    HIP_TRY(c, hipEventSynchronize(c->ev_pool[c->marks.back().b]));
    for (const auto &m : c->marks) {
      float ms = 0.f;
      HIP_TRY(c, hipEventElapsedTime(&ms, c->ev_pool[m.a], c->ev_pool[m.b]));
      if (stats) {
        stats->kernel_ms[m.cls] += ms;
        stats->kernel_launches[m.cls] += 1;
        stats->kernel_bytes[m.cls] += m.bytes;
        stats->kernel_hbm_bytes[m.cls] += m.hbm_bytes;
      }
    }
  }

  if (stats) {
    stats->levels = L;
    int64_t tot = 0;
    for (int s = 0; s < TVL1_MAX_LEVELS; ++s) {
      stats->level_width[s] = s < L ? g.ws[s] : 0;
      stats->level_height[s] = s < L ? g.hs[s] : 0;
      stats->level_iterations[s] = s < L ? level_iters[s] : 0;
      tot += s < L ? level_iters[s] : 0;
    }
    stats->iterations_total = tot;
    stats->checks_total = checks;
    stats->speculation_misses = spec_misses;
    stats->algorithmic_bytes = survey_bytes(g, prm.warps, level_iters);
  }
  if (c->spec_trace && mid_passes)
    fprintf(stderr, "mid-check passes %d, ended on the mid state %d\n", mid_passes, mid_taken);
  return TVL1_OK;
}


// ---------------------------------------------------------------- batched solve
// tvl1_calc_batch: n pairs of one size through the batched kernels (tvl1_batch.hpp), in
// chunks of kBatchMax.  The pairs of a chunk walk the levels and warps in lock step; inside
// a warp each pair keeps its own iteration count, stopping-rule state and u / p buffer set,
// and a pass runs the smallest number of iterations any active pair may fuse before its
// next check (<= kTbMax), so every pair sees exactly the single-pair schedule.
static tvl1_status ensure_batch(tvl1_ctx *c, int W, int H, int n, hipStream_t st) {
  const Geometry &g = c->geo;   // pyramid sizes of (W, H) (ensure_geometry ran)
  // reuse only for the same level sizes: a new scaleStep with the same level count changes
  // every level's plane stride (c->bips), and the kernels would write past each pair's slot
  if (c->barena && c->bW == W && c->bH == H && c->bL == g.L && c->bn >= n &&
      !memcmp(c->bws, g.ws, sizeof(int) * g.L) && !memcmp(c->bhs, g.hs, sizeof(int) * g.L))
    return TVL1_OK;
  const size_t P0 = (size_t)g.ps[0];
  const size_t ps = align_up(P0 * H, 64);
  // residual partials per pair: blocked regions (56 x 24 px) or rolling / fused waves
  // (>= 56-px bands x >= 8-row segments)
  const int tb_blocks = std::max(((W + 55) / 56) * ((H + 23) / 24), ((W + 55) / 56) * ((H + 7) / 8)) + 64;
  size_t bytes = 0;
  size_t ips[TVL1_MAX_LEVELS];
  for (int s = 0; s < g.L; ++s) {
    ips[s] = align_up((size_t)g.ps[s] * g.hs[s], 64);
    bytes += 2 * ips[s] * n * sizeof(float) + 512;
  }
  bytes += (ps * n * sizeof(float) + 256) * (4 + 8 + 3);   // U + P + C
  bytes += (size_t)tb_blocks * n * sizeof(double) + 4096;
  c->bW = c->bH = c->bL = c->bn = 0;
  // a layout that fits re-lays the existing arena (stream-ordered like ensure_geometry's):
  // only growth allocates, so alternating batch geometries hold one arena
  if (bytes > c->barena_bytes) {
    const tvl1_status r = arena_alloc(c, &c->barena, &c->barena_bytes, bytes, st);
    if (r != TVL1_OK) return r;   // TVL1_ENOMEM: the caller retries a smaller chunk
  }
  char *p = c->barena;
  auto take = [&](size_t nbytes) {
    char *r = p;
    p += align_up(nbytes, 256);
    return r;
  };
  for (int s = 0; s < TVL1_MAX_LEVELS; ++s) c->bI0s[s] = c->bI1s[s] = nullptr;
  for (int s = 0; s < g.L; ++s) {
    c->bips[s] = ips[s];
    c->bI0s[s] = (float *)take(ips[s] * n * sizeof(float));
    c->bI1s[s] = (float *)take(ips[s] * n * sizeof(float));
  }
  c->bps = ps;
  for (int k = 0; k < 2; ++k)
    for (int j = 0; j < 2; ++j) c->bU[k][j] = (float *)take(ps * n * sizeof(float));
  for (int k = 0; k < 2; ++k)
    for (int j = 0; j < 4; ++j) c->bP[k][j] = (float *)take(ps * n * sizeof(float));
  for (int j = 0; j < 3; ++j) c->bC[j] = (float *)take(ps * n * sizeof(float));
  c->bpartials = (double *)take((size_t)tb_blocks * n * sizeof(double));
  c->bnblk = tb_blocks;
  c->bW = W;
  c->bH = H;
  c->bL = g.L;
  c->bn = n;
  memcpy(c->bws, g.ws, sizeof(int) * g.L);
  memcpy(c->bhs, g.hs, sizeof(int) * g.L);
  return TVL1_OK;
}

static tvl1_status solve_batch_chunk(tvl1_ctx *c, int n, const uint8_t *I0, size_t pitch0,
                                     size_t stride0, const uint8_t *I1, size_t pitch1,
                                     size_t stride1, int W, int H, float *u, float *v,
                                     size_t fpitch, size_t fstride, tvl1_stats *stats,
                                     hipStream_t st) {
  const tvl1_params &prm = c->prm;
  const Geometry &g = c->geo;
  const int L = g.L;
  {
    const tvl1_status r = ensure_batch(c, W, H, n, st);
    if (r != TVL1_OK) return r;
  }
  const size_t ps = c->bps;
  // counted as a solve in progress (single-pair solves speculate and size their launches
  // by this count); the batched launches themselves are sized for every resident slot (the
  // shared share measured neutral here: 2925 / 2901 against 2919 / 2928 strip solves/s,
  // profiles/r3/ab_batch_fill.txt)
  const SolveCount active(c->device);
  BatchSel all{};
  all.n = n;
  for (int b = 0; b < n; ++b) all.idx[b] = (uint8_t)b;
  if (c->profiling) {   // per-class HIP events of this chunk's launches (shared by its pairs)
    c->ev_used = 0;
    c->marks.clear();
  }

  // [A.1] convertTo + [A.2] pyramid
  hipLaunchKernelGGL(kb_convert, grid2(W, H, 2 * n), kBlk2, 0, st, I0, pitch0, stride0, I1,
                     pitch1, stride1, c->bI0s[0], c->bI1s[0], W, H, g.ps[0], c->bips[0]);
  const float fdown = (float)(1.0 / prm.scale_step);
  const int math = math_of(prm);
  for (int s = 1; s < L; ++s) {
#define KB_DOWN(C)                                                                             \
  hipLaunchKernelGGL(kb_resize_down2<C>, grid2(g.ws[s], g.hs[s], 2 * n), kBlk2, 0, st,         \
                     c->bI0s[s - 1], c->bI1s[s - 1], g.ws[s - 1], g.hs[s - 1], g.ps[s - 1],    \
                     c->bips[s - 1], c->bI0s[s], c->bI1s[s], g.ws[s], g.hs[s], g.ps[s],       \
                     c->bips[s], fdown, fdown);
    if (contracts(math)) {
      KB_DOWN(true)
    } else {
      KB_DOWN(false)
    }
#undef KB_DOWN
  }
  // u = 0 at the coarsest level, set 0 of every pair
  for (int k = 0; k < 2; ++k)
    HIP_TRY(c, hipMemsetAsync(c->bU[0][k], 0, ps * n * sizeof(float), st));
  HIP_TRY(c, hipGetLastError());

  const float l_t = (float)(prm.lambda * prm.theta);
  const float taut = (float)(prm.tau / prm.theta);
  const float upmul = (float)(1.0 / prm.scale_step);
  BatchMask ubit{}, pbit{};
  std::vector<int64_t> level_iters((size_t)n * TVL1_MAX_LEVELS, 0), checks(n, 0), regathers(n, 0);
  std::vector<int> nit(n);
  std::vector<double> err(n), prev(n);
  std::vector<char> act(n);
  // per pair: its previous warp on this level stopped at the first check, so this warp's
  // fused pass is predicted to stop there too and its constants are not stored (k_warp_iter's
  // store_c rule)
  std::vector<char> stopped_first(n, 0);
  for (int s = L - 1; s >= 0; --s) {
    const int lw = g.ws[s], lh = g.hs[s], P = g.ps[s];
    const double scaledEps = prm.epsilon * prm.epsilon * (double)lw * (double)lh;
    BatchMask pzero{};   // p = 0 at every level start
    for (int b = 0; b < n; ++b) pzero.set(b);
    // RollBufs geometry of the batch arena (the kernels point it at each pair's planes)
    RollBufs batch_bufs{};
    {
      const size_t bstride = (size_t)(c->bC[1] - c->bC[0]) * sizeof(float);
      const size_t lvl = (size_t)P * lh * sizeof(float);
      batch_bufs.pstride = (unsigned)bstride;
      batch_bufs.cb = (unsigned)(2 * bstride + lvl);
      batch_bufs.ub = (unsigned)(bstride + lvl);
      batch_bufs.pb = (unsigned)(3 * bstride + lvl);
    }
    IterArgs it{};   // pass geometry and scalars (plane pointers are set per pair)
    it.W = lw;
    it.H = lh;
    it.P = P;
    it.l_t = l_t;
    it.theta = (float)prm.theta;
    it.gamma = 0.0f;
    it.taut = taut;
    it.taut_small = taut_small(taut);
    // The coarsest level on chip (kb_small_level, one workgroup per pair: every warp's gather,
    // iterations, residuals and stopping rule without leaving the workgroup) when it fits one
    // workgroup's registers and LDS; u enters as 0 in set 0 and leaves there, and p is reset
    // at every level anyway
    const bool small = c->batch_small && s == L - 1 && prm.median_filtering <= 1 &&
                       lw <= 64 * kSmallWaves && lh <= kSmallR && lw * lh <= kSmallPx;
    if (small) {
      const size_t need = (size_t)n * (prm.warps + 1) * sizeof(int);
      if (need > c->small_bytes) {
        const tvl1_status r = arena_alloc(c, &c->small_scratch, &c->small_bytes,
                                          std::max<size_t>(need, 64 << 10), st);
        if (r != TVL1_OK) return r;
      }
      BatchSmall sm{};
      sm.I0 = c->bI0s[s];
      sm.I1 = c->bI1s[s];
      sm.u1 = c->bU[0][0];
      sm.u2 = c->bU[0][1];
      sm.ips = c->bips[s];
      sm.ps = ps;
      sm.W = lw;
      sm.H = lh;
      sm.P = P;
      sm.warps = prm.warps;
      sm.iterations = prm.iterations;
      sm.eps_pos = prm.epsilon > 0;
      sm.thr = scaledEps;
      sm.it = it;
      sm.warp_iters = reinterpret_cast<int *>(c->small_scratch);
      sm.checks = sm.warp_iters + (size_t)n * prm.warps;
      sm.sel = all;
      const size_t tks = prof_begin(c, st);
#define KB_SMALL(FM) \
  hipLaunchKernelGGL((kb_small_level<FM>), dim3(n), dim3(64 * ((lw + 63) / 64)), 0, st, sm);
      MATH_SWITCH(math, KB_SMALL)
#undef KB_SMALL
      HIP_TRY(c, hipGetLastError());
      std::vector<int> hw((size_t)n * (prm.warps + 1));
      HIP_TRY(c, hipMemcpyAsync(hw.data(), c->small_scratch, need, hipMemcpyDeviceToHost, st));
      HIP_TRY(c, hipStreamSynchronize(st));
      int64_t it_sum = 0;
      for (int b = 0; b < n; ++b) {
        for (int wp = 0; wp < prm.warps; ++wp) {
          const int nb = hw[(size_t)b * prm.warps + wp];
          level_iters[(size_t)b * TVL1_MAX_LEVELS + s] += nb;
          it_sum += nb;
          if (stats && stats[b].warp_iterations &&
              s * prm.warps + wp < stats[b].warp_iterations_capacity)
            stats[b].warp_iterations[s * prm.warps + wp] = nb;
        }
        checks[b] += hw[(size_t)n * prm.warps + b];
      }
      // its own class (3): SURVEY 8(d)'s bytes of every iteration and warp it ran, but from HBM
      // it only reads I0, I1 and writes u once, so it would skew class 0's HBM roofline
      prof_end(c, st, tks, 3, (double)lw * lh * (64.0 * it_sum + 40.0 * n * prm.warps),
               (double)lw * lh * 16.0 * n);
    }
    for (int wp = 0; wp < (small ? 0 : prm.warps); ++wp) {
      if (prm.median_filtering > 1) {   // build-only median of u before each warp
        BatchMedian md{};
        for (int k = 0; k < 2; ++k)
          for (int j = 0; j < 2; ++j) md.U[k][j] = c->bU[k][j];
        md.ps = ps;
        md.W = lw;
        md.H = lh;
        md.P = P;
        md.ksize = prm.median_filtering;
        md.sel = all;
        md.sel.ubit = ubit;
        hipLaunchKernelGGL(kb_median, grid2(lw, lh, 2 * n), kBlk2, 0, st, md);
        for (int b = 0; b < n; ++b) ubit.flip(b);
      }
      // warpBackward fused with the warp's first pass, which is 2 iterations ending in the
      // first check for every pair (procOneScale with epsilon > 0, iterations >= 2)
      const bool fuse = c->batch_fuse && prm.epsilon > 0 && prm.iterations >= 2;
      if (fuse) {
        BatchWI wi{};
        wi.w.ra.b = batch_bufs;
        wi.w.ra.it = it;
        wi.w.ra.bands = (lw + 123) / 124;
        wi.w.ra.seg_rows = roll_segment(wi.w.ra.bands * n, lh, 2 + 6, c->witer_slots);
        wi.w.ra.waves = wi.w.ra.bands * ((lh + wi.w.ra.seg_rows - 1) / wi.w.ra.seg_rows);
        if (wi.w.ra.waves > c->bnblk)
          return set_err(c, TVL1_EHIP, "internal: %d blocks > batch partials %d", wi.w.ra.waves, c->bnblk);
        wi.I0 = c->bI0s[s];
        wi.I1 = c->bI1s[s];
        for (int k = 0; k < 2; ++k)
          for (int j = 0; j < 2; ++j) wi.U[k][j] = c->bU[k][j];
        for (int k = 0; k < 2; ++k)
          for (int j = 0; j < 4; ++j) wi.Pp[k][j] = c->bP[k][j];
        for (int j = 0; j < 3; ++j) wi.C[j] = c->bC[j];
        wi.ips = c->bips[s];
        wi.ps = ps;
        wi.partials = c->bpartials;
        wi.nblk = wi.w.ra.waves;
        wi.sel = all;
        wi.sel.ubit = ubit;
        wi.sel.pbit = pbit;
        wi.sel.pzero = pzero;
        int nstore = 0;
        for (int b = 0; b < n; ++b)
          if (wp == 0 || !stopped_first[b] || !c->batch_store_pred) {
            wi.sel.storec.set(b);
            ++nstore;
          }
        const size_t tkw = prof_begin(c, st);
#define KB_WITER(FM)                                                                             \
  if (c->wi_nc == 2)                                                                            \
    hipLaunchKernelGGL((kb_warp_iter<6, FM, 2>), dim3(wi.w.ra.waves, n), dim3(256), 0, st, wi); \
  else                                                                                          \
    hipLaunchKernelGGL((kb_warp_iter<6, FM, 1>), dim3(wi.w.ra.waves, n), dim3(192), 0, st, wi);
        MATH_SWITCH(math, KB_WITER)
#undef KB_WITER
        if (tkw) {   // k_warp_iter's accounting per pair (constants always stored), x n
          const int seg = wi.w.ra.seg_rows, segs = (lh + seg - 1) / seg;
          double rows = 0.0;
          for (int sg = 0; sg < segs; ++sg) {
            const int ys = sg * seg, ye = std::min(ys + seg, lh);
            rows += std::min(ye - 1 + 2, lh - 1) - std::max(ys - 2, 0) + 1;
          }
          const double Nl = (double)lw * lh;
          int nz = 0;   // pairs whose p is zero (a level's first warp): p not loaded
          for (int b = 0; b < n; ++b) nz += pzero.test(b) ? 1 : 0;
          const double band_bytes = (double)wi.w.ra.bands * 128 * rows * 4.0;
          const double hbm = band_bytes * ((double)nz * 3 + (double)(n - nz) * 7 +
                                           (double)n * wi_ww<6, 128>() / 128) +
                             Nl * 4.0 * (6.0 * n + 3.0 * nstore);
          prof_end(c, st, tkw, 0, (double)n * Nl * (64.0 * 2 + 40.0), hbm);
        }
        hipLaunchKernelGGL(kb_reduce, dim3(n), dim3(kBlock), 0, st, c->bpartials,
                           (size_t)wi.w.ra.waves, wi.w.ra.waves, all, c->pinned_dev + 8);
        HIP_TRY(c, hipEventRecord(c->ev_check[0], st));
      } else {   // k_warp_ring's streaming LDS-ring gather, per pair
        BatchRing br{};
        br.wa.W = lw;
        br.wa.H = lh;
        br.wa.P = P;
        br.wa.bands = (lw + 63) / 64;
        br.wa.seg_rows = roll_segment(br.wa.bands * n, lh, 6, c->warp_ring_slots);
        br.wa.waves = br.wa.bands * ((lh + br.wa.seg_rows - 1) / br.wa.seg_rows);
        br.I0 = c->bI0s[s];
        br.I1 = c->bI1s[s];
        for (int k = 0; k < 2; ++k)
          for (int j = 0; j < 2; ++j) br.U[k][j] = c->bU[k][j];
        for (int j = 0; j < 3; ++j) br.C[j] = c->bC[j];
        br.ips = c->bips[s];
        br.ps = ps;
        br.sel = all;
        br.sel.ubit = ubit;
        const size_t tkr = prof_begin(c, st);
#define KB_RING(FM) \
  hipLaunchKernelGGL((kb_warp_ring<6, 2, FM>), dim3(br.wa.waves, n), dim3(128), 0, st, br);
        MATH_SWITCH(math, KB_RING)
#undef KB_RING
        prof_end(c, st, tkr, 1, (double)n * lw * lh * 40.0, (double)n * lw * lh * 28.0);
      }
      int nact = 0;
      for (int b = 0; b < n; ++b) {
        nit[b] = 0;
        err[b] = DBL_MAX;
        prev[b] = 0.0;
        act[b] = prm.iterations > 0;
        nact += act[b];
      }
      if (fuse) {   // the fused first pass: n = 0 (no check), n = 1 (check)
        HIP_TRY(c, hipEventSynchronize(c->ev_check[0]));
        nact = 0;
        BatchSel regather{};   // pairs that continue without stored constants
        regather.ubit = ubit;  // u^0: the set the fused pass read
        for (int b = 0; b < n; ++b) {
          const bool stored = wp == 0 || !stopped_first[b] || !c->batch_store_pred;
          nit[b] = 2;
          ubit.flip(b);
          pbit.flip(b);
          pzero.clear(b);
          err[b] = c->pinned[8 + b];
          prev[b] = err[b];
          ++checks[b];
          act[b] = err[b] > scaledEps && nit[b] < prm.iterations;
          nact += act[b];
          stopped_first[b] = !act[b];
          if (act[b] && !stored) regather.idx[regather.n++] = (uint8_t)b;
        }
        if (regather.n > 0) {   // a wrong guess: gather the constants (k_warp_ring's body)
          BatchRing br{};
          br.wa.W = lw;
          br.wa.H = lh;
          br.wa.P = P;
          br.wa.bands = (lw + 63) / 64;
          br.wa.seg_rows = roll_segment(br.wa.bands * regather.n, lh, 6, c->warp_ring_slots);
          br.wa.waves = br.wa.bands * ((lh + br.wa.seg_rows - 1) / br.wa.seg_rows);
          br.I0 = c->bI0s[s];
          br.I1 = c->bI1s[s];
          for (int k = 0; k < 2; ++k)
            for (int j = 0; j < 2; ++j) br.U[k][j] = c->bU[k][j];
          for (int j = 0; j < 3; ++j) br.C[j] = c->bC[j];
          br.ips = c->bips[s];
          br.ps = ps;
          br.sel = regather;
          const size_t tkr = prof_begin(c, st);
#define KB_RING(FM) \
  hipLaunchKernelGGL((kb_warp_ring<6, 2, FM>), dim3(br.wa.waves, regather.n), dim3(128), 0, st, br);
          MATH_SWITCH(math, KB_RING)
#undef KB_RING
          prof_end(c, st, tkr, 1, (double)regather.n * lw * lh * 40.0,
                   (double)regather.n * lw * lh * 28.0);
          for (int j = 0; j < regather.n; ++j) ++regathers[regather.idx[j]];
        }
      } else {
        for (int b = 0; b < n; ++b) stopped_first[b] = 0;
      }
      while (nact > 0) {
        // each active pair's pass (the single-pair rule): k iterations up to and including
        // its next check, at most kTbMax
        std::vector<int> kb(n, 0);
        std::vector<char> ends(n, 0);
        int kmin = kTbMax;
        for (int b = 0; b < n; ++b) {
          if (!act[b]) continue;
          int k = 0;
          double ps_ = prev[b];
          while (k < kTbMax && nit[b] + k < prm.iterations) {
            const bool ce = (prm.epsilon > 0) && ((nit[b] + k) & 1) && (ps_ < scaledEps);
            ++k;
            if (ce) {
              ends[b] = 1;
              break;
            }
            ps_ -= scaledEps;
          }
          kb[b] = k;
          kmin = std::min(kmin, k);
        }
        // r4: pairs grouped by their pass length, one launch per group, so every pair runs
        // its whole pass.  TVL1_BATCH_GROUP=0 keeps r3's lock step: one launch of
        // the shortest pass any active pair allows, the others split theirs.
        if (!c->batch_group)
          for (int b = 0; b < n; ++b)
            if (act[b] && kb[b] > kmin) {
              kb[b] = kmin;
              ends[b] = 0;
            }
        int ngroups = 0;
        for (int K = 1; K <= kTbMax; ++K) {
          BatchSel sel{};
          BatchSel chk{};
          for (int b = 0; b < n; ++b) {
            if (!act[b] || kb[b] != K) continue;
            sel.idx[sel.n++] = (uint8_t)b;
            if (ends[b]) {
              sel.cerr.set(b);
              chk.idx[chk.n++] = (uint8_t)b;
            }
          }
          if (sel.n == 0) continue;
          ++ngroups;
          sel.ubit = ubit;
          sel.pbit = pbit;
          sel.pzero = pzero;
          int blocks;   // residual partials per pair (pair stride c->bnblk)
          {   // wavefront pipelines: 64*PX-px bands down the whole level, one per wave
            BatchRoll br{};
            br.ra.b = batch_bufs;
            br.ra.it = it;
            // PX = 1 (64-px bands) on narrow levels when TVL1_BATCH_PX1_W asks for it
            const int px = lw <= c->batch_px1_w ? 1 : 2;
            const int halo = px == 1 ? K : (K + 1) / 2 * 2;   // roll_halo<K, PX>
            br.ra.bands = (lw + 64 * px - 2 * halo - 1) / (64 * px - 2 * halo);
            // segments sized so the launch's wavefronts fill whole rounds of resident slots,
            // but never shorter than min(rows, batch_seg_min): a pass group of a few pairs (or
            // a tiny level) would otherwise be cut into short segments that repeat the 2K-row
            // halo to fill slots the other batch in flight fills anyway (r5: one segment per
            // band on the strips' <= 100-row levels, +1.7 % strip solves/s,
            // profiles/r5/ab/strips_seg/)
            br.ra.seg_rows = c->roll_seg > 0 ? std::max(c->roll_seg, kRollMinSeg)
                                             : std::max(roll_segment(br.ra.bands * sel.n, lh, K,
                                                                     px == 1 ? c->kb1_slots[K]
                                                                             : c->roll_slots[K][0][2]),
                                                        std::min(lh, c->batch_seg_min));
            br.ra.waves = br.ra.bands * ((lh + br.ra.seg_rows - 1) / br.ra.seg_rows);
            blocks = br.ra.waves;
            if (blocks > c->bnblk)
              return set_err(c, TVL1_EHIP, "internal: %d waves > batch partials %d", blocks, c->bnblk);
            for (int k = 0; k < 2; ++k)
              for (int j = 0; j < 2; ++j) br.U[k][j] = c->bU[k][j];
            for (int k = 0; k < 2; ++k)
              for (int j = 0; j < 4; ++j) br.Pp[k][j] = c->bP[k][j];
            for (int j = 0; j < 3; ++j) br.C[j] = c->bC[j];
            br.ps = ps;
            br.partials = c->bpartials;
            br.nblk = c->bnblk;
            br.sel = sel;
            const dim3 grid((br.ra.waves + 3) / 4, sel.n);
            const size_t tkp = prof_begin(c, st);
#define KB_ROLL_M(FM)                                                                       \
  if (px == 1)                                                                            \
    hipLaunchKernelGGL((kb_iterate_roll<KK, 1, FM>), grid, dim3(256), 0, st, br);         \
  else                                                                                    \
    hipLaunchKernelGGL((kb_iterate_roll<KK, 2, FM>), grid, dim3(256), 0, st, br);
#define KB_ROLL(K_)                 \
  {                                 \
    constexpr int KK = K_;          \
    MATH_SWITCH(math, KB_ROLL_M)    \
  }
            switch (K) {
              case 1: KB_ROLL(1) break;
              case 2: KB_ROLL(2) break;
              case 3: KB_ROLL(3) break;
              default: KB_ROLL(4) break;
            }
#undef KB_ROLL
#undef KB_ROLL_M
            if (tkp) {   // k_iterate_roll's accounting (64*PX-px bands) per pair of the launch
              const int seg = br.ra.seg_rows, segs = (lh + seg - 1) / seg;
              double rows = 0.0;
              for (int sg = 0; sg < segs; ++sg) {
                const int ys = sg * seg, ye = std::min(ys + seg, lh);
                rows += std::min(ye - 1 + K, lh - 1) - std::max(ys - K, 0) + 1;
              }
              const double Nl = (double)lw * lh;
              int nz = 0;
              for (int j = 0; j < sel.n; ++j) nz += pzero.test(sel.idx[j]) ? 1 : 0;
              const double band_bytes = (double)br.ra.bands * 64 * px * rows * 4.0;
              const double hbm = band_bytes * ((double)sel.n * 5 + (double)(sel.n - nz) * 4) +
                                 (double)sel.n * Nl * 4.0 * 6.0;
              prof_end(c, st, tkp, 0, (double)sel.n * Nl * 64.0 * K, hbm);
            }
          }
          if (chk.n > 0)
            hipLaunchKernelGGL(kb_reduce, dim3(chk.n), dim3(kBlock), 0, st, c->bpartials,
                               (size_t)c->bnblk, blocks, chk, c->pinned_dev + 8);
        }
        (void)ngroups;
        bool any_check = false;
        for (int b = 0; b < n; ++b) {
          if (!act[b]) continue;
          const int K = kb[b];
          for (int i = 0; i < K; ++i)
            if (!(ends[b] && i == K - 1)) prev[b] -= scaledEps;
          nit[b] += K;
          ubit.flip(b);
          pbit.flip(b);
          pzero.clear(b);
          err[b] = DBL_MAX;
          any_check = any_check || ends[b];
        }
        if (any_check) {
          HIP_TRY(c, hipEventRecord(c->ev_check[0], st));
          HIP_TRY(c, hipEventSynchronize(c->ev_check[0]));
          for (int b = 0; b < n; ++b) {
            if (!act[b] || !ends[b]) continue;
            err[b] = c->pinned[8 + b];
            prev[b] = err[b];
            ++checks[b];
          }
        }
        nact = 0;
        for (int b = 0; b < n; ++b) {
          if (!act[b]) continue;
          act[b] = err[b] > scaledEps && nit[b] < prm.iterations;
          nact += act[b];
        }
      }
      for (int b = 0; b < n; ++b) {
        level_iters[(size_t)b * TVL1_MAX_LEVELS + s] += nit[b];
        if (stats && stats[b].warp_iterations &&
            s * prm.warps + wp < stats[b].warp_iterations_capacity)
          stats[b].warp_iterations[s * prm.warps + wp] = nit[b];
      }
    }
    HIP_TRY(c, hipGetLastError());
    if (s == 0) break;
    BatchUp up{};
    for (int k = 0; k < 2; ++k)
      for (int j = 0; j < 2; ++j) up.U[k][j] = c->bU[k][j];
    up.ps = ps;
    up.sw = lw;
    up.sh = lh;
    up.sp = P;
    up.dw = g.ws[s - 1];
    up.dh = g.hs[s - 1];
    up.dp = g.ps[s - 1];
    up.fx = (float)(1.0 / ((double)up.dw / lw));
    up.fy = (float)(1.0 / ((double)up.dh / lh));
    up.mul = upmul;
    up.sel = all;
    up.sel.ubit = ubit;
    if (contracts(math))
      hipLaunchKernelGGL(kb_upsample<true>, grid2(up.dw, up.dh, 2 * n), kBlk2, 0, st, up);
    else
      hipLaunchKernelGGL(kb_upsample<false>, grid2(up.dw, up.dh, 2 * n), kBlk2, 0, st, up);
    for (int b = 0; b < n; ++b) ubit.flip(b);
  }
  BatchOut bo{};
  for (int k = 0; k < 2; ++k)
    for (int j = 0; j < 2; ++j) bo.U[k][j] = c->bU[k][j];
  bo.ps = ps;
  bo.W = W;
  bo.H = H;
  bo.P = g.ps[0];
  bo.u = u;
  bo.v = v;
  bo.fpitch = fpitch;
  bo.fstride = fstride;
  bo.sel = all;
  bo.sel.ubit = ubit;
  hipLaunchKernelGGL(kb_output, grid2(W, H, n), kBlk2, 0, st, bo);
  HIP_TRY(c, hipGetLastError());
  if (stats) {
    for (int b = 0; b < n; ++b) {
      tvl1_stats &sb = stats[b];
      sb.levels = L;
      int64_t tot = 0;
      int64_t li[TVL1_MAX_LEVELS] = {};
      for (int s = 0; s < TVL1_MAX_LEVELS; ++s) {
        li[s] = s < L ? level_iters[(size_t)b * TVL1_MAX_LEVELS + s] : 0;
        sb.level_width[s] = s < L ? g.ws[s] : 0;
        sb.level_height[s] = s < L ? g.hs[s] : 0;
        sb.level_iterations[s] = li[s];
        tot += li[s];
      }
      sb.iterations_total = tot;
      sb.checks_total = checks[b];
      sb.speculation_misses = regathers[b];   // constants not stored, then needed (re-gathered)
      sb.algorithmic_bytes = survey_bytes(g, prm.warps, li);
      for (int k = 0; k < 4; ++k) {
        sb.kernel_ms[k] = 0.0;
        sb.kernel_launches[k] = 0;
        sb.kernel_bytes[k] = 0.0;
        sb.kernel_hbm_bytes[k] = 0.0;
      }
    }
  }
  // with tvl1_set_profiling: every pair of the chunk reports the chunk's launches (each
  // launch serves all its pairs; bytes are summed over them)
  if (c->profiling && !c->marks.empty()) {
    HIP_TRY(c, hipEventSynchronize(c->ev_pool[c->marks.back().b]));
    double ms[4] = {}, by[4] = {}, hb[4] = {};
    int64_t nl[4] = {};
    for (const auto &m : c->marks) {
      float t = 0.f;
      HIP_TRY(c, hipEventElapsedTime(&t, c->ev_pool[m.a], c->ev_pool[m.b]));
      ms[m.cls] += t;
      nl[m.cls] += 1;
      by[m.cls] += m.bytes;
      hb[m.cls] += m.hbm_bytes;
    }
    if (stats)
      for (int b = 0; b < n; ++b)
        for (int k = 0; k < 4; ++k) {
          stats[b].kernel_ms[k] = ms[k];
          stats[b].kernel_launches[k] = nl[k];
          stats[b].kernel_bytes[k] = by[k];
          stats[b].kernel_hbm_bytes[k] = hb[k];
        }
  }
  return TVL1_OK;
}


// ---------------------------------------------------------------- feature pre-alignment
// find_alignment (features.cpp:46-167) on the GPU + host (tvl1_align.hpp).
namespace {
struct OrbSet {
  std::vector<OrbKp> kps;     // level coordinates (angle filled when asked, orb_detect)
  std::vector<Pt> pts;        // level-0 coordinates
  std::vector<float> resp;    // Harris responses
  uint32_t *desc = nullptr;   // device, 8 words per keypoint (in the ctx's align scratch)
};

// One frame's ORB pyramid geometry and its quota per level (ORB_Impl::detectAndCompute:
// nfeatures * (1 - f) / (1 - f^L) * f^l, the remainder on the last level).
struct OrbGeom {
  int L = 0;
  std::vector<int> w, h, p, quota;
  std::vector<unsigned> cap, off;   // key-list capacity / offset per level
  size_t keys = 0, lev_floats = 0;
  unsigned kmax = 0;
};

static OrbGeom orb_geom(int W, int H, const tvl1_align_params &ap) {
  OrbGeom g;
  g.L = std::max(1, ap.nlevels);
  const double sf = ap.scale_factor;
  g.w.resize(g.L);
  g.h.resize(g.L);
  g.p.resize(g.L);
  g.quota.assign(g.L, 0);
  g.cap.resize(g.L);
  g.off.resize(g.L);
  for (int l = 0; l < g.L; ++l) {
    const double scale = 1.0 / std::pow(sf, l - ap.first_level);
    g.w[l] = l == 0 ? W : std::max(1, (int)std::lrint(W * scale));
    g.h[l] = l == 0 ? H : std::max(1, (int)std::lrint(H * scale));
    g.p[l] = (int)align_up((size_t)g.w[l], 64);
    g.lev_floats += align_up((size_t)g.p[l] * g.h[l], 64);
    g.cap[l] = (unsigned)(((size_t)g.w[l] + 1) / 2 * (((size_t)g.h[l] + 1) / 2));
    g.off[l] = (unsigned)g.keys;
    g.keys += align_up(g.cap[l], 32);
  }
  const double f = 1.0 / sf;
  double nd = ap.nfeatures * (1 - f) / (1 - std::pow(f, g.L));
  int sum = 0;
  for (int l = 0; l < g.L - 1; ++l) {
    g.quota[l] = (int)std::lrint(nd);
    sum += g.quota[l];
    nd *= f;
  }
  g.quota[g.L - 1] = std::max(ap.nfeatures - sum, 0);
  for (int l = 0; l < g.L; ++l) g.kmax = std::max(g.kmax, (unsigned)g.quota[l]);
  return g;
}

// The align scratch: [kps | desc q | desc t | match best | match dist | pyramid | blurred
// pyramid | score | keys | counts | selected keys | nsel | level table], carved per frame.
struct AlignCarve {
  float *lev = nullptr, *blur = nullptr, *score = nullptr;
  uint64_t *keys = nullptr, *sel = nullptr;
  unsigned *cnt = nullptr, *nsel = nullptr;
  SelLevel *lv = nullptr;
  float **dlev = nullptr;
  int *dlp = nullptr;
  OrbKp *kps = nullptr;
  uint32_t *desc[2] = {nullptr, nullptr};
  int2 *best = nullptr, *dist = nullptr;
  Top2 *part = nullptr;
};
constexpr int kMatchSegs = 16;   // train segments of ka_match2 (grid y)

static size_t align_carve(char *base, const OrbGeom &g, bool blur, int nfeat, AlignCarve &cv) {
  size_t o = 0;
  auto take = [&](size_t bytes) -> char * {
    char *p = base ? base + o : nullptr;
    o += align_up(std::max<size_t>(bytes, 1), 256);
    return p;
  };
  // geometry-independent parts first: the two frames' carves share them
  cv.kps = (OrbKp *)take((size_t)nfeat * sizeof(OrbKp));
  cv.desc[0] = (uint32_t *)take((size_t)nfeat * 32);
  cv.desc[1] = (uint32_t *)take((size_t)nfeat * 32);
  cv.best = (int2 *)take((size_t)nfeat * sizeof(int2));
  cv.dist = (int2 *)take((size_t)nfeat * sizeof(int2));
  cv.part = (Top2 *)take((size_t)nfeat * kMatchSegs * sizeof(Top2));
  cv.lev = (float *)take(g.lev_floats * 4);
  cv.blur = blur ? (float *)take(g.lev_floats * 4) : nullptr;
  cv.score = (float *)take((size_t)g.w[0] * g.h[0] * 4);
  cv.keys = (uint64_t *)take(g.keys * 8);
  cv.cnt = (unsigned *)take(g.L * 4);
  cv.sel = (uint64_t *)take((size_t)g.L * g.kmax * 8);
  cv.nsel = (unsigned *)take(g.L * 4);
  cv.lv = (SelLevel *)take(g.L * sizeof(SelLevel));
  cv.dlev = (float **)take(g.L * sizeof(float *));
  cv.dlp = (int *)take(g.L * 4);
  return o;
}

// ORB detect + describe of one frame (cv::cuda::ORB::detectAndCompute, features.cpp:60-61)
// into out; descriptors go to desc.  All levels are queued back to back: one host sync for
// the selected keys, one for the descriptors.
static tvl1_status orb_detect(tvl1_ctx *c, const uint8_t *img, size_t pitch, const OrbGeom &g,
                              const tvl1_align_params &ap, const AlignCarve &cv, uint32_t *desc,
                              OrbSet &out, hipStream_t st, bool angles = false) {
  const int L = g.L, W = g.w[0], H = g.h[0];
  std::vector<float *> lev(L);
  {
    size_t o = 0;
    for (int l = 0; l < L; ++l) {
      lev[l] = cv.lev + o;
      o += align_up((size_t)g.p[l] * g.h[l], 64);
    }
  }
  hipLaunchKernelGGL(k_convert_u8, grid2(W, H, 1), kBlk2, 0, st, img, pitch, img, pitch, lev[0],
                     lev[0], W, H, g.p[0]);
  for (int l = 1; l < L; ++l)
    hipLaunchKernelGGL(k_resize_hp, grid2(g.w[l], g.h[l], 1), kBlk2, 0, st, lev[l - 1], nullptr,
                       nullptr, g.w[l - 1], g.h[l - 1], g.p[l - 1], lev[l], nullptr, nullptr,
                       g.w[l], g.h[l], g.p[l], (double)g.w[l - 1] / g.w[l],
                       (double)g.h[l - 1] / g.h[l], 0, 0, 1.0f);
  const int border = std::max(ap.edge_threshold, kOrbHalf + 1);
  std::vector<SelLevel> lv(L);
  HIP_TRY(c, hipMemsetAsync(cv.cnt, 0, L * sizeof(unsigned), st));
  for (int l = 0; l < L; ++l) {
    lv[l] = SelLevel{g.off[l], g.cap[l], (unsigned)g.quota[l]};
    if (g.w[l] <= 2 * border || g.h[l] <= 2 * border || g.quota[l] == 0) {
      lv[l].quota = 0;
      lv[l].cap = 0;
      continue;
    }
    hipLaunchKernelGGL(ka_fast_harris, dim3((g.w[l] + kFhW - 1) / kFhW, (g.h[l] + kFhH - 1) / kFhH),
                       dim3(256), 0, st, lev[l], g.w[l], g.h[l], g.p[l], border,
                       (float)ap.fast_threshold, cv.score);
    hipLaunchKernelGGL(ka_nms, dim3((g.w[l] + 63) / 64, (g.h[l] + kNmsRows - 1) / kNmsRows),
                       dim3(256), 0, st, cv.score, g.w[l], g.h[l], cv.keys + g.off[l],
                       cv.cnt + l, g.cap[l]);
  }
  HIP_TRY(c, hipMemcpyAsync(cv.lv, lv.data(), L * sizeof(SelLevel), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(ka_select, dim3(L), dim3(1024), 0, st, cv.keys, cv.cnt, cv.lv, cv.sel,
                     g.kmax, cv.nsel);
  std::vector<unsigned> nsel(L);
  std::vector<uint64_t> sel((size_t)L * g.kmax);
  HIP_TRY(c, hipMemcpyAsync(nsel.data(), cv.nsel, L * sizeof(unsigned), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(sel.data(), cv.sel, sel.size() * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  for (int l = 0; l < L; ++l) {
    const unsigned n = std::min(nsel[l], (unsigned)g.quota[l]);
    uint64_t *k = sel.data() + (size_t)l * g.kmax;
    std::sort(k, k + n, [](uint64_t a, uint64_t b) { return a > b; });   // best first
    const double scale = std::pow(ap.scale_factor, l - ap.first_level);
    for (unsigned i = 0; i < n; ++i) {
      const unsigned pos = 0xFFFFFFFFu - (unsigned)(k[i] & 0xFFFFFFFFu);
      const float x = (float)(pos % (unsigned)g.w[l]), y = (float)(pos / (unsigned)g.w[l]);
      out.kps.push_back(OrbKp{x, y, 0.0f, l});
      out.pts.push_back(Pt{x * scale, y * scale});
      const uint32_t rb = (uint32_t)(k[i] >> 32);   // the key's score bits
      float rf;
      memcpy(&rf, &rb, sizeof rf);
      out.resp.push_back(rf);
    }
  }
  if (ap.blur_for_descriptor) {
    size_t o = 0;
    for (int l = 0; l < L; ++l) {
      float *b = cv.blur + o;
      o += align_up((size_t)g.p[l] * g.h[l], 64);
      hipLaunchKernelGGL(ka_blur7, grid2(g.w[l], g.h[l]), kBlk2, 0, st, lev[l], g.w[l], g.h[l],
                         g.p[l], b);
      lev[l] = b;
    }
  }
  const int nk = (int)out.kps.size();
  out.desc = desc;
  if (nk > 0) {
    HIP_TRY(c, hipMemcpyAsync(cv.kps, out.kps.data(), nk * sizeof(OrbKp), hipMemcpyHostToDevice, st));
    HIP_TRY(c, hipMemcpyAsync(cv.dlev, lev.data(), L * sizeof(float *), hipMemcpyHostToDevice, st));
    HIP_TRY(c, hipMemcpyAsync(cv.dlp, g.p.data(), L * sizeof(int), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(ka_describe, dim3((nk + 63) / 64), dim3(64), 0, st,
                       (const float *const *)cv.dlev, cv.dlp, cv.kps, nk, c->align_pat, desc);
    HIP_TRY(c, hipGetLastError());
    if (angles)
      HIP_TRY(c, hipMemcpyAsync(out.kps.data(), cv.kps, nk * sizeof(OrbKp), hipMemcpyDeviceToHost, st));
    // the host vectors above are the copy sources: they must outlive the copies
    HIP_TRY(c, hipStreamSynchronize(st));
  }
  return TVL1_OK;
}

// the rBRIEF pair pattern on the device (set once per ctx)
static tvl1_status ensure_pattern(tvl1_ctx *c) {
  if (c->align_pat) return TVL1_OK;
  static const std::vector<int> pat = orb_pattern();
  HIP_TRY(c, hipMalloc((void **)&c->align_pat, pat.size() * sizeof(int)));
  HIP_TRY(c, hipMemcpy(c->align_pat, pat.data(), pat.size() * sizeof(int), hipMemcpyHostToDevice));
  return TVL1_OK;
}

static tvl1_status check_orb_params(tvl1_ctx *c, const tvl1_align_params *ap) {
  if (ap->nlevels <= 0 || !(ap->scale_factor > 1.0f) || ap->nfeatures <= 0)
    return set_err(c, TVL1_EINVAL, "bad ORB parameters");
  if (ap->wta_k != 2 || ap->patch_size != 31)
    return set_err(c, TVL1_EINVAL, "only WTA_K = 2 and patchSize = 31 are supported");
  return TVL1_OK;
}

static void affine_inverse(const float M[6], Affine &iM) {
  const double a = M[0], b = M[1], cc = M[2], d = M[3], e = M[4], f = M[5];
  double D = a * e - b * d;
  D = D != 0 ? 1.0 / D : 0.0;
  const double A11 = e * D, A22 = a * D, A12 = -b * D, A21 = -d * D;
  iM.m[0] = (float)A11;
  iM.m[1] = (float)A12;
  iM.m[2] = (float)(-A11 * cc - A12 * f);
  iM.m[3] = (float)A21;
  iM.m[4] = (float)A22;
  iM.m[5] = (float)(-A21 * cc - A22 * f);
}
}  // namespace

extern "C" {

void tvl1_params_default(tvl1_params *p) {
  if (!p) return;
  // generate_TV_args, optflow.cpp:503-512
  p->tau = 0.25;
  p->lambda = 0.05;
  p->theta = 0.3;
  p->nscales = 10;
  p->warps = 5;
  p->epsilon = 0.01;
  p->iterations = 300;
  p->scale_step = 0.8;
  p->gamma = 0.0;
  p->use_initial_flow = 0;
  p->median_filtering = 1;
  p->fast_math = 0;
  p->profile = 0;
  p->inner_iterations = 30;   // cv::DualTVL1OpticalFlow defaults (profile 1)
  p->outer_iterations = 10;
}

int32_t tvl1_abi_version(void) { return TVL1_ABI_VERSION; }

int32_t tvl1_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

tvl1_status tvl1_create(tvl1_ctx **out, int device, const tvl1_params *params) {
  if (!out) return set_err(nullptr, TVL1_EINVAL, "out is NULL");
  *out = nullptr;
  tvl1_status s = check_params(nullptr, params);
  if (s != TVL1_OK) return s;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
    return set_err(nullptr, TVL1_ENODEV, "no HIP device visible");
  if (device < 0 || device >= n)
    return set_err(nullptr, TVL1_ENODEV, "device %d out of range (have %d)", device, n);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess)
    return set_err(nullptr, TVL1_ENODEV, "hipGetDeviceProperties failed");
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return set_err(nullptr, TVL1_ENODEV, "device %d is %s; this build targets gfx950 only",
                   device, prop.gcnArchName);
  tvl1_ctx *c = new (std::nothrow) tvl1_ctx();
  if (!c) return set_err(nullptr, TVL1_ENOMEM, "out of host memory");
  c->device = device;
  c->prm = *params;
  // test / diagnostic knobs (tests/test_gpu_parity.py names what each one reaches)
  if (const char *m = getenv("TVL1_ROLL_SEG")) c->roll_seg = atoi(m);
  if (const char *m = getenv("TVL1_ROLL_PX4_MIN")) c->roll_px4_min = atol(m);
  if (const char *m = getenv("TVL1_FUSE")) c->fuse = atoi(m) != 0;
  if (const char *m = getenv("TVL1_MID")) c->mid = atoi(m) != 0;
  if (const char *m = getenv("TVL1_MID_MIN")) c->mid_min = atof(m);
  if (const char *m = getenv("TVL1_WI_NC")) c->wi_nc = atoi(m) == 1 ? 1 : 2;
  if (const char *m = getenv("TVL1_TB4")) c->tb4 = atoi(m) != 0;
  if (const char *m = getenv("TVL1_POLL")) c->poll = atoi(m);
  if (const char *m = getenv("TVL1_SPEC")) c->spec = atoi(m);
  if (const char *m = getenv("TVL1_SPEC_TRACE")) c->spec_trace = atoi(m);
  if (const char *m = getenv("TVL1_FUSE_MIN")) c->fuse_min = atol(m);
  if (const char *m = getenv("TVL1_BATCH_FUSE")) c->batch_fuse = atoi(m) != 0;
  if (const char *m = getenv("TVL1_BATCH_STORE")) c->batch_store_pred = atoi(m) == 0;
  if (const char *m = getenv("TVL1_BATCH_GROUP")) c->batch_group = atoi(m) != 0;
  if (const char *m = getenv("TVL1_BATCH_PX1_W")) c->batch_px1_w = atoi(m);
  if (const char *m = getenv("TVL1_BATCH_SEG_MIN")) c->batch_seg_min = atoi(m);
  if (const char *m = getenv("TVL1_BATCH_SMALL")) c->batch_small = atoi(m) != 0;
  if (const char *m = getenv("TVL1_PROBE_ROLL_LDS")) c->probe_lds = atoi(m);
  if (const char *m = getenv("TVL1_PROBE_WI_LDS")) c->probe_wi_lds = std::min(atoi(m), 32768);
  if (const char *m = getenv("TVL1_BUF_LIMIT"))   // force the 64-bit-addressed kernels
    c->buf_limit = std::min(c->buf_limit, (size_t)std::max(0LL, atoll(m)));
  if (const char *m = getenv("TVL1_CHECK")) c->check = atoi(m);
  if (const char *m = getenv("TVL1_FILL")) c->fill = std::max(10, atoi(m));
  if (const char *m = getenv("TVL1_FILL_SHARED")) c->fill_shared = std::max(10, atoi(m));
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc((void **)&c->pinned, sizeof(double) * (8 + kBatchMax),
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&c->pinned_dev, c->pinned, 0) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_check[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_check[1], hipEventDisableTiming) != hipSuccess ||
      hipMalloc((void **)&c->gate, 256) != hipSuccess ||
      hipMemset(c->gate, 0, 256) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_order, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_switch, hipEventDisableTiming) != hipSuccess) {
    delete c;
    return set_err(nullptr, TVL1_EHIP, "HIP initialisation failed on device %d", device);
  }
  // hipHostMalloc does not promise zeroed memory: a stale sequence word >= the first check's
  // would let the residual poll return before k_reduce wrote
  memset(c->pinned, 0, sizeof(double) * (8 + kBatchMax));
  // resident wavefronts / blocks of the streaming kernels, for their segment sizing
  {
    auto blocks_of = [&](const void *fn, int threads) {
      int nb = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, threads, 0) != hipSuccess) nb = 0;
      return nb * prop.multiProcessorCount;
    };
#define ROLL_SLOTS(G, K, PX) \
  c->roll_slots[K][G][PX] = 4 * blocks_of((const void *)k_iterate_roll<G, K, PX>, 256);
    ROLL_SLOTS(false, 1, 2) ROLL_SLOTS(false, 2, 2) ROLL_SLOTS(false, 3, 2) ROLL_SLOTS(false, 4, 2)
    ROLL_SLOTS(true, 1, 2) ROLL_SLOTS(true, 2, 2) ROLL_SLOTS(true, 3, 2) ROLL_SLOTS(true, 4, 2)
    ROLL_SLOTS(false, 1, 4) ROLL_SLOTS(false, 2, 4) ROLL_SLOTS(true, 1, 4) ROLL_SLOTS(true, 2, 4)
#undef ROLL_SLOTS
    c->mid_slots = 4 * blocks_of((const void *)k_iterate_roll_mid<kIEEE>, 256);
    c->kb1_slots[1] = 4 * blocks_of((const void *)kb_iterate_roll<1, 1, kIEEE>, 256);
    c->kb1_slots[2] = 4 * blocks_of((const void *)kb_iterate_roll<2, 1, kIEEE>, 256);
    c->kb1_slots[3] = 4 * blocks_of((const void *)kb_iterate_roll<3, 1, kIEEE>, 256);
    c->kb1_slots[4] = 4 * blocks_of((const void *)kb_iterate_roll<4, 1, kIEEE>, 256);
    c->warp_ring_slots = blocks_of((const void *)k_warp_ring<6, 2>, 128);
    c->witer_slots = c->wi_nc == 2 ? blocks_of((const void *)k_warp_iter<kWiMargin, 0, 128, 1, 2>, 256)
                                   : blocks_of((const void *)k_warp_iter<kWiMargin, 0, 128, 1, 1>, 192);
    if (c->probe_wi_lds > 0 && c->wi_nc == 2) {   // the probe's segments fill its own residency
      int nb = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void *)k_warp_iter<kWiMargin, 0, 128, 1, 2>,
                                                       256, c->probe_wi_lds) == hipSuccess && nb > 0)
        c->witer_slots = nb * prop.multiProcessorCount;
      (void)hipGetLastError();
    }
    // >= 3-iteration passes stream when the level has at least 4 wavefronts' worth of 56 x 32
    // tiles per SIMD (the measured crossover against 64 x 32 blocked regions)
    c->roll_long_min = 16L * prop.multiProcessorCount;
    if (const char *m = getenv("TVL1_ROLL_LONG_MIN")) c->roll_long_min = atol(m);   // tests
    (void)hipGetLastError();
  }
  *out = c;
  return TVL1_OK;
}

tvl1_status tvl1_set_params(tvl1_ctx *c, const tvl1_params *params) {
  if (!c) return set_err(nullptr, TVL1_EINVAL, "ctx is NULL");
  tvl1_status s = check_params(c, params);
  if (s != TVL1_OK) return s;
  c->prm = *params;
  c->geo_valid = false;  // pyramid depth may change
  return TVL1_OK;
}

static tvl1_status check_call(tvl1_ctx *c, const void *I0, size_t p0, const void *I1, size_t p1,
                              int W, int H, const void *u, const void *v, size_t fp) {
  if (!c) return set_err(nullptr, TVL1_EINVAL, "ctx is NULL");
  if (!I0 || !I1 || !u || !v) return set_err(c, TVL1_EINVAL, "null image or flow pointer");
  if (W <= 0 || H <= 0) return set_err(c, TVL1_ESIZE, "bad size %dx%d", W, H);
  if ((size_t)W * (size_t)H > (size_t)1 << 31)
    return set_err(c, TVL1_ESIZE, "image %dx%d too large", W, H);
  if (p0 < (size_t)W || p1 < (size_t)W) return set_err(c, TVL1_EINVAL, "input pitch < width");
  if (fp < sizeof(float) * (size_t)W || fp % sizeof(float))
    return set_err(c, TVL1_EINVAL, "flow pitch must be >= 4*width and a multiple of 4");
  return TVL1_OK;
}

tvl1_status tvl1_calc(tvl1_ctx *c, const uint8_t *I0, size_t pitch0, const uint8_t *I1,
                      size_t pitch1, int32_t W, int32_t H, float *u, float *v, size_t fpitch,
                      tvl1_stats *stats, void *stream) {
  tvl1_status s = check_call(c, I0, pitch0, I1, pitch1, W, H, u, v, fpitch);
  if (s != TVL1_OK) return s;
  HIP_TRY(c, hipSetDevice(c->device));
  s = ensure_geometry(c, W, H, (hipStream_t)stream);
  if (s != TVL1_OK) return s;
  return solve(c, Frames{I0, I1, pitch0, pitch1, false}, W, H, u, v, fpitch, stats,
               (hipStream_t)stream);
}

tvl1_status tvl1_find_homography(const float *src_xy, const float *dst_xy, int32_t n,
                                 int32_t method, double thresh, double H[9], uint8_t *mask) {
  if (!src_xy || !dst_xy || !H || n < 4 || !(method == 0 || method == 4 || method == 8))
    return set_err(nullptr, TVL1_EINVAL, "find_homography: need n >= 4 points and method 0, 4 or 8");
  std::vector<Pt> a(n), b(n);
  for (int i = 0; i < n; ++i) {
    a[i] = Pt{src_xy[2 * i], src_xy[2 * i + 1]};
    b[i] = Pt{dst_xy[2 * i], dst_xy[2 * i + 1]};
  }
  if (method == 0) {   // all points: the least-squares fit, then the LM refinement
    if (!dlt_homography(a, b, H))
      return set_err(nullptr, TVL1_ESIZE, "find_homography: degenerate points");
    lm_refine(a, b, H, 10);
    if (mask) std::fill(mask, mask + n, (uint8_t)1);
    return TVL1_OK;
  }
  if (!find_homography(a, b, method, thresh, H, mask))
    return set_err(nullptr, TVL1_ESIZE, "find_homography: no model found");
  return TVL1_OK;
}

tvl1_status tvl1_calc_f32(tvl1_ctx *c, const float *I0, size_t pitch0, const float *I1,
                          size_t pitch1, int32_t W, int32_t H, float *u, float *v, size_t fpitch,
                          tvl1_stats *stats, void *stream) {
  tvl1_status s = check_call(c, I0, pitch0, I1, pitch1, W, H, u, v, fpitch);
  if (s != TVL1_OK) return s;
  if (pitch0 < sizeof(float) * (size_t)W || pitch1 < sizeof(float) * (size_t)W ||
      pitch0 % sizeof(float) || pitch1 % sizeof(float))
    return set_err(c, TVL1_EINVAL, "f32 input pitch must be >= 4*width and a multiple of 4");
  HIP_TRY(c, hipSetDevice(c->device));
  s = ensure_geometry(c, W, H, (hipStream_t)stream);
  if (s != TVL1_OK) return s;
  return solve(c, Frames{I0, I1, pitch0, pitch1, true}, W, H, u, v, fpitch, stats,
               (hipStream_t)stream);
}


tvl1_status tvl1_calc_batch(tvl1_ctx *c, int32_t n, const uint8_t *I0, size_t pitch0,
                            size_t pair_stride0, const uint8_t *I1, size_t pitch1,
                            size_t pair_stride1, int32_t W, int32_t H, float *u, float *v,
                            size_t fpitch, size_t flow_pair_stride, tvl1_stats *stats,
                            void *stream) {
  if (n <= 0) return set_err(c, TVL1_EINVAL, "batch size must be > 0 (got %d)", n);
  tvl1_status s = check_call(c, I0, pitch0, I1, pitch1, W, H, u, v, fpitch);
  if (s != TVL1_OK) return s;
  // an input stride of 0 gives every pair the same frame (e.g. one reference slice)
  if (n > 1 && ((pair_stride0 != 0 && pair_stride0 < pitch0 * (size_t)H) ||
                (pair_stride1 != 0 && pair_stride1 < pitch1 * (size_t)H) ||
                flow_pair_stride < fpitch * (size_t)H))
    return set_err(c, TVL1_EINVAL, "pair strides must be 0 or cover one image; the flow stride one field");
  HIP_TRY(c, hipSetDevice(c->device));
  s = ensure_geometry(c, W, H, (hipStream_t)stream);
  if (s != TVL1_OK) return s;
  const tvl1_params &prm = c->prm;
  const float taut = (float)(prm.tau / prm.theta);
  // the batched kernels cover the reference's path with gamma = 0 (every production
  // config); other parameter sets solve the pairs one by one, same results
  bool batched = prm.profile == 0 && prm.gamma == 0.0 && taut >= 0.0f && taut <= FLT_MAX;
  // chunk size: kBatchMax pairs, fewer when their batch arena would not fit in half of
  // the device memory free now (large frames: one chunk of 256 6144x4096 pairs is 0.7 TB)
  int chunk = kBatchMax;
  if (batched) {
    // the batched passes address the 4 p planes of every pair of a chunk through one buffer
    // descriptor (RollBufs): that group must stay below 2 GiB
    const double pplane = (double)align_up((size_t)c->geo.ps[0] * H, 64) * sizeof(float);
    const int nmax = (int)((double)(((size_t)1 << 31) - 8192) / (4.0 * pplane));
    if (nmax < 1)
      batched = false;   // frames this large solve one by one (tvl1_calc's fallbacks)
    else
      chunk = std::min(chunk, nmax);
  }
  if (batched) {
    const Geometry &g = c->geo;
    double per_pair = 15.0 * align_up((size_t)g.ps[0] * H, 64) * sizeof(float);
    for (int l = 0; l < g.L; ++l) per_pair += 2.0 * (double)g.ps[l] * g.hs[l] * sizeof(float);
    per_pair += (((W + 55) / 56) * ((H + 23) / 24) + 64) * sizeof(double);
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0) {
      const double avail = 0.5 * (double)free_b + (double)c->barena_bytes;
      chunk = (int)std::max(1.0, std::min((double)chunk, avail / per_pair));
    }
  }
  // other contexts on the device may take memory between hipMemGetInfo and the arena's
  // hipMalloc: a chunk whose arena does not fit is retried at half the size
  for (int b0 = 0; b0 < n;) {
    const int m = batched ? std::min(chunk, n - b0) : 1;
    const uint8_t *i0 = I0 + (size_t)b0 * pair_stride0, *i1 = I1 + (size_t)b0 * pair_stride1;
    float *ub = reinterpret_cast<float *>(reinterpret_cast<char *>(u) + (size_t)b0 * flow_pair_stride);
    float *vb = reinterpret_cast<float *>(reinterpret_cast<char *>(v) + (size_t)b0 * flow_pair_stride);
    s = batched ? solve_batch_chunk(c, m, i0, pitch0, pair_stride0, i1, pitch1, pair_stride1, W,
                                    H, ub, vb, fpitch, flow_pair_stride, stats ? stats + b0 : nullptr,
                                    (hipStream_t)stream)
                : solve(c, Frames{i0, i1, pitch0, pitch1, false}, W, H, ub, vb, fpitch, stats ? stats + b0 : nullptr,
                        (hipStream_t)stream);
    if (s == TVL1_ENOMEM && batched && m > 1) {
      chunk = m / 2;
      continue;
    }
    if (s != TVL1_OK) return s;
    b0 += m;
  }
  return TVL1_OK;
}


void tvl1_align_params_default(tvl1_align_params *p) {
  if (!p) return;
  // orb_defaults (features.cpp:19-31), the ratio test (:109), findHomography (:133)
  p->nfeatures = 5000;
  p->scale_factor = 1.2f;
  p->nlevels = 8;
  p->edge_threshold = 31;
  p->first_level = 0;
  p->wta_k = 2;
  p->patch_size = 31;
  p->fast_threshold = 20;
  p->blur_for_descriptor = 0;
  p->ratio = 0.8f;
  p->method = 8;   // cv::RANSAC
  p->ransac_threshold = 5.0;
}

tvl1_status tvl1_find_alignment(tvl1_ctx *c, const uint8_t *frame1, size_t pitch1, int32_t w1,
                                int32_t h1, const uint8_t *frame0, size_t pitch0, int32_t w0,
                                int32_t h0, const tvl1_align_params *ap, float affine[6],
                                int32_t *n_good, int32_t *outcome, void *stream) {
  if (!c) return set_err(nullptr, TVL1_EINVAL, "ctx is NULL");
  if (!frame1 || !frame0 || !ap || !affine) return set_err(c, TVL1_EINVAL, "null argument");
  if (w1 <= 0 || h1 <= 0 || w0 <= 0 || h0 <= 0) return set_err(c, TVL1_ESIZE, "bad frame size");
  {
    const tvl1_status r = check_orb_params(c, ap);
    if (r != TVL1_OK) return r;
  }
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  order_streams(c, st);
  {
    const tvl1_status r = ensure_pattern(c);
    if (r != TVL1_OK) return r;
  }
  const OrbGeom g1 = orb_geom(w1, h1, *ap), g0 = orb_geom(w0, h0, *ap);
  const bool blur = ap->blur_for_descriptor != 0;
  AlignCarve cv;
  const size_t need = std::max(align_carve(nullptr, g1, blur, ap->nfeatures, cv),
                               align_carve(nullptr, g0, blur, ap->nfeatures, cv));
  if (need > c->align_bytes) {
    const tvl1_status r = arena_alloc(c, &c->align_scratch, &c->align_bytes, need, st);
    if (r != TVL1_OK) return r;
  }
  static const bool timing = getenv("TVL1_ALIGN_TIMING") != nullptr;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  const auto t0 = now();
  // query = frame1, train = frame0 (find_alignment(frame1_GPU, frame0_GPU)); the two frames
  // share the scratch's pyramid and keys and keep their descriptors apart
  OrbSet q, t;
  align_carve(c->align_scratch, g1, blur, ap->nfeatures, cv);
  tvl1_status s = orb_detect(c, frame1, pitch1, g1, *ap, cv, cv.desc[0], q, st);
  const auto t1 = now();
  AlignCarve cv0;
  align_carve(c->align_scratch, g0, blur, ap->nfeatures, cv0);
  if (s == TVL1_OK) s = orb_detect(c, frame0, pitch0, g0, *ap, cv0, cv0.desc[1], t, st);
  const auto t2 = now();
  if (s != TVL1_OK) return s;
  std::vector<int2> best, dist;
  const int nq = (int)q.kps.size(), nt = (int)t.kps.size();
  if (nq > 0 && nt > 0) {
    const int nseg = std::max(1, std::min(kMatchSegs, (nt + 255) / 256));
    const int seg = (int)align_up((size_t)((nt + nseg - 1) / nseg), 64);
    hipLaunchKernelGGL(ka_match2, dim3((nq + 63) / 64, nseg), dim3(64), 0, st, q.desc, nq,
                       t.desc, nt, seg, cv.part);
    hipLaunchKernelGGL(ka_match2_merge, dim3((nq + 255) / 256), dim3(256), 0, st, cv.part, nq,
                       nseg, cv.best, cv.dist);
    best.resize(nq);
    dist.resize(nq);
    HIP_TRY(c, hipMemcpyAsync(best.data(), cv.best, nq * sizeof(int2), hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipMemcpyAsync(dist.data(), cv.dist, nq * sizeof(int2), hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
  }
  const auto t3 = now();
  // the ratio test over the first min(train rows - 1, queries) queries (features.cpp:105-112)
  struct Good {
    int qi, ti, d;
  };
  std::vector<Good> good;
  for (int i = 0; i < std::min(nt - 1, nq); ++i)
    if (best[i].y >= 0 && dist[i].x < ap->ratio * dist[i].y) good.push_back(Good{i, best[i].x, dist[i].x});
  std::stable_sort(good.begin(), good.end(), [](const Good &a, const Good &b) { return a.d < b.d; });
  if (n_good) *n_good = (int32_t)good.size();
  const float ident[6] = {1, 0, 0, 0, 1, 0};
  int oc = 0;
  if (good.size() > 10) {
    std::vector<Pt> p0, p1;
    for (auto &g : good) {
      p0.push_back(q.pts[g.qi]);
      p1.push_back(t.pts[g.ti]);
    }
    double H[9];
    const bool ok = find_homography(p0, p1, ap->method, ap->ransac_threshold, H);
    if (!ok || std::fabs(1 - H[0]) > 0.20 || std::fabs(1 - H[4]) > 0.20) {
      std::copy(ident, ident + 6, affine);
      oc = 2;
    } else {
      for (int k = 0; k < 6; ++k) affine[k] = (float)H[k];
    }
  } else {
    std::copy(ident, ident + 6, affine);
    oc = 1;
  }
  if (outcome) *outcome = oc;
  if (timing)
    fprintf(stderr, "[align] detect1 %.2f ms, detect0 %.2f ms, match %.2f ms, model %.2f ms "
                    "(%d / %d keypoints, %zu good)\n",
            ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, now()), nq, nt, good.size());
  return TVL1_OK;
}

tvl1_status tvl1_orb_detect(tvl1_ctx *c, const uint8_t *frame, size_t pitch, int32_t w, int32_t h,
                            const tvl1_align_params *ap, float *kp, uint8_t *desc, int32_t cap,
                            int32_t *n, void *stream) {
  if (!c) return set_err(nullptr, TVL1_EINVAL, "ctx is NULL");
  if (!frame || !ap || !n || cap < 0 || (cap > 0 && (!kp || !desc)))
    return set_err(c, TVL1_EINVAL, "null argument");
  if (w <= 0 || h <= 0 || pitch < (size_t)w) return set_err(c, TVL1_ESIZE, "bad frame size");
  {
    const tvl1_status r = check_orb_params(c, ap);
    if (r != TVL1_OK) return r;
  }
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  order_streams(c, st);
  {
    const tvl1_status r = ensure_pattern(c);
    if (r != TVL1_OK) return r;
  }
  const OrbGeom g = orb_geom(w, h, *ap);
  const bool blur = ap->blur_for_descriptor != 0;
  AlignCarve cv;
  const size_t need = align_carve(nullptr, g, blur, ap->nfeatures, cv);
  if (need > c->align_bytes) {
    const tvl1_status r = arena_alloc(c, &c->align_scratch, &c->align_bytes, need, st);
    if (r != TVL1_OK) return r;
  }
  align_carve(c->align_scratch, g, blur, ap->nfeatures, cv);
  OrbSet q;
  {
    const tvl1_status r = orb_detect(c, frame, pitch, g, *ap, cv, cv.desc[0], q, st, true);
    if (r != TVL1_OK) return r;
  }
  const int nk = (int)q.kps.size(), m = std::min(nk, cap);
  *n = nk;
  if (m > 0) {
    HIP_TRY(c, hipMemcpyAsync(desc, cv.desc[0], (size_t)m * 32, hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    for (int i = 0; i < m; ++i) {
      float deg = q.kps[i].angle * (float)(180.0 / M_PI);   // cv::KeyPoint::angle
      if (deg < 0.f) deg += 360.f;
      if (deg >= 360.f) deg = 0.f;   // -tiny + 360 rounds to 360
      kp[5 * i + 0] = (float)q.pts[i].x;
      kp[5 * i + 1] = (float)q.pts[i].y;
      kp[5 * i + 2] = (float)q.kps[i].level;
      kp[5 * i + 3] = deg;
      kp[5 * i + 4] = q.resp[i];
    }
  }
  return TVL1_OK;
}

tvl1_status tvl1_match_knn2(tvl1_ctx *c, const uint8_t *query, int32_t nq, const uint8_t *train,
                            int32_t nt, int32_t *idx, int32_t *dist, void *stream) {
  if (!c) return set_err(nullptr, TVL1_EINVAL, "ctx is NULL");
  if (nq < 0 || nt < 0 || (nq > 0 && (!query || !idx || !dist)) || (nt > 0 && !train))
    return set_err(c, TVL1_EINVAL, "bad argument");
  if (nq == 0) return TVL1_OK;
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  order_streams(c, st);
  const int nseg = std::max(1, std::min(kMatchSegs, (nt + 255) / 256));
  const int seg = (int)align_up((size_t)((std::max(nt, 1) + nseg - 1) / nseg), 64);
  // scratch: query and train descriptors, the per-segment top-2, the merged top-2
  const size_t oq = 0, ot = align_up((size_t)nq * 32, 256);
  const size_t op = ot + align_up((size_t)std::max(nt, 1) * 32, 256);
  const size_t ob = op + align_up((size_t)nq * nseg * sizeof(Top2), 256);
  const size_t od = ob + align_up((size_t)nq * sizeof(int2), 256);
  const size_t need = od + align_up((size_t)nq * sizeof(int2), 256);
  if (need > c->align_bytes) {
    const tvl1_status r = arena_alloc(c, &c->align_scratch, &c->align_bytes, need, st);
    if (r != TVL1_OK) return r;
  }
  char *b = c->align_scratch;
  uint32_t *dq = (uint32_t *)(b + oq), *dt = (uint32_t *)(b + ot);
  Top2 *part = (Top2 *)(b + op);
  int2 *best = (int2 *)(b + ob), *dd = (int2 *)(b + od);
  HIP_TRY(c, hipMemcpyAsync(dq, query, (size_t)nq * 32, hipMemcpyHostToDevice, st));
  if (nt > 0) HIP_TRY(c, hipMemcpyAsync(dt, train, (size_t)nt * 32, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(ka_match2, dim3((nq + 63) / 64, nseg), dim3(64), 0, st, dq, nq, dt, nt, seg, part);
  hipLaunchKernelGGL(ka_match2_merge, dim3((nq + 255) / 256), dim3(256), 0, st, part, nq, nseg, best, dd);
  HIP_TRY(c, hipGetLastError());
  static_assert(sizeof(int2) == 2 * sizeof(int32_t), "int2 layout");
  HIP_TRY(c, hipMemcpyAsync(idx, best, (size_t)nq * sizeof(int2), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(dist, dd, (size_t)nq * sizeof(int2), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  return TVL1_OK;
}

tvl1_status tvl1_warp_affine_u8(tvl1_ctx *c, const uint8_t *src, size_t sp, int32_t sw, int32_t sh,
                                uint8_t *dst, size_t dp, int32_t dw, int32_t dh,
                                const float affine[6], void *stream) {
  if (!c) return set_err(nullptr, TVL1_EINVAL, "ctx is NULL");
  if (!src || !dst || !affine) return set_err(c, TVL1_EINVAL, "null argument");
  if (sw <= 0 || sh <= 0 || dw <= 0 || dh <= 0) return set_err(c, TVL1_ESIZE, "bad size");
  HIP_TRY(c, hipSetDevice(c->device));
  Affine iM;
  affine_inverse(affine, iM);
  hipLaunchKernelGGL(ka_warp_u8, grid2(dw, dh), kBlk2, 0, (hipStream_t)stream, src, sp, sw, sh,
                     dst, dp, dw, dh, iM);
  HIP_TRY(c, hipGetLastError());
  return TVL1_OK;
}

tvl1_status tvl1_postprocess_affine(tvl1_ctx *c, float *u, float *v, size_t fp, const uint8_t *I1,
                                    size_t p1, int32_t W, int32_t H, int32_t flow_output,
                                    const float affine[6], void *stream) {
  if (!c) return set_err(nullptr, TVL1_EINVAL, "ctx is NULL");
  if (!u || !v || !I1 || !affine) return set_err(c, TVL1_EINVAL, "null argument");
  if (W <= 0 || H <= 0) return set_err(c, TVL1_ESIZE, "bad size");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  order_streams(c, st);
  const size_t need = 2 * (size_t)W * H * sizeof(float);
  if (need > c->map_bytes) {
    char *m = reinterpret_cast<char *>(c->map_scratch);
    const tvl1_status r = arena_alloc(c, &m, &c->map_bytes, need, st);
    c->map_scratch = reinterpret_cast<float *>(m);
    if (r != TVL1_OK) return r;
  }
  float *m1 = c->map_scratch, *m2 = c->map_scratch + (size_t)W * H;
  Affine iM;
  affine_inverse(affine, iM);
  hipLaunchKernelGGL(ka_map_stage, grid2(W, H), kBlk2, 0, st, u, v, fp, W, H, m1, m2);
  hipLaunchKernelGGL(ka_map_warp, grid2(W, H), kBlk2, 0, st, m1, m2, W, H, iM, flow_output ? 1 : 0,
                     I1, p1, u, v, fp);
  HIP_TRY(c, hipGetLastError());
  return TVL1_OK;
}

tvl1_status tvl1_calc_host(tvl1_ctx *c, const uint8_t *I0, size_t pitch0, const uint8_t *I1,
                           size_t pitch1, int32_t W, int32_t H, float *u, float *v,
                           size_t fpitch, tvl1_stats *stats) {
  tvl1_status s = check_call(c, I0, pitch0, I1, pitch1, W, H, u, v, fpitch);
  if (s != TVL1_OK) return s;
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t st = c->own_stream;
  s = ensure_geometry(c, W, H, st);
  if (s != TVL1_OK) return s;
  const size_t P0 = (size_t)c->geo.ps[0];
  // GpuMat::upload (optflow.cpp:315-316)
  HIP_TRY(c, hipMemcpy2DAsync(c->in0, P0, I0, pitch0, W, H, hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipMemcpy2DAsync(c->in1, P0, I1, pitch1, W, H, hipMemcpyHostToDevice, st));
  s = solve(c, Frames{c->in0, c->in1, P0, P0, false}, W, H, c->outu, c->outv, P0 * sizeof(float),
            stats, st);
  if (s != TVL1_OK) return s;
  // download (optflow.cpp:475-476)
  HIP_TRY(c, hipMemcpy2DAsync(u, fpitch, c->outu, P0 * sizeof(float), W * sizeof(float), H,
                              hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpy2DAsync(v, fpitch, c->outv, P0 * sizeof(float), W * sizeof(float), H,
                              hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  return TVL1_OK;
}

tvl1_status tvl1_postprocess_batch(tvl1_ctx *c, int32_t n, float *u, float *v, size_t fpitch,
                                   size_t fstride, const uint8_t *I1, size_t pitch1,
                                   size_t stride1, int32_t W, int32_t H, int32_t mode,
                                   void *stream) {
  if (n < 0) return set_err(c, TVL1_EINVAL, "n must be >= 0");
  if (n == 0) return c ? TVL1_OK : set_err(nullptr, TVL1_EINVAL, "ctx is NULL");
  tvl1_status s = check_call(c, I1, pitch1, I1, pitch1, W, H, u, v, fpitch);
  if (s != TVL1_OK) return s;
  if (mode < 0 || mode > 2)
    return set_err(c, TVL1_EINVAL, "mode must be 0 (flow), 1 (map) or 2 (map - grid)");
  if (n > 1 && (fstride < fpitch * (size_t)H || fstride % 4 || stride1 < pitch1 * (size_t)(H - 1) + W))
    return set_err(c, TVL1_EINVAL, "pair strides overlap the pairs");
  if (n > 65535) return set_err(c, TVL1_EINVAL, "at most 65535 pairs per call");
  HIP_TRY(c, hipSetDevice(c->device));
  hipLaunchKernelGGL(k_postprocess_batch, grid2(W, H, n), kBlk2, 0, (hipStream_t)stream, u, v,
                     fpitch, fstride, I1, pitch1, stride1, W, H, mode);
  HIP_TRY(c, hipGetLastError());
  return TVL1_OK;
}

tvl1_status tvl1_gather_flow(tvl1_ctx *c, const float *u, const float *v, int64_t plane_elems,
                             const int64_t *offsets, int32_t n, float *out_u, float *out_v,
                             void *stream) {
  if (!c) return set_err(nullptr, TVL1_EINVAL, "ctx is NULL");
  if (n < 0 || (n > 0 && (!u || !v || !offsets || !out_u || !out_v)))
    return set_err(c, TVL1_EINVAL, "bad argument");
  if (n == 0) return TVL1_OK;
  for (int32_t i = 0; i < n; ++i)
    if (offsets[i] < 0 || offsets[i] >= plane_elems)   // never an out-of-range device read
      return set_err(c, TVL1_EINVAL, "offset %lld at %d outside [0, %lld)",
                     (long long)offsets[i], i, (long long)plane_elems);
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  order_streams(c, st);
  const size_t need = align_up((size_t)n * sizeof(int64_t), 256) + (size_t)n * sizeof(float2);
  if (need > c->gather_bytes) {
    const tvl1_status r = arena_alloc(c, &c->gather_scratch, &c->gather_bytes,
                                      std::max<size_t>(need, 64 << 10), st);
    if (r != TVL1_OK) return r;
  }
  int64_t *doff = reinterpret_cast<int64_t *>(c->gather_scratch);
  float2 *dout = reinterpret_cast<float2 *>(c->gather_scratch + align_up((size_t)n * sizeof(int64_t), 256));
  std::vector<float2> host((size_t)n);
  HIP_TRY(c, hipMemcpyAsync(doff, offsets, (size_t)n * sizeof(int64_t), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_gather_flow, dim3((n + 255) / 256), dim3(256), 0, st, u, v, doff, n, dout);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipMemcpyAsync(host.data(), dout, (size_t)n * sizeof(float2), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  for (int32_t i = 0; i < n; ++i) {
    out_u[i] = host[i].x;
    out_v[i] = host[i].y;
  }
  return TVL1_OK;
}

tvl1_status tvl1_postprocess(tvl1_ctx *c, float *u, float *v, size_t fpitch, const uint8_t *I1,
                             size_t pitch1, int32_t W, int32_t H, int32_t mode, void *stream) {
  tvl1_status s = check_call(c, I1, pitch1, I1, pitch1, W, H, u, v, fpitch);
  if (s != TVL1_OK) return s;
  if (mode < 0 || mode > 2)
    return set_err(c, TVL1_EINVAL, "mode must be 0 (flow), 1 (map) or 2 (map - grid)");
  HIP_TRY(c, hipSetDevice(c->device));
  hipLaunchKernelGGL(k_postprocess, grid2(W, H), kBlk2, 0, (hipStream_t)stream, u, v, fpitch, I1,
                     pitch1, W, H, mode);
  HIP_TRY(c, hipGetLastError());
  return TVL1_OK;
}

void *tvl1_stream(tvl1_ctx *c) { return c ? (void *)c->own_stream : nullptr; }

tvl1_status tvl1_set_profiling(tvl1_ctx *c, int32_t enable) {
  if (!c) return set_err(nullptr, TVL1_EINVAL, "ctx is NULL");
  c->profiling = enable != 0;
  return TVL1_OK;
}

void tvl1_destroy(tvl1_ctx *c) {
  if (!c) return;
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  (void)hipSetDevice(c->device);
  if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
  // hipFree waits for the device: callers' streams included
  if (c->arena) (void)hipFree(c->arena);
  if (c->barena) (void)hipFree(c->barena);
  if (c->align_scratch) (void)hipFree(c->align_scratch);
  if (c->map_scratch) (void)hipFree(c->map_scratch);
  if (c->gather_scratch) (void)hipFree(c->gather_scratch);
  if (c->small_scratch) (void)hipFree(c->small_scratch);
  for (auto &r : c->retired) free_retired(r);
  if (c->align_pat) (void)hipFree(c->align_pat);
  if (c->pinned) (void)hipHostFree(c->pinned);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  for (hipEvent_t e : c->ev_check)
    if (e) (void)hipEventDestroy(e);
  if (c->gate) (void)hipFree(c->gate);
  if (c->ev_order) (void)hipEventDestroy(c->ev_order);
  if (c->ev_switch) (void)hipEventDestroy(c->ev_switch);
  delete c;
}

const char *tvl1_last_error(const tvl1_ctx *c) {
  return c ? c->err.c_str() : g_create_error.c_str();
}

}  // extern "C"
