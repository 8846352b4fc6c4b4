// optflow.cpp — the `optflow` command-line driver, MI355X edition.
//
// Keeps the reference CLI/JSON surface (/root/reference/src/optflow.cpp) and calls
// the HIP engine through the C-ABI of include/tvl1.h:
//
//   main            optflow.cpp:29-72    argv, JSON (+gunzip), style dispatch
//   from_file       optflow.cpp:75-178   pair loop, p/q/scale, frame reuse, ROIs,
//                                        output naming, point-match batching
//   get_rois        optflow.cpp:228-261  top / bottom / custom / custom_diff
//   roi_from_array  optflow.cpp:302-310
//   solve_rois      optflow.cpp:312-392  upload, features flag, sorted ROI loop
//   solve_wrapper   optflow.cpp:395-496  TVL1 solve + map/flow/mask + TIFF output
//   generate_TV_args optflow.cpp:500-514
//   TVL1_solve      optflow.cpp:516-520  -> tvl1_calc (the drop-in boundary)
//   random_points   optflow.cpp:522-572
//   move_pm         optflow.cpp:574-593
//   upload_points   optflow.cpp:595-641  -> the render-ws payload is written to a
//                                           file (network upload is out of scope)
//
// Deliberate differences (documented in DESIGN.md):
//   * feature pre-alignment (features.cpp) runs on the engine's GPU ORB path; SURF
//     (features = 2, the default type) is served by ORB with a warning;
//   * per-image "rois" are honoured (the reference passes images["rois"], :140, so
//     they are silently ignored there);
//   * a malformed JSON file is an error (the reference ignores parse failure);
//   * build-only keys: "devices" (list of GPU ordinals, pairs sharded over them),
//     "inflight" (pairs in flight per GPU, default 3), "decode_threads" (slice decode-ahead
//     pool, default min(16, cores - 1)), "medianFiltering",
//     "matches_file", "stats_json", "timing_json" (per-stage host seconds of strip jobs),
//     "skip_existing", "pinned_host" (page-locked slices and
//     flows, default off).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <future>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <map>
#include <mutex>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <vector>

#include "../../include/tvl1.h"
#include "imageio.hpp"
#include "json.hpp"

using ofjson::Value;

namespace {

struct Rect {
  int x = 0, y = 0, width = 0, height = 0;
};

// roi_from_array (optflow.cpp:302-310)
Rect roi_from_array(const Value &a) {
  Rect r;
  r.x = a[(size_t)0].asInt();
  r.y = a[(size_t)1].asInt();
  r.width = a[(size_t)2].asInt();
  r.height = a[(size_t)3].asInt();
  return r;
}

// get_rois (optflow.cpp:228-261)
void get_rois(Value &rois, const Value &args, int rows, int cols) {
  if (args.isMember("top")) {
    rois["top"][0] = 0;
    rois["top"][1] = 0;
    rois["top"][2] = cols;
    rois["top"][3] = args.get("top", 300).asInt();
  }
  if (args.isMember("bottom")) {
    const int bottom = args.get("bottom", 300).asInt();
    rois["bottom"][0] = 0;
    rois["bottom"][1] = rows - bottom;
    rois["bottom"][2] = cols;
    rois["bottom"][3] = bottom;
  }
  if (args.isMember("custom")) {
    if (args["custom"].isMember("0")) {
      rois["custom_diff"]["0"] = args["custom"]["0"];
      if (!args["custom"].isMember("1"))
        fprintf(stderr, "If you specify a custom for the first frame, you must specify a custom "
                        "for the second.\n");
      rois["custom_diff"]["1"] = args["custom"]["1"];
    } else {
      rois["custom"] = args["custom"];
    }
  }
}

// generate_TV_args (optflow.cpp:500-514): per-image value, else global, else default.
tvl1_params generate_TV_args(const Value &im, const Value &args) {
  tvl1_params p;
  tvl1_params_default(&p);
  auto D = [&](const char *k, double d) { return im.get(k, args.get(k, d).asDouble()).asDouble(); };
  auto I = [&](const char *k, int d) { return im.get(k, args.get(k, d).asInt()).asInt(); };
  p.tau = D("tau", 0.25);
  p.lambda = D("lambda", 0.05);
  p.theta = D("theta", 0.3);
  p.nscales = I("nscales", 10);
  p.warps = I("warps", 5);
  p.epsilon = D("epsilon", 0.01);
  p.iterations = I("iterations", 300);
  p.scale_step = D("scaleStep", 0.8);
  p.gamma = D("gamma", 0.0);
  p.use_initial_flow = im.get("useInitialFlow", args.get("useInitialFlow", false).asBool()).asBool();
  p.median_filtering = I("medianFiltering", 1);
  p.fast_math = I("fastMath", 0);
  // build-only: OpenCV's CPU DualTVL1OpticalFlow schedule
  p.profile = I("profile", 0);
  p.inner_iterations = I("innerIterations", 30);
  p.outer_iterations = I("outerIterations", 10);
  return p;
}

std::string output_type_of(const Value &im, const Value &args) {
  return im.get("output_type", args.get("output_type", "map").asString()).asString();
}

// solve_rois' tri-state "features" resolution (optflow.cpp:323-338)
bool resolve_features(const Value &im, const Value &args) {
  if (im.isMember("features") && !im["features"].asBool()) return false;
  if (args.isMember("features") && !args["features"].asBool()) return false;
  if (im.get("features", false).asBool() || args.get("features", false).asBool()) return true;
  return false;
}

bool file_exists(const std::string &p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0;
}

// ---------------------------------------------------------------- per-device worker
struct DeviceCtx {
  int device = 0;
  tvl1_ctx *ctx = nullptr;
  hipStream_t stream = nullptr;
  // device buffers, grown on demand
  uint8_t *d0 = nullptr, *d1 = nullptr;
  uint8_t *dw = nullptr;   // warpAffine target of frame1 (feature pre-alignment)
  size_t cap_img = 0;
  float *du = nullptr, *dv = nullptr;
  size_t cap_flow = 0;
  // frame reuse: the (name, scale) currently resident in d0 / d1
  std::string key0, key1;
  ofio::Image8 h0, h1;
  bool faulted = false;   // a HIP / engine call failed: the context is reset before reuse
};

std::mutex g_io_mutex;

// Per-stage host timing of a job (the build-only "timing_json" key, tools/cli_e2e.py): where
// a strip job's wall time goes -- band reads on the decode pool, and per batch worker the
// wait for its chunk's bands, packing, upload, solve, point sampling, flow read-back and
// output writes.  Seconds of each thread's own clock, summed.
using Clock = std::chrono::steady_clock;
const Clock::time_point g_t0 = Clock::now();
std::atomic<int64_t> g_band_read_ns{0}, g_band_reads{0};
std::mutex g_stage_mutex;
Value g_stage_workers;   // one object per batch worker

inline double secs_since(Clock::time_point t) {
  return std::chrono::duration<double>(Clock::now() - t).count();
}

// Page-locked host buffers for what crosses PCIe (the reference uploads
// with GpuMat::upload, optflow.cpp:315-316): the decode pool writes each slice straight
// into one, so its upload is a single DMA with no pageable staging copy, and full flow
// fields download into them.  hipHostMalloc costs milliseconds per 25 MB slice, so a
// released buffer returns to a free list (best fit, up to 4x the request) instead of
// being unpinned; the list keeps at most kKeep bytes and the pool pins at most kMax, past
// which buffers are pageable; buffers under kMin stay pageable.  Pinning runs outside the
// pool's lock, so decode threads never wait on each other's hipHostMalloc.  A buffer is released only
// after the stream that read or wrote it was synchronised (each pair's solve and downloads
// end in a stream sync before the next pair replaces DeviceCtx::h0 / h1).
class PinnedPool {
 public:
  static void *alloc(size_t n) { return pool().get(n); }
  static void release(void *p, size_t n) { pool().put(p, n); }
  static size_t pinned_bytes() {
    std::lock_guard<std::mutex> lk(pool().m_);
    return pool().pinned_;
  }
  // pins, free-list hits, pageable fallbacks and the time spent pinning (OPTFLOW_PINNED_TRACE)
  static std::string summary() {
    PinnedPool &q = pool();
    std::lock_guard<std::mutex> lk(q.m_);
    char b[200];
    snprintf(b, sizeof b, "pinned pool: %zu MiB pinned, %ld pins (%.1f ms), %ld reuses, %ld pageable",
             q.pinned_ >> 20, q.n_pin_, q.pin_ms_, q.n_hit_, q.n_page_);
    return b;
  }

 private:
  static constexpr size_t kMin = 256u << 10, kKeep = 2ull << 30, kMax = 16ull << 30;
  static PinnedPool &pool() {
    static PinnedPool *p = new PinnedPool;   // never destroyed: buffers may outlive main's locals
    return *p;
  }
  void *get(size_t n) {
    if (n >= kMin && !off_) {
      const size_t cap = (n + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
      std::vector<void *> drop;
      {
        std::lock_guard<std::mutex> lk(m_);
        auto it = free_.lower_bound(cap);   // smallest kept buffer that holds n, up to 4x
        if (it != free_.end() && it->first <= 4 * cap) {
          void *p = it->second;
          kept_ -= it->first;
          live_[p] = it->first;
          free_.erase(it);
          ++n_hit_;
          return p;
        }
        // make room under kMax from the free list before pinning more
        while (pinned_ + cap > kMax && !free_.empty()) {
          auto f = free_.begin();
          drop.push_back(f->second);
          pinned_ -= f->first;
          kept_ -= f->first;
          free_.erase(f);
        }
        if (pinned_ + cap <= kMax) pinned_ += cap;   // reserved; pinned outside the lock
        else {
          ++n_page_;
          return ::operator new(n, std::nothrow);
        }
      }
      for (void *q : drop) (void)hipHostFree(q);
      void *p = nullptr;   // hipHostMalloc takes milliseconds: other threads go on meanwhile
      const auto t0 = std::chrono::steady_clock::now();
      if (hipHostMalloc(&p, cap, hipHostMallocPortable) == hipSuccess && p) {
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::lock_guard<std::mutex> lk(m_);
        live_[p] = cap;
        ++n_pin_;
        pin_ms_ += ms;
        return p;
      }
      std::lock_guard<std::mutex> lk(m_);
      pinned_ -= cap;
      off_ = true;   // no device / no pinnable memory: pageable from here on
    }
    return ::operator new(n, std::nothrow);
  }
  void put(void *p, size_t) {
    if (!p) return;
    {
      std::lock_guard<std::mutex> lk(m_);
      auto it = live_.find(p);
      if (it != live_.end()) {
        const size_t cap = it->second;
        live_.erase(it);
        if (kept_ + cap <= kKeep) {
          free_.emplace(cap, p);
          kept_ += cap;
        } else {
          (void)hipHostFree(p);
          pinned_ -= cap;
        }
        return;
      }
    }
    ::operator delete(p);
  }
  std::mutex m_;
  std::multimap<size_t, void *> free_;   // capacity -> buffer
  std::map<void *, size_t> live_;        // pinned buffers handed out -> capacity
  size_t kept_ = 0, pinned_ = 0;
  std::atomic<bool> off_{false};
  long n_pin_ = 0, n_hit_ = 0, n_page_ = 0;
  double pin_ms_ = 0;
};

bool ensure(DeviceCtx &dc, size_t img_bytes, size_t flow_bytes, bool &realloc, std::string &err) {
  realloc = false;
  if ((img_bytes > dc.cap_img || flow_bytes > dc.cap_flow) && dc.stream)
    (void)hipStreamSynchronize(dc.stream);  // buffers may still be in use by queued work
  if (img_bytes > dc.cap_img) {
    realloc = true;
    for (uint8_t **b : {&dc.d0, &dc.d1, &dc.dw}) {
      if (*b) (void)hipFree(*b);
      *b = nullptr;
    }
    dc.cap_img = 0;
    if (hipMalloc((void **)&dc.d0, img_bytes) != hipSuccess ||
        hipMalloc((void **)&dc.d1, img_bytes) != hipSuccess ||
        hipMalloc((void **)&dc.dw, img_bytes) != hipSuccess) {
      err = "hipMalloc failed for frames", dc.faulted = true;
      return false;
    }
    dc.cap_img = img_bytes;
    dc.key0.clear();
    dc.key1.clear();
  }
  if (flow_bytes > dc.cap_flow) {
    for (float **b : {&dc.du, &dc.dv}) {
      if (*b) (void)hipFree(*b);
      *b = nullptr;
    }
    dc.cap_flow = 0;
    if (hipMalloc((void **)&dc.du, flow_bytes) != hipSuccess ||
        hipMalloc((void **)&dc.dv, flow_bytes) != hipSuccess) {
      err = "hipMalloc failed for flow", dc.faulted = true;
      return false;
    }
    dc.cap_flow = flow_bytes;
  }
  return true;
}

// The reference draws with glibc rand() after std::srand(time(0)) (or, with "debug",
// from the unseeded default state = seed 1).  Other code in this process (the HIP
// runtime) also consumes rand(), so use a PRIVATE generator with glibc's exact
// rand() algorithm (random_r on a 128-byte TYPE_3 state, what rand()/srand() use).
std::mutex g_rand_mutex;
struct GlibcRand {
  random_data rd{};
  char state[128];
  GlibcRand() { initstate_r(1, state, sizeof state, &rd); }
  void seed(unsigned s) { srandom_r(s, &rd); }
  int next() {
    int32_t r;
    random_r(&rd, &r);
    return r;
  }
};
GlibcRand &g_rand() {
  static GlibcRand r;
  return r;
}

// random_points (optflow.cpp:522-572) + the libstdc++ std::random_shuffle it uses.
// The point_matches fields of random_points (optflow.cpp:537-569) for the chosen points;
// any == false gives the dummy point.
void emit_points(const std::vector<std::pair<int, int>> &pts, const std::vector<float> &vx,
                 const std::vector<float> &vy, bool any, Value &im, const Rect &r0, const Rect &r1,
                 float inv_scale, bool features) {
  Value &pm = im["point_matches"];
  for (size_t i = 0; i < pts.size(); ++i) {
    const int px = pts[i].first, py = pts[i].second;
    pm["w"].append(1);
    pm["p"][0].append((double)((px + r0.x) * inv_scale));
    pm["p"][1].append((double)((py + r0.y) * inv_scale));
    if (features) {
      pm["q"][0].append((double)((vx[i] + r1.x) * inv_scale));
      pm["q"][1].append((double)((vy[i] + r1.y) * inv_scale));
    } else {
      pm["q"][0].append((double)((px + r1.x + vx[i]) * inv_scale));
      pm["q"][1].append((double)((py + r1.y + vy[i]) * inv_scale));
    }
  }
  if (!any) {  // dummy point so the fields are full
    pm["p"][0].append(-1);
    pm["p"][1].append(-1);
    pm["q"][0].append(-1);
    pm["q"][1].append(-1);
    pm["w"].append(0);
  }
}

void random_points(const float *fx, const float *fy, int W, int H,
                   Value &im, const Value &args, const Rect &r0, const Rect &r1,
                   const std::vector<uint8_t> &mask, bool features) {
  const bool debug = args.get("debug", false).asBool();
  const float scale = im.get("scale", args.get("scale", 0.5).asFloat()).asFloat();
  const float inv_scale = 1. / scale;
  std::vector<std::pair<int, int>> loc;  // cv::findNonZero: row-major (x, y)
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x)
      if (mask[(size_t)y * W + x]) loc.emplace_back(x, y);
  const int npoints = im.get("npoints", args.get("npoints", 25).asInt()).asInt();
  {
    std::lock_guard<std::mutex> lk(g_rand_mutex);
    if (!debug) g_rand().seed((unsigned)std::time(0));
    for (size_t i = 1; i < loc.size(); ++i) {  // std::random_shuffle (libstdc++)
      const size_t j = (size_t)g_rand().next() % (i + 1);
      if (i != j) std::swap(loc[i], loc[j]);
    }
  }
  std::vector<std::pair<int, int>> pts(loc.begin(), loc.begin() + std::min<size_t>(loc.size(), std::max(npoints, 0)));
  std::vector<float> vx(pts.size()), vy(pts.size());
  for (size_t i = 0; i < pts.size(); ++i) {
    vx[i] = fx[(size_t)pts[i].second * W + pts[i].first];
    vy[i] = fy[(size_t)pts[i].second * W + pts[i].first];
  }
  emit_points(pts, vx, vy, !loc.empty(), im, r0, r1, inv_scale, features);
}

// An engine status that leaves the device context in doubt (a HIP call failed, memory ran
// out): the pair is retried on a rebuilt context.  TVL1_EINVAL / TVL1_ESIZE are input or
// config errors (a bad medianFiltering, an ROI the solver rejects): reported like the
// reference's input errors, without a context rebuild.
static bool device_fault(tvl1_status s) {
  return s == TVL1_EHIP || s == TVL1_ENOMEM || s == TVL1_ENODEV;
}

// The px the sampled random_points draws: npoints distinct px of the mask (frame0 > 1) |
// (frame1 > 1) over a W x H ROI whose rows are row0(y) / row1(y); *total = the mask's size.
template <class R0, class R1>
std::vector<std::pair<int, int>> sample_points(R0 row0, R1 row1, int W, int H, int npoints,
                                               uint64_t *total_out) {
  // mask = (frame0 > 1) | (frame1 > 1) on the ROIs (optflow.cpp:486-494), counted per row
  std::vector<uint64_t> prefix((size_t)H + 1, 0);
  for (int y = 0; y < H; ++y) {
    const uint8_t *a = row0(y), *b = row1(y);
    unsigned c = 0;
    for (int x = 0; x < W; ++x) c += (a[x] > 1) | (b[x] > 1);
    prefix[y + 1] = prefix[y] + c;
  }
  const uint64_t total = prefix[H];
  std::vector<uint64_t> pick;
  {
    std::lock_guard<std::mutex> lk(g_rand_mutex);
    g_rand().seed((unsigned)std::time(0));
    std::map<uint64_t, uint64_t> swapped;   // sparse Fisher-Yates: index -> current value
    auto at = [&](uint64_t i) {
      auto it = swapped.find(i);
      return it == swapped.end() ? i : it->second;
    };
    const uint64_t k = std::min<uint64_t>(total, (uint64_t)std::max(npoints, 0));
    for (uint64_t i = 0; i < k; ++i) {
      const uint64_t r = ((uint64_t)g_rand().next() << 31) ^ (uint64_t)g_rand().next();
      const uint64_t j = i + r % (total - i);
      const uint64_t vi = at(i), vj = at(j);
      swapped[i] = vj;
      swapped[j] = vi;
      pick.push_back(vj);
    }
  }
  std::vector<std::pair<int, int>> pts;
  for (uint64_t idx : pick) {
    const int y = (int)(std::upper_bound(prefix.begin(), prefix.end(), idx) - prefix.begin()) - 1;
    uint64_t left = idx - prefix[y];
    const uint8_t *a = row0(y), *b = row1(y);
    int x = 0;
    for (;; ++x)
      if (((a[x] > 1) | (b[x] > 1)) && left-- == 0) break;
    pts.emplace_back(x, y);
  }
  *total_out = total;
  return pts;
}

// random_points without the debug flag, where the reference seeds rand() with the time
// (optflow.cpp:532-535) and keeps the first npoints of a random_shuffle of all the masked
// px: npoints distinct uniformly random masked px in random order is the same distribution.
// Drawn by a partial Fisher-Yates over the implicit list (row counts + a sparse swap map),
// and only those px's flow values are read back: no 25 M-entry shuffle, no full download.
// Debug runs keep the exact shuffle (random_points above) so their output is reproducible.
bool random_points_sampled(DeviceCtx &dc, size_t fp, int W, int H, const ofio::Image8 &f0,
                           const ofio::Image8 &f1, const Rect &r0, const Rect &r1, Value &im,
                           const Value &args, bool features, std::string &err) {
  const float scale = im.get("scale", args.get("scale", 0.5).asFloat()).asFloat();
  const float inv_scale = 1. / scale;
  const int npoints = im.get("npoints", args.get("npoints", 25).asInt()).asInt();
  uint64_t total = 0;
  const std::vector<std::pair<int, int>> pts = sample_points(
      [&](int y) { return f0.row(r0.y + y) + r0.x; }, [&](int y) { return f1.row(r1.y + y) + r1.x; },
      W, H, npoints, &total);
  std::vector<float> vx(pts.size()), vy(pts.size());
  std::vector<int64_t> off(pts.size());
  for (size_t i = 0; i < pts.size(); ++i)
    off[i] = (int64_t)(pts[i].second * (fp / 4) + pts[i].first);
  // only the chosen px's flow crosses PCIe (tvl1_gather_flow: one upload, one gather, one
  // download), synchronous
  if (const tvl1_status s = tvl1_gather_flow(dc.ctx, dc.du, dc.dv,
                                             (int64_t)((size_t)(H - 1) * (fp / 4) + W), off.data(),
                                             (int32_t)off.size(), vx.data(), vy.data(), dc.stream);
      s != TVL1_OK) {
    err = std::string("flow read-back failed: ") + tvl1_last_error(dc.ctx), dc.faulted = device_fault(s);
    return false;
  }
  emit_points(pts, vx, vy, total > 0, im, r0, r1, inv_scale, features);
  return true;
}

// move_pm (optflow.cpp:574-593)
Value move_pm(Value &im) {
  Value single;
  single["pGroupId"] = im["pGroupId"];
  single["pId"] = im["pId"];
  single["qGroupId"] = im["qGroupId"];
  single["qId"] = im["qId"];
  single["matches"] = im["point_matches"];
  im["point_matches"].clear();
  im["point_matches"] = Value();
  return single;
}

struct PairResult {
  bool done = false;
  bool ok = false;
  std::vector<Value> pms;   // point-match records (random_points)
  Value stats;
};


// solve_wrapper (optflow.cpp:395-496) for one ROI.
bool solve_wrapper(DeviceCtx &dc, const ofio::Image8 &f0, const ofio::Image8 &f1, const Rect &r0,
                   const Rect &r1, Value &im, const Value &args, bool features,
                   const float *affine, PairResult &res, std::string &err) {
  const int W = r0.width, H = r0.height;
  tvl1_params prm = generate_TV_args(im, args);
  if (const tvl1_status s = tvl1_set_params(dc.ctx, &prm); s != TVL1_OK) {
    err = tvl1_last_error(dc.ctx), dc.faulted = device_fault(s);
    return false;
  }
  const size_t pitch = (size_t)f0.width;  // device frames are packed, pitch = width
  const uint8_t *a = dc.d0 + (size_t)r0.y * f0.width + r0.x;
  const uint8_t *b = dc.d1 + (size_t)r1.y * f1.width + r1.x;
  const size_t pitch1 = (size_t)f1.width;
  const size_t fp = (size_t)W * sizeof(float);
  tvl1_stats st;
  memset(&st, 0, sizeof st);
  // per-warp executed iterations (level-major), reported in stats_json beside the totals
  std::vector<int32_t> warp_iters((size_t)TVL1_MAX_LEVELS * std::max(1, prm.warps), -1);
  st.warp_iterations = warp_iters.data();
  st.warp_iterations_capacity = (int32_t)warp_iters.size();
  const auto t0 = std::chrono::steady_clock::now();
  auto record = [&] {
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    Value sv;
    sv["roi"][0] = r0.x;
    sv["roi"][1] = r0.y;
    sv["roi"][2] = W;
    sv["roi"][3] = H;
    sv["seconds"] = secs;
    sv["levels"] = st.levels;
    sv["iterations"] = (int64_t)st.iterations_total;
    sv["checks"] = (int64_t)st.checks_total;
    const size_t nw = std::min(warp_iters.size(), (size_t)std::max(0, st.levels) * std::max(1, prm.warps));
    for (size_t k = 0; k < nw; ++k) sv["warp_iterations"][(int)k] = warp_iters[k];
    res.stats["solves"].append(sv);
  };
  tvl1_status s = tvl1_calc(dc.ctx, a, pitch, b, pitch1, W, H, dc.du, dc.dv, fp, &st, dc.stream);
  if (s != TVL1_OK) {
    err = tvl1_last_error(dc.ctx), dc.faulted = device_fault(s);
    return false;
  }
  const std::string otype = output_type_of(im, args);
  // features: map = flow + grid -> warpAffine(identity) -> flow = map - grid (mode 2),
  // or the map itself (mode 1);
  // "map": flow + grid (mode 1); otherwise unchanged.  Then zero where I1 <= 1.
  const int mode = features ? (otype == "flow" ? 2 : 1) : (otype == "map" ? 1 : 0);
  if (features && affine)   // the features branch with the alignment's affine (:429-443)
    s = tvl1_postprocess_affine(dc.ctx, dc.du, dc.dv, fp, b, pitch1, W, H, otype == "flow" ? 1 : 0,
                                affine, dc.stream);
  else
    s = tvl1_postprocess(dc.ctx, dc.du, dc.dv, fp, b, pitch1, W, H, mode, dc.stream);
  if (s != TVL1_OK) {
    err = tvl1_last_error(dc.ctx), dc.faulted = device_fault(s);
    return false;
  }
  const bool sampled = otype == "random_points" && !args.get("debug", false).asBool();
  if (sampled) {
    if (hipStreamSynchronize(dc.stream) != hipSuccess) {
      err = "solve failed", dc.faulted = true;
      return false;
    }
    record();
    return random_points_sampled(dc, fp, W, H, f0, f1, r0, r1, im, args, features, err);
  }
  ofio::HostVec<float> fx((size_t)W * H), fy((size_t)W * H);   // pinned (PinnedPool)
  if (hipMemcpyAsync(fx.data(), dc.du, fx.size() * 4, hipMemcpyDeviceToHost, dc.stream) != hipSuccess ||
      hipMemcpyAsync(fy.data(), dc.dv, fy.size() * 4, hipMemcpyDeviceToHost, dc.stream) != hipSuccess ||
      hipStreamSynchronize(dc.stream) != hipSuccess) {
    err = "flow download failed", dc.faulted = true;
    return false;
  }
  record();
  if (otype == "map" || otype == "flow") {
    const std::string base = im["output"].asString() + im["output_suffix"].asString();
    std::string e;
    if (!ofio::write_tiff_f32(base + "_x.tiff", fx.data(), W, H, fp, e) ||
        !ofio::write_tiff_f32(base + "_y.tiff", fy.data(), W, H, fp, e)) {
      err = e;
      return false;
    }
  }
  if (otype == "random_points") {
    // mask = (frame0 > 1) | (frame1 > 1) on the ROIs (optflow.cpp:486-494)
    std::vector<uint8_t> mask((size_t)W * H);
    for (int y = 0; y < H; ++y)
      for (int x = 0; x < W; ++x)
        mask[(size_t)y * W + x] = (f0.row(r0.y + y)[r0.x + x] > 1) | (f1.row(r1.y + y)[r1.x + x] > 1);
    random_points(fx.data(), fy.data(), W, H, im, args, r0, r1, mask, features);
  }
  return true;
}

bool in_bounds(const Rect &r, const ofio::Image8 &f) {
  return r.x >= 0 && r.y >= 0 && r.width > 0 && r.height > 0 && r.x + r.width <= f.width &&
         r.y + r.height <= f.height;
}

// orb_defaults (features.cpp:19-32) + the ratio / homo / ransac keys of find_alignment
// (:109, :133), each looked up in the image's args first, then the global args.
tvl1_align_params align_params_of(const Value &im, const Value &args) {
  tvl1_align_params p;
  tvl1_align_params_default(&p);
  auto i = [&](const char *k, int d) { return im.get(k, Value(args.get(k, Value(d)).asInt())).asInt(); };
  auto f = [&](const char *k, double d) {
    return im.get(k, Value(args.get(k, Value(d)).asDouble())).asDouble();
  };
  p.nfeatures = i("nfeatures", p.nfeatures);
  p.scale_factor = (float)f("scaleFactor", p.scale_factor);
  p.nlevels = i("nlevels", p.nlevels);
  p.edge_threshold = i("edgeThreshold", p.edge_threshold);
  p.first_level = i("firstLevel", p.first_level);
  p.wta_k = i("WTA_K", p.wta_k);
  p.patch_size = i("patchSize", p.patch_size);
  p.fast_threshold = i("fastThreshold", p.fast_threshold);
  p.blur_for_descriptor = im.get("blurForDescriptor", Value(args.get("blurForDescriptor", Value(false)).asBool())).asBool();
  p.ratio = (float)f("ratio", p.ratio);
  p.method = i("homo", p.method);
  p.ransac_threshold = f("ransac", p.ransac_threshold);
  return p;
}

// find_alignment(frame1, frame0) + warpAffine(frame1 -> frame0 size) (optflow.cpp:372-376,
// features.cpp:46-167).  The aligned frame replaces frame1 on the device (and on the host,
// for the random_points mask), as frame1_GPU = new_frame1 does in the reference.
bool align_frame1(DeviceCtx &dc, const ofio::Image8 &f0, const ofio::Image8 &f1,
                  ofio::Image8 &aligned, const Value &im, const Value &args, float affine[6],
                  std::string &err) {
  const int w1 = f1.width, h1 = f1.height;   // f1 may be `aligned` itself (a second key)
  const int feature_type = im.get("features", Value(args.get("features", Value(2)).asInt())).asInt();
  if (feature_type != 1)   // SURF_TYPE (features.h:9) and anything else
    fprintf(stderr, "SURF features are not part of this build; using ORB features for the "
                    "alignment of %s.\n", im["p"].asString().c_str());
  const tvl1_align_params p = align_params_of(im, args);
  int32_t n_good = 0, outcome = 0;
  tvl1_status s = tvl1_find_alignment(dc.ctx, dc.d1, (size_t)w1, w1, h1, dc.d0,
                                      (size_t)f0.width, f0.width, f0.height, &p, affine, &n_good,
                                      &outcome, dc.stream);
  if (s != TVL1_OK) {
    err = std::string("find_alignment: ") + tvl1_last_error(dc.ctx), dc.faulted = device_fault(s);
    return false;
  }
  if (args.get("debug", Value(false)).asBool())
    printf("Number of good features: %d\n", n_good);
  if (outcome == 1) printf("Not enough matches. Using no transformation\n");
  if (outcome == 2)
    printf("More than twenty percent variance in zoom or no homography found, this is probably "
           "an error, ignoring the transformation.\n");
  s = tvl1_warp_affine_u8(dc.ctx, dc.d1, (size_t)w1, w1, h1, dc.dw,
                          (size_t)f0.width, f0.width, f0.height, affine, dc.stream);
  if (s != TVL1_OK) {
    err = std::string("warpAffine: ") + tvl1_last_error(dc.ctx), dc.faulted = device_fault(s);
    return false;
  }
  aligned.width = f0.width;
  aligned.height = f0.height;
  aligned.data.resize((size_t)f0.width * f0.height);
  if (hipMemcpyAsync(aligned.data.data(), dc.dw, aligned.data.size(), hipMemcpyDeviceToHost, dc.stream) !=
          hipSuccess ||
      hipStreamSynchronize(dc.stream) != hipSuccess) {
    err = "download of the aligned frame failed", dc.faulted = true;
    return false;
  }
  std::swap(dc.d1, dc.dw);
  dc.key1.clear();  // the device copy is the aligned frame, not the slice
  return true;
}

// Device context of one worker: engine ctx, stream and buffers.
bool open_device(DeviceCtx &dc, int device, std::string &err) {
  dc.device = device;
  tvl1_params p;
  tvl1_params_default(&p);
  if (tvl1_create(&dc.ctx, device, &p) != TVL1_OK) {
    err = tvl1_last_error(nullptr);
    dc.ctx = nullptr;
    return false;
  }
  (void)hipSetDevice(device);
  if (hipStreamCreateWithFlags(&dc.stream, hipStreamNonBlocking) != hipSuccess) {
    err = "hipStreamCreate failed";
    dc.stream = nullptr;
    return false;
  }
  dc.faulted = false;
  return true;
}

void close_device(DeviceCtx &dc) {
  if (dc.stream) (void)hipStreamSynchronize(dc.stream);
  if (dc.ctx) tvl1_destroy(dc.ctx);
  if (dc.stream) (void)hipStreamDestroy(dc.stream);
  for (void *ptr : {(void *)dc.d0, (void *)dc.d1, (void *)dc.dw, (void *)dc.du, (void *)dc.dv})
    if (ptr) (void)hipFree(ptr);
  dc.ctx = nullptr;
  dc.stream = nullptr;
  dc.d0 = dc.d1 = dc.dw = nullptr;
  dc.du = dc.dv = nullptr;
  dc.cap_img = dc.cap_flow = 0;
  dc.key0.clear();
  dc.key1.clear();
}

// Test hook: OPTFLOW_INJECT_FAULT="i,j,..." makes the first attempt of those pairs fail as
// a device error would (before any device work), to exercise the recovery below.
bool inject_fault(size_t pair) {
  static const std::vector<size_t> list = [] {
    std::vector<size_t> v;
    if (const char *e = getenv("OPTFLOW_INJECT_FAULT"))
      for (const char *q = e; *q;) {
        char *end;
        const unsigned long x = strtoul(q, &end, 10);
        if (end == q) break;
        v.push_back(x);
        q = *end ? end + 1 : end;
      }
    return v;
  }();
  return std::find(list.begin(), list.end(), pair) != list.end();
}

// solve_rois (optflow.cpp:312-392)
bool solve_rois(DeviceCtx &dc, const ofio::Image8 &f0, const ofio::Image8 &f1_in, bool f0_resident,
                bool f1_resident, const Value &rois, Value &im, const Value &args,
                PairResult &res, std::string &err) {
  ofio::Image8 f1_aligned;               // frame1 after find_alignment + warpAffine
  const ofio::Image8 *f1p = &f1_in;      // the frame1 the ROIs read: the slice or f1_aligned
  bool features = resolve_features(im, args);
  const std::string otype = output_type_of(im, args);
  // cv::Mat affine(cv::Size(3,2), CV_32FC1) (optflow.cpp:319) is uninitialised until
  // find_alignment fills it; the identity stands in for that here.
  float affine[6] = {1.f, 0.f, 0.f, 0.f, 1.f, 0.f};
  size_t img_bytes = std::max(f0.data.size(), f1p->data.size());
  size_t flow_bytes = 0;
  for (auto &k : rois.memberNames()) {
    if (k == "custom_diff") {
      const Rect r = roi_from_array(rois[k]["0"]);
      flow_bytes = std::max(flow_bytes, (size_t)std::max(0, r.width) * std::max(0, r.height) * 4);
    } else {
      const Rect r = roi_from_array(rois[k]);
      flow_bytes = std::max(flow_bytes, (size_t)std::max(0, r.width) * std::max(0, r.height) * 4);
    }
  }
  bool realloc = false;
  if (!ensure(dc, img_bytes, std::max<size_t>(flow_bytes, 4), realloc, err)) return false;
  // PinnedPool's invariant (cli/imageio.hpp): a host buffer goes back to the pool only after
  // the stream that reads it was synchronised.  Every successful path below ends in a
  // synchronising download; a failing one (an ROI outside the image, EINVAL / ESIZE, an
  // alignment error) may leave the uploads of f0 / f1 queued, so it waits here.
  struct SyncOnFailure {
    DeviceCtx &dc;
    bool ok = false;
    ~SyncOnFailure() {
      if (!ok && dc.stream) (void)hipStreamSynchronize(dc.stream);
    }
  } sync_guard{dc};
  if (realloc) f0_resident = f1_resident = false;
  // GpuMat::upload (optflow.cpp:315-316), skipped when the slice is already resident
  if (!f0_resident && hipMemcpyAsync(dc.d0, f0.data.data(), f0.data.size(), hipMemcpyHostToDevice, dc.stream) != hipSuccess) {
    err = "upload failed", dc.faulted = true;
    return false;
  }
  if (!f1_resident && hipMemcpyAsync(dc.d1, f1p->data.data(), f1p->data.size(), hipMemcpyHostToDevice, dc.stream) != hipSuccess) {
    err = "upload failed", dc.faulted = true;
    return false;
  }
  bool ok = true;
  for (const auto &key : rois.memberNames()) {  // sorted, like jsoncpp getMemberNames
    im["output_suffix"] = (key == "top" || key == "bottom") ? "_" + key : std::string();
    Rect r0, r1;
    if (key == "custom_diff") {
      if (features) fprintf(stderr, "Features isn't compatible with different ROIs for each image.\n Ignoring features.\n");
      r0 = roi_from_array(rois[key]["0"]);
      r1 = roi_from_array(rois[key]["1"]);
      if (r0.width != r1.width || r0.height != r1.height) {
        err = "custom ROIs of the two frames must have the same size";
        ok = false;
        continue;
      }
    } else {
      const bool size_differs = f0.width != f1p->width || f0.height != f1p->height;
      if (features || size_differs || key == "default") {   // optflow.cpp:366-377
        if (size_differs || (key == "default" && !features))
          fprintf(stderr, "Rows or columns differ between frames no ROI selected, reverting to "
                          "features even though it wasn't selected.\n");
        if (!align_frame1(dc, f0, *f1p, f1_aligned, im, args, affine, err)) return false;
        f1p = &f1_aligned;
        features = true;
      }
      r0 = r1 = roi_from_array(rois[key]);
    }
    if (!in_bounds(r0, f0) || !in_bounds(r1, *f1p)) {
      err = "ROI '" + key + "' is outside the image";
      ok = false;
      continue;
    }
    if (!solve_wrapper(dc, f0, *f1p, r0, r1, im, args, features, affine, res, err)) ok = false;
  }
  if (otype == "random_points") res.pms.push_back(move_pm(im));
  sync_guard.ok = ok;
  return ok;
}

struct Job {
  size_t index;
  Value im;
};

// Decode-ahead pool.  A 6144x4096 PNG takes ~0.3 s of one core to decode
// (zlib inflate ~0.23 s), 5x one pair's GPU solve, so slices are read + pre-scaled by a
// pool of host threads while the GPU works: a worker queues every slice of its current and
// next chunk of pairs and then takes them in pair order.
struct Loaded {
  bool ok = false;
  ofio::Image8 img;
  std::string err;
  // load_bands: the pre-scaled slice's size and the row bands asked for
  int W = 0, H = 0;
  std::vector<ofio::Image8> bands;
  bool partial = false;   // only the bands' source rows were read
};
using LoadFuture = std::shared_future<std::shared_ptr<Loaded>>;

class DecodePool {
 public:
  explicit DecodePool(int n) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this] { run(); });
  }
  ~DecodePool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  // imread(IMREAD_GRAYSCALE) + resize(scale) (optflow.cpp:104-131) on a pool thread
  LoadFuture load(const std::string &path, float scale) {
    auto task = std::make_shared<std::packaged_task<std::shared_ptr<Loaded>()>>([path, scale] {
      auto r = std::make_shared<Loaded>();
      ofio::Image8 img;
      if (!ofio::read_gray8(path, img, r->err) || img.width == 0 || img.height == 0) return r;
      if (scale != 1) ofio::resize_u8(img, scale, scale, r->img);
      else r->img = std::move(img);
      r->ok = true;
      return r;
    });
    LoadFuture f = task->get_future().share();
    {
      std::lock_guard<std::mutex> lk(m_);
      q_.emplace_back([task] { (*task)(); });
    }
    cv_.notify_one();
    return f;
  }
  // imread + resize(scale) of only the rows of get_rois' top / bottom ROIs (SURVEY 3.2's
  // production strips): bands in `keys` order, top = [0, top), bottom = [H - bottom, H) of
  // the pre-scaled slice (ofio::read_gray8_bands: strip-organised TIFF reads just those rows)
  LoadFuture load_bands(const std::string &path, float scale, std::vector<std::string> keys,
                        int top, int bottom) {
    auto task = std::make_shared<std::packaged_task<std::shared_ptr<Loaded>()>>([=] {
      const auto t0 = Clock::now();
      auto r = std::make_shared<Loaded>();
      r->ok = ofio::read_gray8_bands(
          path, scale,
          [&](int, int h) {
            std::vector<std::pair<int, int>> b;
            for (const auto &k : keys) b.push_back(k == "top" ? std::make_pair(0, top)
                                                              : std::make_pair(h - bottom, h));
            return b;
          },
          r->W, r->H, r->bands, r->err, &r->partial);
      g_band_read_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count();
      ++g_band_reads;
      return r;
    });
    LoadFuture f = task->get_future().share();
    {
      std::lock_guard<std::mutex> lk(m_);
      q_.emplace_back([task] { (*task)(); });
    }
    cv_.notify_one();
    return f;
  }

 // any host job (the strip workers' point sampling runs here while their batch solves)
  std::shared_future<void> submit(std::function<void()> fn) {
    auto task = std::make_shared<std::packaged_task<void()>>(std::move(fn));
    std::shared_future<void> f = task->get_future().share();
    {
      std::lock_guard<std::mutex> lk(m_);
      q_.emplace_back([task] { (*task)(); });
    }
    cv_.notify_one();
    return f;
  }

 private:
  void run() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        job = std::move(q_.front());
        q_.pop_front();
      }
      job();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  std::vector<std::thread> th_;
  bool stop_ = false;
};

}  // namespace

// ---------------------------------------------------------------- from_file
static int from_file(Value &args, bool plan_only) {
  Value images = args["images"];
  const bool debug = args.get("debug", false).asBool();
  const size_t n = images.size();
  std::vector<PairResult> results(n);
  std::vector<Value> plans(n);

  // build-only: shard pairs over several GPUs (contiguous chunks keep slice reuse)
  std::vector<int> devices;
  if (args.isMember("devices")) {
    for (size_t i = 0; i < args["devices"].size(); ++i) devices.push_back(args["devices"][i].asInt());
  } else {
    devices.push_back(args.get("device", 0).asInt());
  }
  const bool skip_existing = args.get("skip_existing", false).asBool();

  // build-only "pinned_host" (env OPTFLOW_PINNED overrides): page-locked slices and flow
  // fields (PinnedPool), installed before the first image is allocated.  Off by default:
  // on 96-pair jobs it measured 2-5 % slower end to end -- each 25 MB buffer
  // costs 10-20 ms to pin, a C2 job's decode-ahead window spans ~100 slices, and the
  // pageable upload it replaces (~1 ms per pair) runs on a worker that is not the bound
  bool pinned = args.get("pinned_host", false).asBool();
  if (const char *e = getenv("OPTFLOW_PINNED")) pinned = atoi(e) != 0;
  if (!plan_only && pinned) ofio::set_host_alloc({PinnedPool::alloc, PinnedPool::release});
  // build-only "decode_threads": host threads decoding slices ahead of the GPU
  const unsigned hc = std::max(2u, std::thread::hardware_concurrency());
  DecodePool pool(std::max(1, args.get("decode_threads", (int)std::min(16u, hc - 1)).asInt()));
  std::atomic<size_t> next{0};
  // the pairs the per-pair workers solve (all of them unless strip batching takes some)
  std::vector<size_t> todo;
  size_t m = 0;
  std::vector<char> batch_ok(n, 0);     // the pair goes to the strip batch workers
  size_t chunk = 1;
  std::atomic<int> hard_error{0};

  auto worker = [&](int device) {
    DeviceCtx dc;
    dc.device = device;
    if (!plan_only) {
      std::string err;
      if (!open_device(dc, device, err)) {
        std::lock_guard<std::mutex> lk(g_io_mutex);
        fprintf(stderr, "Error: cannot use GPU %d: %s\n", device, err.c_str());
        close_device(dc);
        hard_error = 1;
        return;
      }
    }
    // this worker's chunks of pairs: the current one and the next, both queued for decode
    std::map<std::string, LoadFuture> pending;   // slice key -> its decode
    auto scale_of = [&](size_t i) {
      return images[i].get("scale", args.get("scale", 0.5).asFloat()).asFloat();
    };
    auto key_of = [&](const std::string &path, float scale) {
      char b[32];
      snprintf(b, sizeof b, "%0.2f", scale);
      return path + "|" + b;
    };
    auto queue_chunk = [&](size_t start) {
      for (size_t k = start; k < std::min(m, start + chunk); ++k) {
        const size_t i = todo[k];
        const float sc = scale_of(i);
        for (const char *side : {"p", "q"}) {
          const std::string path = images[i][side].asString(), k = key_of(path, sc);
          if (!pending.count(k)) pending.emplace(k, pool.load(path, sc));
        }
      }
    };
    size_t next_start = next.fetch_add(chunk);
    if (next_start < m) queue_chunk(next_start);
    for (;;) {
      const size_t start = next_start;
      if (start >= m) break;
      next_start = next.fetch_add(chunk);
      if (next_start < m) queue_chunk(next_start);
      for (size_t kk = start; kk < std::min(m, start + chunk); ++kk) {
        const size_t i = todo[kk];
        Value im = images[i];
        const std::string p = im["p"].asString(), q = im["q"].asString();
        const float scale = scale_of(i);
        im["scale"] = im.get("scale", (double)scale).asDouble();
        {
          std::lock_guard<std::mutex> lk(g_io_mutex);
          printf("%s %s\n", p.c_str(), q.c_str());
          fflush(stdout);
        }
        char buf[32];
        snprintf(buf, sizeof buf, "%0.2f", scale);
        im["output"] = im.get("output", args["output_dir"].asString() + "/" +
                                            im["output_name"].asString() + "_" + buf);
        // load (and pre-scale) the two slices, reusing what is resident
        const std::string k0 = p + "|" + buf, k1 = q + "|" + buf;
        bool r0 = false, r1 = false;
        if (k0 == dc.key0) {
          r0 = true;
        } else if (k0 == dc.key1) {  // previous q is this p: swap roles
          std::swap(dc.d0, dc.d1);
          std::swap(dc.key0, dc.key1);
          std::swap(dc.h0, dc.h1);
          r0 = true;
        }
        r1 = (k1 == dc.key1);
        std::string err;
        // the pooled decode of a slice; a queued slice leaves `pending` (retire) after the
        // last pair of the two queued chunks that names it, whether or not it was decoded
        // for nothing because the slice was already resident
        auto needed_later = [&](const std::string &k) {
          for (size_t jj = kk + 1; jj < std::min(m, start + chunk); ++jj) {
            const size_t j = todo[jj];
            if (key_of(images[j]["p"].asString(), scale_of(j)) == k ||
                key_of(images[j]["q"].asString(), scale_of(j)) == k)
              return true;
          }
          for (size_t jj = next_start; jj < std::min(m, next_start + chunk); ++jj) {
            const size_t j = todo[jj];
            if (key_of(images[j]["p"].asString(), scale_of(j)) == k ||
                key_of(images[j]["q"].asString(), scale_of(j)) == k)
              return true;
          }
          return false;
        };
        auto retire = [&](const std::string &k) {
          if (!needed_later(k)) pending.erase(k);
        };
        auto load = [&](const std::string &name, ofio::Image8 &dst) {
          const std::string k = key_of(name, scale);
          auto it = pending.find(k);
          LoadFuture f = it != pending.end() ? it->second : pool.load(name, scale);
          const std::shared_ptr<Loaded> r = f.get();
          if (!r->ok) {
            err = r->err;
            return false;
          }
          if (needed_later(k)) dst = r->img;   // a later pair reads it again: copy
          else dst = std::move(r->img);        // last use: nobody reads it after this
          return true;
        };
        if (!r0 && !load(p, dc.h0)) {
          std::lock_guard<std::mutex> lk(g_io_mutex);
          printf("Error: %s \n", p.c_str());
          dc.key0.clear();
          results[i].done = true;
          retire(k0);
          retire(k1);
          continue;
        }
        if (!r1 && !load(q, dc.h1)) {
          std::lock_guard<std::mutex> lk(g_io_mutex);
          printf("Error: %s \n", q.c_str());
          dc.key1.clear();
          results[i].done = true;
          retire(k0);
          retire(k1);
          continue;
        }
        dc.key0 = k0;
        dc.key1 = k1;
        retire(k0);
        retire(k1);
        const int rows = std::min(dc.h0.height, dc.h1.height), cols = std::min(dc.h0.width, dc.h1.width);
        Value rois;
        if (im.isMember("rois")) {
          get_rois(rois, im["rois"], rows, cols);
        } else if (args.isMember("rois")) {
          get_rois(rois, args["rois"], rows, cols);
        } else {
          rois["default"][0] = 0;
          rois["default"][1] = 0;
          rois["default"][2] = cols;
          rois["default"][3] = rows;
        }
        if (plan_only) {
          Value pl;
          pl["index"] = (int64_t)i;
          pl["p"] = p;
          pl["q"] = q;
          pl["scale"] = (double)scale;
          pl["size0"][0] = dc.h0.width;
          pl["size0"][1] = dc.h0.height;
          pl["output"] = im["output"];
          pl["rois"] = rois;
          pl["output_type"] = output_type_of(im, args);
          pl["features"] = resolve_features(im, args);
          pl["strip_batch"] = (bool)batch_ok[i];   // solved in a tvl1_calc_batch chunk
          const tvl1_params tp = generate_TV_args(im, args);
          pl["tv"]["tau"] = tp.tau;
          pl["tv"]["lambda"] = tp.lambda;
          pl["tv"]["theta"] = tp.theta;
          pl["tv"]["nscales"] = tp.nscales;
          pl["tv"]["warps"] = tp.warps;
          pl["tv"]["epsilon"] = tp.epsilon;
          pl["tv"]["iterations"] = tp.iterations;
          pl["tv"]["scaleStep"] = tp.scale_step;
          pl["tv"]["gamma"] = tp.gamma;
          pl["tv"]["medianFiltering"] = tp.median_filtering;
          pl["tv"]["fastMath"] = tp.fast_math;
          pl["tv"]["profile"] = tp.profile;
          pl["tv"]["innerIterations"] = tp.inner_iterations;
          pl["tv"]["outerIterations"] = tp.outer_iterations;
          for (auto &key : rois.memberNames())
            pl["files"].append(im["output"].asString() +
                               ((key == "top" || key == "bottom") ? "_" + key : std::string()));
          plans[i] = pl;
          results[i].done = results[i].ok = true;
          continue;
        }
        if (skip_existing && output_type_of(im, args) != "random_points") {
          bool all = true;
          for (auto &key : rois.memberNames()) {
            const std::string base = im["output"].asString() +
                                     ((key == "top" || key == "bottom") ? "_" + key : std::string());
            all = all && file_exists(base + "_x.tiff") && file_exists(base + "_y.tiff");
          }
          if (all) {
            results[i].done = results[i].ok = true;
            continue;
          }
        }
        if (inject_fault(i)) {
          results[i].ok = false;
          dc.faulted = true;
          err = "injected device fault";
        } else {
          results[i].ok = solve_rois(dc, dc.h0, dc.h1, r0, r1, rois, im, args, results[i], err);
        }
        if (!results[i].ok) {  // device contents are unknown after a failure
          dc.key0.clear();
          dc.key1.clear();
        }
        // failure recovery: a pair that failed on a device error is solved once
        // more on a fresh context (engine ctx, stream and buffers rebuilt); input errors
        // (an ROI outside the image) are reported as the reference reports them
        if (!results[i].ok && dc.faulted) {
          {
            std::lock_guard<std::mutex> lk(g_io_mutex);
            fprintf(stderr, "Warning: pair %zu (%s %s): %s; retrying on a fresh device context\n",
                    i, p.c_str(), q.c_str(), err.c_str());
          }
          close_device(dc);
          results[i] = PairResult();
          std::string e2;
          if (!open_device(dc, device, e2)) {
            err = "device context could not be rebuilt: " + e2;
          } else {
            err.clear();
            results[i].ok = solve_rois(dc, dc.h0, dc.h1, false, false, rois, im, args, results[i], err);
            if (!results[i].ok) {
              dc.key0.clear();
              dc.key1.clear();
            } else {
              dc.key0 = k0;
              dc.key1 = k1;
            }
          }
        }
        results[i].done = true;
        if (!results[i].ok) {
          std::lock_guard<std::mutex> lk(g_io_mutex);
          fprintf(stderr, "Error: pair %zu (%s %s): %s\n", i, p.c_str(), q.c_str(), err.c_str());
        }
      }
    }
    close_device(dc);
  };

  // ---- batched strip jobs.  The production shape (SURVEY 3.2,
  // gen_cross_file_list.py:75-99: global top / bottom ROIs at scale 0.5, per-image keys only
  // p, q, the ids and output_name) is two ~100-row strips per pair: one tvl1_calc per strip
  // is ~400 launches of a few microseconds, so the GPU idles on dispatch.  Here a worker
  // takes a chunk of such pairs, reads only the strips' rows of each slice (read_gray8_bands),
  // and solves each ROI key's strips of the whole chunk in one tvl1_calc_batch (every strip's
  // flow and iteration counts identical to its own tvl1_calc), then writes each pair's
  // outputs as solve_wrapper would (optflow.cpp:395-496).  Pairs that turn out not to fit
  // (frames of different sizes, an ROI outside the slice, an unreadable file) are solved by
  // the per-pair path afterwards, which reports them exactly as before.
  std::vector<std::string> roi_keys;   // sorted, like solve_rois' std::map (optflow.cpp:339)
  int roi_top = 0, roi_bottom = 0;
  std::vector<char> deferred(n, 0);
  std::vector<size_t> batched;         // pairs for the batch workers, in order
  std::atomic<size_t> bnext{0};
  size_t bchunk = 0;
  auto batch_worker = [&](int device) {
    DeviceCtx dc;
    std::string err;
    if (!open_device(dc, device, err)) {
      std::lock_guard<std::mutex> lk(g_io_mutex);
      fprintf(stderr, "Error: cannot use GPU %d: %s\n", device, err.c_str());
      close_device(dc);
      hard_error = 1;
      return;
    }
    const float scale = args.get("scale", 0.5).asFloat();
    char sbuf[32];
    snprintf(sbuf, sizeof sbuf, "%0.2f", scale);
    const tvl1_params prm = generate_TV_args(Value(), args);
    const std::string otype = output_type_of(Value(), args);
    const int mode = otype == "map" ? 1 : 0;   // no features on this path
    // device buffers (grown): the chunk's packed frames and flows of one ROI key
    uint8_t *dP = nullptr, *dQ = nullptr;
    float *dU = nullptr, *dV = nullptr;
    size_t cap_px = 0;
    uint8_t *hP = nullptr, *hQ = nullptr;   // page-locked packing buffers (reused)
    size_t cap_h = 0;
    auto release = [&] {
      for (void *q : {(void *)dP, (void *)dQ, (void *)dU, (void *)dV})
        if (q) (void)hipFree(q);
      for (void *q : {(void *)hP, (void *)hQ})
        if (q) (void)hipHostFree(q);
      dP = dQ = nullptr, dU = dV = nullptr, hP = hQ = nullptr;
      cap_px = cap_h = 0;
    };
    auto grow = [&](size_t px) {
      if (px > cap_px) {
        for (void *q : {(void *)dP, (void *)dQ, (void *)dU, (void *)dV})
          if (q) (void)hipFree(q);
        dP = dQ = nullptr, dU = dV = nullptr, cap_px = 0;
        if (hipMalloc((void **)&dP, px) != hipSuccess || hipMalloc((void **)&dQ, px) != hipSuccess ||
            hipMalloc((void **)&dU, 4 * px) != hipSuccess || hipMalloc((void **)&dV, 4 * px) != hipSuccess)
          return false;
        cap_px = px;
      }
      if (px > cap_h) {
        for (void *q : {(void *)hP, (void *)hQ})
          if (q) (void)hipHostFree(q);
        hP = hQ = nullptr, cap_h = 0;
        if (hipHostMalloc((void **)&hP, px, hipHostMallocPortable) != hipSuccess ||
            hipHostMalloc((void **)&hQ, px, hipHostMallocPortable) != hipSuccess)
          return false;
        cap_h = px;
      }
      return true;
    };
    std::map<std::string, double> tm;   // stage -> seconds on this worker (timing_json)
    size_t t_chunks = 0, t_pairs = 0;
    const auto t_worker = Clock::now();
    hipEvent_t ev_up0 = nullptr, ev_up1 = nullptr;   // the chunk's uploads on the stream
    (void)hipEventCreate(&ev_up0);
    (void)hipEventCreate(&ev_up1);
    std::map<std::string, LoadFuture> pending;   // path -> its bands (this chunk + the next)
    auto queue_chunk = [&](size_t start) {
      for (size_t k = start; k < std::min(batched.size(), start + bchunk); ++k)
        for (const char *side : {"p", "q"}) {
          const std::string path = images[batched[k]][side].asString();
          if (!pending.count(path))
            pending.emplace(path, pool.load_bands(path, scale, roi_keys, roi_top, roi_bottom));
        }
    };
    size_t next_start = bnext.fetch_add(bchunk);
    if (next_start < batched.size()) queue_chunk(next_start);
    for (;;) {
      const size_t start = next_start;
      if (start >= batched.size()) break;
      next_start = bnext.fetch_add(bchunk);
      if (next_start < batched.size()) queue_chunk(next_start);
      const size_t end = std::min(batched.size(), start + bchunk);
      // the chunk's pairs whose two slices decoded to equal sizes, with their bands
      struct Item {
        size_t i;
        Value im;
        std::shared_ptr<Loaded> p, q;
      };
      std::vector<Item> items;
      for (size_t k = start; k < end; ++k) {
        const size_t i = batched[k];
        Item it{i, images[i], nullptr, nullptr};
        const std::string p = it.im["p"].asString(), q = it.im["q"].asString();
        it.im["scale"] = it.im.get("scale", (double)scale).asDouble();
        it.im["output"] = it.im.get("output", args["output_dir"].asString() + "/" +
                                                  it.im["output_name"].asString() + "_" + sbuf);
        {
          const auto tw = Clock::now();
          it.p = pending.at(p).get();
          it.q = pending.at(q).get();
          tm["wait_bands"] += secs_since(tw);
        }
        if (!it.p->ok || !it.q->ok || it.p->W != it.q->W || it.p->H != it.q->H) {
          deferred[i] = 1;   // the per-pair path reports or aligns it as the reference does
          continue;
        }
        {
          std::lock_guard<std::mutex> lk(g_io_mutex);
          printf("%s %s\n", p.c_str(), q.c_str());
          fflush(stdout);
        }
        if (skip_existing && otype != "random_points") {
          bool all = true;
          for (auto &key : roi_keys) {
            const std::string base = it.im["output"].asString() + "_" + key;
            all = all && file_exists(base + "_x.tiff") && file_exists(base + "_y.tiff");
          }
          if (all) {
            results[i].done = results[i].ok = true;
            continue;
          }
        }
        items.push_back(std::move(it));
      }
      // slices no later pair of this or the next chunk names leave the map
      {
        std::map<std::string, LoadFuture> keep;
        for (size_t k = next_start; k < std::min(batched.size(), next_start + bchunk); ++k)
          for (const char *side : {"p", "q"}) {
            const std::string path = images[batched[k]][side].asString();
            auto f = pending.find(path);
            if (f != pending.end()) keep.emplace(path, f->second);
          }
        pending.swap(keep);
      }
      const int nb = (int)items.size();
      if (nb == 0) continue;
      bool inject = false;
      for (auto &it : items) inject = inject || inject_fault(it.i);
      // one attempt, and after a device error one more on a rebuilt context
      for (int attempt = 0; attempt < 2; ++attempt) {
        std::string e;
        bool ok = true;
        std::vector<std::vector<Value>> solves(nb);
        // debug random_points: the flows of every key, drawn pair by pair afterwards so the
        // unseeded generator is consumed in the per-pair path's order (pair, then key)
        std::vector<std::vector<float>> dbg_fx(roi_keys.size()), dbg_fy(roi_keys.size());
        auto fail = [&](const std::string &what, tvl1_status st) {
          e = what + (dc.ctx ? std::string(": ") + tvl1_last_error(dc.ctx) : std::string());
          dc.faulted = device_fault(st);
          ok = false;
        };
        if (attempt == 0 && inject) fail("injected device fault", TVL1_EHIP);
        if (ok && tvl1_set_params(dc.ctx, &prm) != TVL1_OK) fail("tvl1_set_params", TVL1_EINVAL);
        for (size_t kk = 0; ok && kk < roi_keys.size(); ++kk) {
          const std::string &key = roi_keys[kk];
          const int W = items[0].p->W, h = items[0].p->bands[kk].height;
          const int y0 = key == "top" ? 0 : items[0].p->H - h;
          const size_t px = (size_t)W * h;
          bool same = true;   // one geometry per launch: every pair's slices of one size
          for (auto &it : items) same = same && it.p->W == W && it.p->bands[kk].height == h && it.p->H == items[0].p->H;
          if (!same) {   // mixed slice sizes in one job: the per-pair path takes the chunk
            for (auto &it : items) deferred[it.i] = 1;
            items.clear();
            break;
          }
          if (!grow(px * nb)) {
            fail("hipMalloc failed for a strip batch", TVL1_ENOMEM);
            break;
          }
          auto ts = Clock::now();
          for (int b = 0; b < nb; ++b) {
            memcpy(hP + px * b, items[b].p->bands[kk].data.data(), px);
            memcpy(hQ + px * b, items[b].q->bands[kk].data.data(), px);
          }
          tm["pack"] += secs_since(ts);
          (void)hipEventRecord(ev_up0, dc.stream);
          if (hipMemcpyAsync(dP, hP, px * nb, hipMemcpyHostToDevice, dc.stream) != hipSuccess ||
              hipMemcpyAsync(dQ, hQ, px * nb, hipMemcpyHostToDevice, dc.stream) != hipSuccess) {
            fail("upload failed", TVL1_EHIP);
            break;
          }
          (void)hipEventRecord(ev_up1, dc.stream);
          std::vector<tvl1_stats> st(nb);
          std::vector<int32_t> wi((size_t)nb * TVL1_MAX_LEVELS * std::max(1, prm.warps), -1);
          for (int b = 0; b < nb; ++b) {
            memset(&st[b], 0, sizeof st[b]);
            st[b].warp_iterations = wi.data() + (size_t)b * TVL1_MAX_LEVELS * std::max(1, prm.warps);
            st[b].warp_iterations_capacity = TVL1_MAX_LEVELS * std::max(1, prm.warps);
          }
          // random_points without debug: which px each pair reports depends only on its
          // bands' masks, so the draws run on the decode pool while the batch solves (they
          // were 16 % of a strip worker's time on the worker thread, profiles/r6/cli/)
          const bool sampled = otype == "random_points" && !debug;
          std::vector<std::vector<std::pair<int, int>>> pts(nb);
          std::vector<uint64_t> tot(nb, 0);
          std::vector<std::shared_future<void>> draws;
          if (sampled) {
            const int per = std::max(1, nb / 16);   // 16 jobs of the chunk's pairs
            for (int b0 = 0; b0 < nb; b0 += per)
              draws.push_back(pool.submit([&, b0, per, kk] {
                for (int b = b0; b < std::min(nb, b0 + per); ++b) {
                  const ofio::Image8 &a = items[b].p->bands[kk], &c = items[b].q->bands[kk];
                  const int np = items[b].im.get("npoints", args.get("npoints", 25).asInt()).asInt();
                  pts[b] = sample_points([&](int y) { return a.row(y); }, [&](int y) { return c.row(y); },
                                         a.width, a.height, np, &tot[b]);
                }
              }));
          }
          const auto t0 = std::chrono::steady_clock::now();
          tvl1_status sc = tvl1_calc_batch(dc.ctx, nb, dP, W, px, dQ, W, px, W, h, dU, dV, 4 * (size_t)W,
                                           4 * px, st.data(), dc.stream);
          if (sc == TVL1_OK)
            sc = tvl1_postprocess_batch(dc.ctx, nb, dU, dV, 4 * (size_t)W, 4 * px, dQ, W, px, W, h,
                                        mode, dc.stream);
          if (sc != TVL1_OK) {
            for (auto &f : draws) f.wait();   // they read this chunk's bands
            fail("strip batch", sc);
            break;
          }
          tm["solve"] += secs_since(t0);   // the batch's host time (it syncs at every check)
          {
            float up_ms = 0.0f;   // the uploads, on the GPU clock (done before the first check)
            if (hipEventElapsedTime(&up_ms, ev_up0, ev_up1) == hipSuccess) tm["upload_gpu"] += 1e-3 * up_ms;
          }
          ts = Clock::now();
          std::vector<float> fx, fy;   // whole flows (TIFF outputs, debug point matches)
          if (sampled) {
            for (auto &f : draws) f.wait();
            std::vector<int64_t> off;
            for (int b = 0; b < nb; ++b)
              for (auto &pt : pts[b]) off.push_back((int64_t)(px * b + (size_t)pt.second * W + pt.first));
            tm["sample_points_wait"] += secs_since(ts);
            ts = Clock::now();
            fx.resize(off.size());
            fy.resize(off.size());
            sc = tvl1_gather_flow(dc.ctx, dU, dV, (int64_t)(px * nb), off.data(), (int32_t)off.size(),
                                  fx.data(), fy.data(), dc.stream);
            if (sc != TVL1_OK) {
              fail("flow read-back", sc);
              break;
            }
          } else {
            fx.resize(px * nb);
            fy.resize(px * nb);
            if (hipMemcpyAsync(fx.data(), dU, 4 * px * nb, hipMemcpyDeviceToHost, dc.stream) != hipSuccess ||
                hipMemcpyAsync(fy.data(), dV, 4 * px * nb, hipMemcpyDeviceToHost, dc.stream) != hipSuccess ||
                hipStreamSynchronize(dc.stream) != hipSuccess) {
              fail("flow download failed", TVL1_EHIP);
              break;
            }
          }
          const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
          tm["read_back"] += secs_since(ts);
          ts = Clock::now();
          const Rect r{0, y0, W, h};
          size_t o = 0;
          for (int b = 0; b < nb && ok; ++b) {
            Value &im = items[b].im;
            Value sv;
            sv["roi"][0] = 0;
            sv["roi"][1] = y0;
            sv["roi"][2] = W;
            sv["roi"][3] = h;
            sv["seconds"] = secs;
            sv["batch"] = nb;
            sv["levels"] = st[b].levels;
            sv["iterations"] = (int64_t)st[b].iterations_total;
            sv["checks"] = (int64_t)st[b].checks_total;
            const size_t nw = std::min((size_t)st[b].warp_iterations_capacity,
                                       (size_t)std::max(0, st[b].levels) * std::max(1, prm.warps));
            for (size_t k = 0; k < nw; ++k) sv["warp_iterations"][(int)k] = st[b].warp_iterations[k];
            sv["read_rows_only"] = items[b].p->partial && items[b].q->partial;
            solves[b].push_back(sv);
            if (sampled) {
              std::vector<float> vx(fx.begin() + o, fx.begin() + o + pts[b].size()),
                  vy(fy.begin() + o, fy.begin() + o + pts[b].size());
              o += pts[b].size();
              emit_points(pts[b], vx, vy, tot[b] > 0, im, r, r, 1.f / scale, false);
            } else if (otype == "random_points") {   // debug: drawn below, pair by pair
            } else {
              const std::string base = im["output"].asString() + "_" + key;
              std::string we;
              if (!ofio::write_tiff_f32(base + "_x.tiff", fx.data() + px * b, W, h, 4 * (size_t)W, we) ||
                  !ofio::write_tiff_f32(base + "_y.tiff", fy.data() + px * b, W, h, 4 * (size_t)W, we)) {
                e = we, ok = false;   // an output error, not a device fault
                dc.faulted = false;
              }
            }
          }
          if (otype == "random_points" && !sampled) {
            dbg_fx[kk].swap(fx);
            dbg_fy[kk].swap(fy);
          }
          tm["write_outputs"] += secs_since(ts);
        }
        // hP / hQ are reused page-locked buffers: after a failure the chunk's uploads from
        // them may still be queued, so the stream is drained before the retry or the next
        // chunk refills them (PinnedPool's rule, as solve_rois' SyncOnFailure)
        if (!ok && dc.stream) (void)hipStreamSynchronize(dc.stream);
        if (items.empty()) break;   // handed to the per-pair path
        if (ok && otype == "random_points" && debug) {   // the exact shuffle (random_points)
          for (int b = 0; b < nb; ++b)
            for (size_t kk = 0; kk < roi_keys.size(); ++kk) {
              const ofio::Image8 &a = items[b].p->bands[kk], &c = items[b].q->bands[kk];
              const int W = a.width, h = a.height;
              const size_t px = (size_t)W * h;
              const Rect r{0, roi_keys[kk] == "top" ? 0 : items[b].p->H - h, W, h};
              std::vector<uint8_t> mask(px);
              for (size_t k = 0; k < px; ++k) mask[k] = (a.data[k] > 1) | (c.data[k] > 1);
              random_points(dbg_fx[kk].data() + px * b, dbg_fy[kk].data() + px * b, W, h,
                            items[b].im, args, r, r, mask, false);
            }
        }
        if (ok) {
          ++t_chunks;
          t_pairs += nb;
          for (int b = 0; b < nb; ++b) {
            const size_t i = items[b].i;
            for (auto &sv : solves[b]) results[i].stats["solves"].append(sv);
            if (otype == "random_points") results[i].pms.push_back(move_pm(items[b].im));
            results[i].ok = results[i].done = true;
          }
          break;
        }
        if (attempt == 0 && dc.faulted) {
          {
            std::lock_guard<std::mutex> lk(g_io_mutex);
            fprintf(stderr, "Warning: strip batch of %d pairs (%zu..): %s; retrying on a fresh device context\n",
                    nb, items[0].i, e.c_str());
          }
          for (auto &it : items) {   // the retry starts from the decoded bands again
            it.im = images[it.i];
            it.im["scale"] = it.im.get("scale", (double)scale).asDouble();
            it.im["output"] = it.im.get("output", args["output_dir"].asString() + "/" +
                                                      it.im["output_name"].asString() + "_" + sbuf);
          }
          release();
          close_device(dc);
          std::string e2;
          if (!open_device(dc, device, e2)) {
            e = "device context could not be rebuilt: " + e2;
          } else {
            continue;
          }
        }
        std::lock_guard<std::mutex> lk(g_io_mutex);
        for (auto &it : items) {
          results[it.i].done = true;
          results[it.i].ok = false;
          fprintf(stderr, "Error: pair %zu (%s %s): %s\n", it.i, it.im["p"].asString().c_str(),
                  it.im["q"].asString().c_str(), e.c_str());
        }
        break;
      }
    }
    if (dc.stream) (void)hipStreamSynchronize(dc.stream);
    (void)hipEventDestroy(ev_up0);
    (void)hipEventDestroy(ev_up1);
    release();
    close_device(dc);
    {
      Value w;
      w["device"] = device;
      w["chunks"] = (int64_t)t_chunks;
      w["pairs"] = (int64_t)t_pairs;
      w["worker_s"] = secs_since(t_worker);
      for (auto &kv : tm) w["stage_s"][kv.first] = kv.second;
      std::lock_guard<std::mutex> lk(g_stage_mutex);
      g_stage_workers.append(w);
    }
  };

  // build-only "inflight": pairs solved concurrently per GPU (one worker thread, ctx and
  // stream each) so one pair's residual read-backs overlap another pair's kernels.  Strip
  // jobs (every ROI "top" / "bottom", the production shape: two 100-row strips per pair)
  // are launch- and sync-bound per solve, so they default to 8 in flight, full frames to 3
  // (DESIGN.md 5.1, 9).
  bool strip_job = args.isMember("rois") && args["rois"].isObject() && args["rois"].size() > 0;
  if (strip_job)
    for (auto &k : args["rois"].memberNames()) strip_job = strip_job && (k == "top" || k == "bottom");
  // build-only "strip_batch": strip pairs per tvl1_calc_batch (default 256; 0 or 1 = one
  // tvl1_calc per strip, the r3 path).  A pair is batched when the job's ROIs are all top /
  // bottom and its own keys are only the production ones (gen_cross_file_list.py:47-54);
  // features, per-image ROIs / scales / TV parameters go the per-pair way.
  const int strip_batch = std::min(256, std::max(0, args.get("strip_batch", 256).asInt()));
  const std::string gotype = output_type_of(Value(), args);
  const bool batching = strip_job && strip_batch > 1 && !resolve_features(Value(), args) &&
                        (gotype == "map" || gotype == "flow" || gotype == "random_points");
  if (batching) {
    roi_keys = args["rois"].memberNames();
    roi_top = args["rois"].get("top", 300).asInt();
    roi_bottom = args["rois"].get("bottom", 300).asInt();
    static const char *kProd[] = {"p", "q", "pId", "qId", "pGroupId", "qGroupId", "output_name", "output"};
    for (size_t i = 0; i < n; ++i) {
      bool ok = images[i].isObject();
      for (auto &k : images[i].memberNames())
        ok = ok && std::find_if(std::begin(kProd), std::end(kProd), [&](const char *x) { return k == x; }) !=
                       std::end(kProd);
      (ok ? batched : todo).push_back(i);
      batch_ok[i] = ok;
    }
    if (plan_only) {   // --plan reports the split; the per-pair worker resolves every pair
      batched.clear();
      todo.clear();
      for (size_t i = 0; i < n; ++i) todo.push_back(i);
    }
  } else {
    for (size_t i = 0; i < n; ++i) todo.push_back(i);
  }
  if (!batched.empty()) {
    // "inflight" batches per GPU (default 2: one batch's residual syncs overlap the other's
    // kernels), chunks small enough that every worker gets one
    const int binflight = std::max(1, args.get("inflight", 2).asInt());
    const size_t workers = devices.size() * (size_t)binflight;
    bchunk = std::max<size_t>(1, std::min<size_t>(strip_batch, (batched.size() + workers - 1) / workers));
    std::vector<std::thread> th;
    for (int f = 0; f < binflight; ++f)
      for (int d : devices) th.emplace_back(batch_worker, d);
    for (auto &t : th) t.join();
    for (size_t i = 0; i < n; ++i)
      if (deferred[i]) todo.push_back(i);
    std::sort(todo.begin(), todo.end());
  }
  m = todo.size();
  chunk = std::max<size_t>(1, std::min<size_t>(16, m / std::max<size_t>(1, devices.size() * 4)));
  const int inflight = std::max(1, args.get("inflight", strip_job ? 8 : 3).asInt());
  if (m == 0) {
  } else if (plan_only || (devices.size() == 1 && inflight == 1)) {
    worker(devices[0]);
  } else {
    std::vector<std::thread> th;
    for (int f = 0; f < inflight; ++f)
      for (int d : devices) th.emplace_back(worker, d);
    for (auto &t : th) t.join();
  }
  if (hard_error) return 1;

  if (plan_only) {
    Value out;
    for (auto &p : plans) out.append(p);
    printf("%s\n", out.dump(1).c_str());
    return 0;
  }

  // point-match batching in pair order (optflow.cpp:160-175): the reference PUTs
  // args["point_matches"] every batch_size pairs; here each batch is one JSON file.
  const std::string mfile = args.get("matches_file", args["output_dir"].asString() + "/point_matches").asString();
  const int batch = args.get("batch_size", 100).asInt();
  Value pending;
  bool any_since = false;
  size_t last_upload = 0;
  int nbatch = 0;
  // the batches are grouped in pair order (cheap), then serialised and written on the decode
  // pool in parallel: 40,860 strip pairs' records took 1.6 s on one thread (profiles/r6/cli/)
  std::vector<std::shared_future<void>> writes;
  auto upload = [&]() {
    const std::string owner = args.get("owner", "flyem").asString();
    const std::string mc = args.get("matchCollection", "forgetful_owner").asString();
    const std::string host = args.get("host", "10.40.3.162").asString();
    const std::string port = args.get("port", "8080").asString();
    const std::string url = "http://" + host + ":" + port + "/render-ws/v1/owner/" + owner +
                            "/matchCollection/" + mc + "/matches";
    const std::string path = mfile + "_" + std::to_string(nbatch++) + ".json";
    auto body = std::make_shared<Value>(std::move(pending));
    auto job = [body, path, url, debug] {
      const std::string payload = body->dump(3);
      if (debug) {
        std::lock_guard<std::mutex> lk(g_io_mutex);
        printf("%s\n%s", payload.c_str(), url.c_str());
      }
      FILE *f = fopen(path.c_str(), "w");
      if (!f) {
        std::lock_guard<std::mutex> lk(g_io_mutex);
        fprintf(stderr, "cannot write point matches to %s\n", path.c_str());
        return;
      }
      fprintf(f, "%s\n", payload.c_str());
      fclose(f);
    };
    if (debug) job();   // debug prints the payloads in batch order, as the reference does
    else writes.push_back(pool.submit(job));
  };
  const auto t_records = Clock::now();
  for (size_t i = 0; i < n; ++i) {
    const Value &im = images[i];
    for (auto &pm : results[i].pms) pending.append(pm);
    if (output_type_of(im, args) == "random_points") {
      any_since = true;
      if (i > last_upload + (size_t)batch) {
        upload();
        pending = Value();
        last_upload = i;
        any_since = false;
      }
    }
  }
  if (any_since) upload();
  for (auto &w : writes) w.wait();
  const double records_s = secs_since(t_records);

  if (args.isMember("timing_json")) {   // build-only: per-stage host timing (tools/cli_e2e.py)
    Value t;
    t["wall_s"] = secs_since(g_t0);
    t["pairs"] = (int64_t)n;
    t["decode"]["band_reads"] = (int64_t)g_band_reads.load();
    t["decode"]["band_read_s"] = 1e-9 * (double)g_band_read_ns.load();
    t["decode"]["threads"] = args.get("decode_threads", (int)std::min(16u, hc - 1)).asInt();
    t["point_match_records_s"] = records_s;
    t["batch_workers"] = g_stage_workers.isNull() ? Value() : g_stage_workers;
    FILE *f = fopen(args["timing_json"].asString().c_str(), "w");
    if (f) {
      fprintf(f, "%s\n", t.dump(1).c_str());
      fclose(f);
    }
  }

  if (args.isMember("stats_json")) {
    Value st;
    for (size_t i = 0; i < n; ++i) {
      Value e = results[i].stats;
      e["index"] = (int64_t)i;
      e["ok"] = results[i].ok;
      e["host_pinned_bytes"] = (int64_t)PinnedPool::pinned_bytes();   // process total at exit
      st.append(e);
    }
    FILE *f = fopen(args["stats_json"].asString().c_str(), "w");
    if (f) {
      fprintf(f, "%s\n", st.dump(1).c_str());
      fclose(f);
    }
  }
  if (const char *e = getenv("OPTFLOW_PINNED_TRACE"); e && atoi(e))
    fprintf(stderr, "%s\n", PinnedPool::summary().c_str());
  return 0;  // like the reference: per-pair failures are reported, exit status 0
}

static void usage() {
  printf("Usage: optflow [--plan] <config.json[.gz]>\n"
         "       optflow --decode <image> <out.tiff> [scale]\n"
         "  Dense TV-L1 optical flow for FIB-SEM slice pairs on AMD MI355X (gfx950).\n"
         "  --plan    resolve the config (pairs, ROIs, output files, TV-L1 parameters)\n"
         "            and print it as JSON without touching the GPU.\n"
         "  --decode  read an image as the pair loop does (IMREAD_GRAYSCALE + optional\n"
         "            cv::resize pre-scale) and write it as an 8-bit TIFF.\n");
}

int main(int argc, const char *argv[]) {
  bool plan = false;
  std::string filename;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "-h" || a == "--help") {
      usage();
      return 0;
    }
    if (a == "--plan") {
      plan = true;
      continue;
    }
    if (a == "--decode-bands") {   // tests: the ROI-limited read of strip jobs
      // optflow --decode-bands <image> <out.tiff> <scale> <top> <bottom>: the top and bottom
      // row bands of the pre-scaled slice (get_rois' top / bottom), stacked, as an 8-bit TIFF;
      // stdout says whether only their rows were read
      if (i + 5 >= argc) {
        usage();
        return 2;
      }
      const float sc = (float)atof(argv[i + 3]);
      const int top = atoi(argv[i + 4]), bottom = atoi(argv[i + 5]);
      int W = 0, H = 0;
      bool partial = false;
      std::vector<ofio::Image8> bands;
      std::string err;
      if (!ofio::read_gray8_bands(argv[i + 1], sc,
                                  [&](int, int h) {
                                    return std::vector<std::pair<int, int>>{{0, top}, {h - bottom, h}};
                                  },
                                  W, H, bands, err, &partial)) {
        fprintf(stderr, "%s\n", err.c_str());
        return 1;
      }
      ofio::Image8 out;
      out.width = W;
      out.height = bands[0].height + bands[1].height;
      out.data.resize((size_t)W * out.height);
      memcpy(out.data.data(), bands[0].data.data(), bands[0].data.size());
      memcpy(out.data.data() + bands[0].data.size(), bands[1].data.data(), bands[1].data.size());
      if (!ofio::write_tiff_u8(argv[i + 2], out, err)) {
        fprintf(stderr, "%s\n", err.c_str());
        return 1;
      }
      printf("%dx%d %s\n", W, H, partial ? "partial" : "whole");
      return 0;
    }
    if (a == "--decode") {
      if (i + 2 >= argc) {
        usage();
        return 2;
      }
      ofio::Image8 img, out;
      std::string err;
      if (!ofio::read_gray8(argv[i + 1], img, err)) {
        fprintf(stderr, "%s\n", err.c_str());
        return 1;
      }
      const double sc = i + 3 < argc ? atof(argv[i + 3]) : 1.0;
      if (sc != 1.0) ofio::resize_u8(img, (float)sc, (float)sc, out);
      else out = img;
      if (!ofio::write_tiff_u8(argv[i + 2], out, err)) {
        fprintf(stderr, "%s\n", err.c_str());
        return 1;
      }
      return 0;
    }
    filename = a;
  }
  if (filename.empty()) {
    usage();
    return 2;
  }
  std::string text, err;
  if (!ofio::read_file(filename, text, err, true)) {
    fprintf(stderr, "%s\n", err.c_str());
    return 2;
  }
  Value args;
  try {
    args = ofjson::parse(text);
  } catch (const std::exception &e) {
    fprintf(stderr, "%s: %s\n", filename.c_str(), e.what());
    return 2;
  }
  int rc = 0;
  const int style = args.get("style", 1).asInt();
  if (style == 1) {
    try {
      rc = from_file(args, plan);
    } catch (const std::exception &e) {
      fprintf(stderr, "error: %s\n", e.what());
      rc = 2;
    }
  } else {
    fprintf(stderr, "style %d is not implemented (only style 1, optflow.cpp:62-66)\n", style);
    rc = 2;
  }
  return rc;
}
