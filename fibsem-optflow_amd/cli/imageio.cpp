// imageio.cpp — see imageio.hpp.
#include "imageio.hpp"

#include <dlfcn.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <fstream>
#include <sstream>

namespace ofio {

namespace {
void *default_alloc(size_t n) { return ::operator new(n, std::nothrow); }
void default_release(void *p, size_t) { ::operator delete(p); }
HostAllocHooks g_hooks{default_alloc, default_release};
}  // namespace

void set_host_alloc(const HostAllocHooks &h) { g_hooks = h; }
void *host_alloc(size_t bytes) { return g_hooks.alloc(bytes); }
void host_release(void *p, size_t bytes) { g_hooks.release(p, bytes); }

// The largest image a decoder accepts: the solver's limit (tvl1_calc: W * H <= 2^31).
constexpr uint64_t kMaxPixels = (uint64_t)1 << 31;

// ------------------------------------------------------------------ files
bool read_file(const std::string &path, std::string &out, std::string &err, bool gunzip_if_gz) {
  out.clear();
  const bool gz = gunzip_if_gz && path.size() >= 3 && path.compare(path.size() - 3, 3, ".gz") == 0;
  if (gz) {
    gzFile f = gzopen(path.c_str(), "rb");
    if (!f) {
      err = "cannot open " + path;
      return false;
    }
    char buf[1 << 16];
    int n;
    while ((n = gzread(f, buf, sizeof buf)) > 0) out.append(buf, (size_t)n);
    const bool bad = n < 0;
    gzclose(f);
    if (bad) {
      err = "gzip error reading " + path;
      return false;
    }
    return true;
  }
  FILE *f = fopen(path.c_str(), "rb");
  if (!f) {
    err = "cannot open " + path;
    return false;
  }
  // one sized read (an ostringstream copy cost ~10 ms per 25-MB slice)
  bool ok = fseek(f, 0, SEEK_END) == 0;
  const long size = ok ? ftell(f) : -1;
  ok = ok && size >= 0 && fseek(f, 0, SEEK_SET) == 0;
  if (ok) {
    out.resize((size_t)size);
    ok = fread(&out[0], 1, out.size(), f) == out.size();
  }
  fclose(f);
  if (!ok) {
    err = "cannot read " + path;
    return false;
  }
  return true;
}

static inline uint32_t be32(const uint8_t *p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

// libpng png_set_rgb_to_gray(png, 1, 0.299, 0.587) as OpenCV's PNG decoder requests
// for IMREAD_GRAYSCALE: 15-bit fixed-point coefficients.
static inline uint8_t rgb_to_gray_png(unsigned r, unsigned g, unsigned b) {
  if (r == g && r == b) return (uint8_t)r;
  const unsigned rc = 9798, gc = 19235, bc = 32768 - 9798 - 19235;
  return (uint8_t)((rc * r + gc * g + bc * b + 16384) >> 15);
}

// ------------------------------------------------------------------ PNG
// Inflate: libdeflate's whole-buffer zlib decoder when the image has it (≈2x zlib's
// streaming inflate on these slices; loaded with dlopen, so a system without it simply
// uses zlib), zlib otherwise and whenever libdeflate rejects the stream.
namespace {
struct Libdeflate {
  void *(*alloc)() = nullptr;
  int (*zlib_decompress)(void *, const void *, size_t, void *, size_t, size_t *) = nullptr;
  void (*release)(void *) = nullptr;
  Libdeflate() {
    if (getenv("OPTFLOW_NO_LIBDEFLATE")) return;   // force the zlib path (tests)
    void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    alloc = (void *(*)())dlsym(h, "libdeflate_alloc_decompressor");
    zlib_decompress = (int (*)(void *, const void *, size_t, void *, size_t, size_t *))dlsym(
        h, "libdeflate_zlib_decompress");
    release = (void (*)(void *))dlsym(h, "libdeflate_free_decompressor");
    if (!alloc || !zlib_decompress || !release) alloc = nullptr;
  }
};
const Libdeflate &libdeflate() {
  static const Libdeflate l;
  return l;
}
struct Decompressor {   // one per decoding thread
  void *d = nullptr;
  ~Decompressor() {
    if (d) libdeflate().release(d);
  }
};

bool inflate_all(const std::vector<uint8_t> &in, std::vector<uint8_t> &out) {
  const Libdeflate &L = libdeflate();
  if (L.alloc) {
    thread_local Decompressor dc;
    if (!dc.d) dc.d = L.alloc();
    size_t got = 0;
    if (dc.d && L.zlib_decompress(dc.d, in.data(), in.size(), out.data(), out.size(), &got) == 0 &&
        got == out.size())
      return true;
  }
  z_stream zs;
  memset(&zs, 0, sizeof zs);
  if (inflateInit(&zs) != Z_OK) return false;
  zs.next_in = (Bytef *)in.data();
  zs.avail_in = (uInt)in.size();
  zs.next_out = out.data();
  zs.avail_out = (uInt)out.size();
  const int zr = inflate(&zs, Z_FINISH);
  inflateEnd(&zs);
  return !(zr != Z_STREAM_END && zs.avail_out != 0);
}
}  // namespace

// One Paeth-filtered byte (bpp 1): a = left, b = up, c = up-left (PNG specification 9.4).
static inline uint8_t paeth_byte(uint8_t in, int a, int b, int c) {
  const int pa = abs(b - c), pb = abs(a - c), pc = abs(a + b - 2 * c);
  const int bc = pb <= pc ? b : c;
  return (uint8_t)(in + ((pa <= pb) & (pa <= pc) ? a : bc));
}

// Unfilter 4 consecutive Paeth rows of an 8-bit gray image: raw = the first row's filter
// byte (rows of n + 1 bytes), prev = the row above (zeros for the first), out = 4 rows of
// n bytes.  Row k runs one column behind row k-1, so at each step the 4 chains are
// independent; every byte gets the same operations as the one-row loop.
static void paeth4(const uint8_t *raw, size_t n, const uint8_t *prev, uint8_t *out) {
  const uint8_t *in[4];
  const uint8_t *up[4];
  uint8_t *o[4];
  for (int k = 0; k < 4; ++k) {
    in[k] = raw + k * (n + 1) + 1;
    o[k] = out + k * n;
    up[k] = k == 0 ? prev : out + (k - 1) * n;
  }
  // x = 0: Paeth(0, b, 0) = b; row k's column 0 needs row k-1's column 0 only
  int a[4];
  auto step = [&](int k, size_t x) {
    a[k] = paeth_byte(in[k][x], a[k], up[k][x], up[k][x - 1]);
    o[k][x] = (uint8_t)a[k];
  };
  // prologue: steps t = 0..2 (row k at x = t - k)
  for (int t = 0; t < 3; ++t)
    for (int k = 0; k <= t; ++k) {
      const size_t x = (size_t)(t - k);
      if (x == 0) {
        a[k] = (uint8_t)(in[k][0] + up[k][0]);
        o[k][0] = (uint8_t)a[k];
      } else {
        step(k, x);
      }
    }
  for (size_t t = 3; t < n; ++t) {   // all 4 rows active, row 3 at x = t - 3 >= 0... >= 1 here
    if (t == 3) {
      step(0, 3);
      step(1, 2);
      step(2, 1);
      a[3] = (uint8_t)(in[3][0] + up[3][0]);
      o[3][0] = (uint8_t)a[3];
      continue;
    }
    step(0, t);
    step(1, t - 1);
    step(2, t - 2);
    step(3, t - 3);
  }
  // epilogue: rows 1..3 finish their last columns
  for (size_t t = n; t < n + 3; ++t)
    for (int k = (int)(t - n) + 1; k < 4; ++k) step(k, t - k);
}

#ifdef OFIO_TIMING
double ofio_t_inflate = 0, ofio_t_unfilter = 0, ofio_t_chunks = 0;
#define OFIO_NOW() std::chrono::steady_clock::now()
#define OFIO_ADD(v, a, b) v += std::chrono::duration<double>((b) - (a)).count()
#else
#define OFIO_NOW() 0
#define OFIO_ADD(v, a, b) (void)0
#endif

static bool decode_png(const std::string &buf, Image8 &img, std::string &err) {
  [[maybe_unused]] auto tc0 = OFIO_NOW();
  const uint8_t *p = (const uint8_t *)buf.data();
  const size_t n = buf.size();
  size_t off = 8;
  uint32_t W = 0, H = 0;
  int depth = 0, ctype = -1, interlace = 0;
  // the concatenated IDAT stream and the inflated rows live in per-thread buffers reused
  // from slice to slice (a fresh 25 MB vector per slice costs its page faults + zero fill)
  thread_local std::vector<uint8_t> idat;
  idat.clear();
  std::vector<uint8_t> plte;
  while (off + 12 <= n) {
    const uint32_t len = be32(p + off);
    const char *type = (const char *)p + off + 4;
    if (off + 12 + (size_t)len > n) break;
    const uint8_t *d = p + off + 8;
    if (!memcmp(type, "IHDR", 4) && len >= 13) {
      W = be32(d);
      H = be32(d + 4);
      depth = d[8];
      ctype = d[9];
      interlace = d[12];
    } else if (!memcmp(type, "PLTE", 4)) {
      plte.assign(d, d + len);
    } else if (!memcmp(type, "IDAT", 4)) {
      idat.insert(idat.end(), d, d + len);
    } else if (!memcmp(type, "IEND", 4)) {
      break;
    }
    off += 12 + (size_t)len;
  }
  if (!W || !H || ctype < 0) {
    err = "PNG: missing IHDR";
    return false;
  }
  if (interlace) {
    err = "PNG: interlaced images are not supported";
    return false;
  }
  int ch;
  bool depth_ok;   // the PNG specification's allowed bit depths per colour type
  switch (ctype) {
    case 0: ch = 1; depth_ok = depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16; break;
    case 2: ch = 3; depth_ok = depth == 8 || depth == 16; break;
    case 3: ch = 1; depth_ok = depth == 1 || depth == 2 || depth == 4 || depth == 8; break;
    case 4: ch = 2; depth_ok = depth == 8 || depth == 16; break;
    case 6: ch = 4; depth_ok = depth == 8 || depth == 16; break;
    default: err = "PNG: bad colour type"; return false;
  }
  if (!depth_ok) {
    err = "PNG: bit depth " + std::to_string(depth) + " is not valid for colour type " +
          std::to_string(ctype);
    return false;
  }
  // dimensions: at most 2^31 - 1 each (PNG), and an image the solver can take
  if (W > 0x7fffffffu || H > 0x7fffffffu || (uint64_t)W * H > kMaxPixels) {
    err = "PNG: image too large (" + std::to_string(W) + "x" + std::to_string(H) + ")";
    return false;
  }
  const size_t rowbytes = ((size_t)W * ch * depth + 7) / 8;
  const size_t bpp = std::max<size_t>(1, (size_t)ch * depth / 8);
  thread_local std::vector<uint8_t> raw;
  raw.resize((rowbytes + 1) * H);
  [[maybe_unused]] auto tc1 = OFIO_NOW();
  OFIO_ADD(ofio_t_chunks, tc0, tc1);
  if (!inflate_all(idat, raw)) {
    err = "PNG: corrupt image data";
    return false;
  }
  [[maybe_unused]] auto tc2 = OFIO_NOW();
  OFIO_ADD(ofio_t_inflate, tc1, tc2);
  (void)tc2;
  // unfilter (each row: 1 filter byte + rowbytes), one tight loop per filter type; 8-bit
  // gray rows unfilter straight into the image
  const bool gray8 = ctype == 0 && depth == 8;
  std::vector<uint8_t> px(gray8 ? 0 : (size_t)rowbytes * H);
  if (gray8) {
    img.width = (int)W;
    img.height = (int)H;
    img.data.resize((size_t)W * H);
  }
  std::vector<uint8_t> zero(rowbytes, 0);
  for (uint32_t y = 0; y < H;) {
    // 8-bit gray, 4 consecutive Paeth rows (the usual encoder choice for these slices): the
    // per-byte chain through the left neighbour is serial within a row, so the 4 rows are
    // unfiltered together, row k one column behind row k-1 (it needs row k-1's bytes at x
    // and x-1): 4 independent chains per step instead of one.
    if (gray8 && bpp == 1 && rowbytes >= 8 && y + 4 <= H && raw[y * (rowbytes + 1)] == 4 &&
        raw[(y + 1) * (rowbytes + 1)] == 4 && raw[(y + 2) * (rowbytes + 1)] == 4 &&
        raw[(y + 3) * (rowbytes + 1)] == 4) {
      paeth4(raw.data() + (size_t)y * (rowbytes + 1), rowbytes,
             y == 0 ? zero.data() : img.row((int)y - 1), img.row((int)y));
      y += 4;
      continue;
    }
    const uint8_t f = raw[y * (rowbytes + 1)];
    const uint8_t *in = raw.data() + y * (rowbytes + 1) + 1;
    uint8_t *out = gray8 ? img.row((int)y) : px.data() + (size_t)y * rowbytes;
    const uint8_t *prev = y == 0 ? zero.data() : (gray8 ? img.row((int)y - 1) : out - rowbytes);
    const size_t lead = std::min(bpp, rowbytes);
    switch (f) {
      case 0:
        memcpy(out, in, rowbytes);
        break;
      case 1:
        memcpy(out, in, lead);
        for (size_t i = lead; i < rowbytes; ++i) out[i] = (uint8_t)(in[i] + out[i - bpp]);
        break;
      case 2:
        for (size_t i = 0; i < rowbytes; ++i) out[i] = (uint8_t)(in[i] + prev[i]);
        break;
      case 3:
        for (size_t i = 0; i < lead; ++i) out[i] = (uint8_t)(in[i] + (prev[i] >> 1));
        for (size_t i = lead; i < rowbytes; ++i)
          out[i] = (uint8_t)(in[i] + ((unsigned)out[i - bpp] + prev[i]) / 2);
        break;
      case 4:
        for (size_t i = 0; i < lead; ++i) out[i] = (uint8_t)(in[i] + prev[i]);   // Paeth(0, b, 0) = b
        if (bpp == 1) {   // the serial chain runs through a: keep it in a register, no branches
          int a = out[0];
          for (size_t i = 1; i < rowbytes; ++i) {
            const int b = prev[i], c = prev[i - 1];
            const int pa = abs(b - c), pb = abs(a - c), pc = abs(a + b - 2 * c);
            const int bc = pb <= pc ? b : c;
            a = (uint8_t)(in[i] + ((pa <= pb) & (pa <= pc) ? a : bc));
            out[i] = (uint8_t)a;
          }
        } else {
          for (size_t i = lead; i < rowbytes; ++i) {
            const int a = out[i - bpp], b = prev[i], c = prev[i - bpp];
            const int pa = abs(b - c), pb = abs(a - c), pc = abs(a + b - 2 * c);
            const int pr = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
            out[i] = (uint8_t)(in[i] + pr);
          }
        }
        break;
      default:
        err = "PNG: bad filter type";
        return false;
    }
    ++y;
  }
  OFIO_ADD(ofio_t_unfilter, tc2, OFIO_NOW());
  if (gray8) return true;
  img.width = (int)W;
  img.height = (int)H;
  img.data.assign((size_t)W * H, 0);
  auto sample = [&](const uint8_t *row, uint32_t x, int c) -> unsigned {
    // returns an 8-bit sample (16-bit: high byte = png_set_strip_16)
    const size_t idx = (size_t)x * ch + c;
    if (depth == 8) return row[idx];
    if (depth == 16) return row[2 * idx];
    const size_t bit = idx * depth;
    const unsigned v = (row[bit / 8] >> (8 - depth - (bit % 8))) & ((1u << depth) - 1);
    return v;
  };
  for (uint32_t y = 0; y < H; ++y) {
    const uint8_t *row = px.data() + (size_t)y * rowbytes;
    uint8_t *o = img.row((int)y);
    for (uint32_t x = 0; x < W; ++x) {
      switch (ctype) {
        case 0:
        case 4: {
          unsigned v = sample(row, x, 0);
          if (depth < 8) v = v * (255u / ((1u << depth) - 1));  // expand_gray_1_2_4_to_8
          o[x] = (uint8_t)v;
          break;
        }
        case 3: {
          const unsigned i = sample(row, x, 0);
          if ((size_t)i * 3 + 2 >= plte.size()) {
            err = "PNG: palette index out of range";
            return false;
          }
          o[x] = rgb_to_gray_png(plte[i * 3], plte[i * 3 + 1], plte[i * 3 + 2]);
          break;
        }
        default:
          o[x] = rgb_to_gray_png(sample(row, x, 0), sample(row, x, 1), sample(row, x, 2));
      }
    }
  }
  return true;
}

// ------------------------------------------------------------------ TIFF
namespace {
struct TiffReader {
  const uint8_t *p;
  size_t n;
  bool le;
  uint16_t u16(size_t o) const {
    if (o + 2 > n) return 0;
    return le ? (uint16_t)(p[o] | p[o + 1] << 8) : (uint16_t)(p[o] << 8 | p[o + 1]);
  }
  uint32_t u32(size_t o) const {
    if (o + 4 > n) return 0;
    return le ? (uint32_t)p[o] | (uint32_t)p[o + 1] << 8 | (uint32_t)p[o + 2] << 16 |
                    (uint32_t)p[o + 3] << 24
              : (uint32_t)p[o] << 24 | (uint32_t)p[o + 1] << 16 | (uint32_t)p[o + 2] << 8 | p[o + 3];
  }
};

bool lzw_decode(const uint8_t *in, size_t n, std::vector<uint8_t> &out, size_t expect) {
  struct Ent {
    int prefix;
    uint8_t first, last;
    int len;
  };
  std::vector<Ent> tab(4096);
  auto reset = [&]() {
    for (int i = 0; i < 256; ++i) tab[i] = {-1, (uint8_t)i, (uint8_t)i, 1};
  };
  reset();
  int next = 258, width = 9, old = -1;
  size_t bitpos = 0;
  auto read = [&](int w) -> int {
    if (bitpos + w > n * 8) return 257;
    int v = 0;
    for (int i = 0; i < w; ++i, ++bitpos) v = (v << 1) | ((in[bitpos >> 3] >> (7 - (bitpos & 7))) & 1);
    return v;
  };
  auto emit = [&](int code) {
    const size_t start = out.size();
    out.resize(start + tab[code].len);
    int c = code;
    for (int i = tab[code].len - 1; i >= 0; --i) {
      out[start + i] = tab[c].last;
      c = tab[c].prefix;
    }
  };
  while (out.size() < expect) {
    int code = read(width);
    if (code == 257) break;
    if (code == 256) {
      reset();
      next = 258;
      width = 9;
      code = read(width);
      if (code == 257) break;
      if (code > 255) return false;
      emit(code);
      old = code;
      continue;
    }
    if (old < 0) return false;
    if (code < next) {
      emit(code);
      if (next < 4096) tab[next] = {old, tab[old].first, tab[code].first, tab[old].len + 1}, ++next;
    } else if (code == next) {
      if (next < 4096) tab[next] = {old, tab[old].first, tab[old].first, tab[old].len + 1}, ++next;
      emit(code);
    } else {
      return false;
    }
    old = code;
    if (next >= (1 << width) - 1 && width < 12) ++width;  // TIFF "early change"
  }
  return true;
}
}  // namespace

static bool decode_tiff(const std::string &buf, Image8 &img, std::string &err) {
  TiffReader t{(const uint8_t *)buf.data(), buf.size(), buf[0] == 'I'};
  const uint32_t ifd = t.u32(4);
  const uint16_t nent = t.u16(ifd);
  uint32_t W = 0, H = 0, bps = 8, comp = 1, photo = 1, spp = 1, rps = 0, planar = 1, pred = 1,
           fmt = 1;
  std::vector<uint32_t> offs, cnts;
  // an entry's values; false if they do not fit in the file (a count field of up to 2^32
  // would otherwise allocate that many values)
  auto values = [&](size_t e, std::vector<uint32_t> &v) {
    const uint16_t type = t.u16(e + 2);
    const uint32_t cnt = t.u32(e + 4);
    const size_t sz = type == 3 ? 2 : 4;
    const size_t base = (size_t)cnt * sz <= 4 ? e + 8 : t.u32(e + 8);
    if (base > t.n || (size_t)cnt * sz > t.n - base) return false;
    v.resize(cnt);
    for (uint32_t i = 0; i < cnt; ++i) v[i] = sz == 2 ? t.u16(base + i * 2) : t.u32(base + i * 4);
    return true;
  };
  if ((size_t)ifd + 2 + (size_t)nent * 12 > t.n) {
    err = "TIFF: IFD out of range";
    return false;
  }
  for (uint16_t i = 0; i < nent; ++i) {
    const size_t e = ifd + 2 + (size_t)i * 12;
    const uint16_t tag = t.u16(e);
    std::vector<uint32_t> v;
    if (!values(e, v)) {
      err = "TIFF: tag " + std::to_string(tag) + " values out of range";
      return false;
    }
    const uint32_t v0 = v.empty() ? 0 : v[0];
    switch (tag) {
      case 256: W = v0; break;
      case 257: H = v0; break;
      case 258: bps = v0; break;
      case 259: comp = v0; break;
      case 262: photo = v0; break;
      case 273: offs = v; break;
      case 277: spp = v0; break;
      case 278: rps = v0; break;
      case 279: cnts = v; break;
      case 284: planar = v0; break;
      case 317: pred = v0; break;
      case 339: fmt = v0; break;
      default: break;
    }
  }
  if (!W || !H || offs.empty() || offs.size() != cnts.size()) {
    err = "TIFF: unsupported layout (need strips)";
    return false;
  }
  if ((bps != 8 && bps != 16) || fmt == 3 || (spp != 1 && spp != 3 && spp != 4) || planar != 1) {
    err = "TIFF: only 8/16-bit integer, 1/3/4 samples, chunky layout supported";
    return false;
  }
  if ((uint64_t)W * H > kMaxPixels) {
    err = "TIFF: image too large (" + std::to_string(W) + "x" + std::to_string(H) + ")";
    return false;
  }
  if (!rps) rps = H;
  const size_t bytes_pp = (size_t)spp * bps / 8;
  const size_t rowbytes = (size_t)W * bytes_pp;
  std::vector<uint8_t> px;
  px.reserve(rowbytes * H);
  for (size_t s = 0; s < offs.size(); ++s) {
    if ((size_t)offs[s] + cnts[s] > t.n) {
      err = "TIFF: strip out of range";
      return false;
    }
    const uint8_t *src = t.p + offs[s];
    const size_t rows = std::min<size_t>(rps, H - std::min<size_t>(H, s * rps));
    const size_t expect = rows * rowbytes;
    std::vector<uint8_t> strip;
    if (comp == 1) {
      strip.assign(src, src + std::min<size_t>(cnts[s], expect));
    } else if (comp == 5) {
      if (!lzw_decode(src, cnts[s], strip, expect)) {
        err = "TIFF: corrupt LZW strip";
        return false;
      }
    } else if (comp == 8 || comp == 32946) {
      strip.resize(expect);
      uLongf dl = (uLongf)expect;
      if (uncompress(strip.data(), &dl, src, cnts[s]) != Z_OK) {
        err = "TIFF: corrupt deflate strip";
        return false;
      }
    } else if (comp == 32773) {  // PackBits
      size_t i = 0;
      while (i < cnts[s] && strip.size() < expect) {
        const int8_t c = (int8_t)src[i++];
        if (c >= 0) {
          strip.insert(strip.end(), src + i, src + std::min<size_t>(cnts[s], i + c + 1));
          i += c + 1;
        } else if (c != -128) {
          if (i < cnts[s]) strip.insert(strip.end(), (size_t)(1 - c), src[i]);
          ++i;
        }
      }
    } else {
      err = "TIFF: unsupported compression " + std::to_string(comp);
      return false;
    }
    strip.resize(expect, 0);
    if (pred == 2) {  // horizontal differencing
      for (size_t r = 0; r < rows; ++r) {
        uint8_t *row = strip.data() + r * rowbytes;
        if (bps == 8) {
          for (size_t i = spp; i < rowbytes; ++i) row[i] = (uint8_t)(row[i] + row[i - spp]);
        } else {
          for (size_t i = spp; i < (size_t)W * spp; ++i) {
            const size_t a = 2 * i, b = 2 * (i - spp);
            uint16_t cur = t.le ? (uint16_t)(row[a] | row[a + 1] << 8) : (uint16_t)(row[a] << 8 | row[a + 1]);
            const uint16_t pv = t.le ? (uint16_t)(row[b] | row[b + 1] << 8) : (uint16_t)(row[b] << 8 | row[b + 1]);
            cur = (uint16_t)(cur + pv);
            if (t.le) { row[a] = (uint8_t)cur; row[a + 1] = (uint8_t)(cur >> 8); }
            else { row[a] = (uint8_t)(cur >> 8); row[a + 1] = (uint8_t)cur; }
          }
        }
      }
    }
    px.insert(px.end(), strip.begin(), strip.end());
  }
  // fewer strips than ceil(H / RowsPerStrip): the rows below are missing, not zero
  if (px.size() < rowbytes * H) {
    err = "TIFF: strips cover " + std::to_string(rowbytes ? px.size() / rowbytes : 0) + " of " +
          std::to_string(H) + " rows";
    return false;
  }
  img.width = (int)W;
  img.height = (int)H;
  img.data.assign((size_t)W * H, 0);
  if (spp == 1 && bps == 8) {   // 8-bit gray: rows as they are (inverted for WhiteIsZero)
    for (uint32_t y = 0; y < H; ++y) {
      const uint8_t *row = px.data() + (size_t)y * rowbytes;
      uint8_t *o = img.row((int)y);
      if (photo == 0) {
        for (uint32_t x = 0; x < W; ++x) o[x] = (uint8_t)(255 - row[x]);
      } else {
        memcpy(o, row, W);
      }
    }
    return true;
  }
  for (uint32_t y = 0; y < H; ++y) {
    const uint8_t *row = px.data() + (size_t)y * rowbytes;
    uint8_t *o = img.row((int)y);
    for (uint32_t x = 0; x < W; ++x) {
      unsigned s[3];
      for (uint32_t c = 0; c < std::min<uint32_t>(spp, 3); ++c) {
        const size_t i = ((size_t)x * spp + c) * (bps / 8);
        s[c] = bps == 8 ? row[i] : (t.le ? row[i + 1] : row[i]);  // 16-bit: high byte
      }
      unsigned v;
      if (spp == 1) {
        v = s[0];
        if (photo == 0) v = 255 - v;  // WhiteIsZero
      } else {  // cv::cvtColor(RGB2GRAY): 14-bit fixed point
        v = (s[0] * 4899 + s[1] * 9617 + s[2] * 1868 + (1 << 13)) >> 14;
      }
      o[x] = (uint8_t)v;
    }
  }
  return true;
}

// ------------------------------------------------------------------ PGM
static bool decode_pgm(const std::string &buf, Image8 &img, std::string &err) {
  size_t i = 2;
  int vals[3];
  for (int k = 0; k < 3; ++k) {
    while (i < buf.size()) {
      if (buf[i] == '#') {
        while (i < buf.size() && buf[i] != '\n') ++i;
      } else if (isspace((unsigned char)buf[i])) {
        ++i;
      } else {
        break;
      }
    }
    long long v = 0;
    while (i < buf.size() && isdigit((unsigned char)buf[i])) {
      v = v * 10 + (buf[i++] - '0');
      if (v > 0x7fffffff) {
        err = "PGM: header value out of range";
        return false;
      }
    }
    vals[k] = (int)v;
  }
  ++i;
  const int W = vals[0], H = vals[1], maxv = vals[2];
  const size_t bps = maxv > 255 ? 2 : 1;
  if (W <= 0 || H <= 0 || (uint64_t)W * H > kMaxPixels || buf.size() < i + (size_t)W * H * bps) {
    err = "PGM: truncated";
    return false;
  }
  img.width = W;
  img.height = H;
  img.data.resize((size_t)W * H);
  for (size_t k = 0; k < (size_t)W * H; ++k) img.data[k] = (uint8_t)buf[i + k * bps];
  return true;
}

static bool decode_any(const std::string &path, Image8 &img, std::string &err) {
  std::string buf;
  img = Image8();
  if (!read_file(path, buf, err, false)) return false;
  if (buf.size() >= 8 && !memcmp(buf.data(), "\x89PNG\r\n\x1a\n", 8)) return decode_png(buf, img, err);
  if (buf.size() >= 8 && (!memcmp(buf.data(), "II*\0", 4) || !memcmp(buf.data(), "MM\0*", 4)))
    return decode_tiff(buf, img, err);
  if (buf.size() >= 2 && buf[0] == 'P' && buf[1] == '5') return decode_pgm(buf, img, err);
  err = "unsupported image format: " + path;
  return false;
}

// cv::imread returns an empty Mat for any file it cannot decode and the reference skips the
// pair (optflow.cpp:108-112): no decode failure -- an allocation a corrupt header asks for
// included -- may escape as an exception (on a decode-pool thread it would terminate the run).
bool read_gray8(const std::string &path, Image8 &img, std::string &err) {
  try {
    const bool ok = decode_any(path, img, err);
    if (!ok) img = Image8();
    return ok;
  } catch (const std::exception &e) {
    img = Image8();
    err = "cannot decode " + path + ": " + e.what();
    return false;
  }
}

// ------------------------------------------------------------------ resize
static inline int cv_round(double v) { return (int)std::lrint(v); }
static inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// cv::resize on the CPU, output rows [dy0, dy1) only: `row(sy)` gives source row sy and is
// asked only for the rows resize_src_rows() names.  Every output row depends on its own
// source rows alone, so a band computed here is byte-identical to the same rows of the whole
// resized image (read_gray8_bands relies on it).
template <class RowF>
static void resize_rows(RowF row, int sw, int sh, double fx, double fy, int dy0, int dy1,
                        uint8_t *dst) {
  const int dw = cv_round(sw * fx), dh = cv_round(sh * fy);
  if (dw == sw && dh == sh) {
    for (int dy = dy0; dy < dy1; ++dy) memcpy(dst + (size_t)(dy - dy0) * dw, row(dy), dw);
    return;
  }
  const double scale_x = 1. / fx, scale_y = 1. / fy;
  const int iscale_x = cv_round(scale_x), iscale_y = cv_round(scale_y);
  const bool area_fast = std::abs(scale_x - iscale_x) < DBL_EPSILON &&
                         std::abs(scale_y - iscale_y) < DBL_EPSILON;
  if (area_fast && iscale_x == 2 && iscale_y == 2) {
    // INTER_LINEAR at exactly 1/2 -> INTER_AREA fast path: 2x2 mean.  The vector part
    // of OpenCV's 8u kernel rounds (s + 2) >> 2, its scalar tail cvRound(s * 0.25f);
    // partial 2x2 cells at odd borders average the samples that exist.
    const int dwidth1 = sw / 2;
    for (int dy = dy0; dy < dy1; ++dy) {
      uint8_t *D = dst + (size_t)(dy - dy0) * dw;
      const int sy0 = dy * 2;
      if (sy0 >= sh) {
        memset(D, 0, dw);
        continue;
      }
      const int w = sy0 + 2 <= sh ? dwidth1 : 0;
      int dx = 0;
      const uint8_t *S0 = row(sy0);
      const uint8_t *S1 = sy0 + 1 < sh ? row(sy0 + 1) : S0;
      for (; dx + 8 <= w; dx += 8)
        for (int k = dx; k < dx + 8; ++k)
          D[k] = (uint8_t)((S0[2 * k] + S0[2 * k + 1] + S1[2 * k] + S1[2 * k + 1] + 2) >> 2);
      for (; dx < w; ++dx) {
        const int s = S0[2 * dx] + S0[2 * dx + 1] + S1[2 * dx] + S1[2 * dx + 1];
        D[dx] = sat_u8(cv_round((float)s * 0.25f));
      }
      for (; dx < dw; ++dx) {
        int sum = 0, count = 0;
        const int sx0 = dx * 2;
        for (int sy = 0; sy < 2 && sy0 + sy < sh; ++sy)
          for (int sx = 0; sx < 2 && sx0 + sx < sw; ++sx) {
            sum += row(sy0 + sy)[sx0 + sx];
            ++count;
          }
        D[dx] = count ? sat_u8(cv_round((float)sum / count)) : 0;
      }
    }
    return;
  }
  // Generic INTER_LINEAR (resizeGeneric_ with 11-bit fixed-point coefficients).
  constexpr int BITS = 11, SCALE = 1 << BITS;
  std::vector<int> xofs(dw);
  std::vector<short> ax(2 * dw);
  for (int dx = 0; dx < dw; ++dx) {
    float f = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = (int)std::floor(f);
    f -= sx;
    if (sx < 0) {
      f = 0, sx = 0;
    }
    if (sx >= sw - 1) {
      f = 0, sx = sw - 1;
    }
    xofs[dx] = sx;
    ax[2 * dx] = (short)cv_round((1.f - f) * SCALE);
    ax[2 * dx + 1] = (short)(SCALE - ax[2 * dx]);
  }
  std::vector<int> h0(dw), h1(dw);
  auto hres = [&](const uint8_t *S, std::vector<int> &D) {
    for (int dx = 0; dx < dw; ++dx) {
      const int sx = xofs[dx];
      D[dx] = sx + 1 < sw ? S[sx] * ax[2 * dx] + S[sx + 1] * ax[2 * dx + 1] : S[sx] * SCALE;
    }
  };
  for (int dy = dy0; dy < dy1; ++dy) {
    float f = (float)((dy + 0.5) * scale_y - 0.5);
    int sy = (int)std::floor(f);
    f -= sy;
    if (sy < 0) {
      f = 0, sy = 0;
    }
    if (sy >= sh - 1) {
      f = 0, sy = sh - 1;
    }
    const short ay0 = (short)cv_round((1.f - f) * SCALE), ay1 = (short)(SCALE - ay0);
    hres(row(sy), h0);
    hres(row(std::min(sy + 1, sh - 1)), h1);
    uint8_t *D = dst + (size_t)(dy - dy0) * dw;
    for (int dx = 0; dx < dw; ++dx)
      D[dx] = sat_u8((ay0 * h0[dx] + ay1 * h1[dx] + (1 << (2 * BITS - 1))) >> (2 * BITS));
  }
}

void resized_size(int sw, int sh, double fx, double fy, int &dw, int &dh) {
  dw = cv_round(sw * fx);
  dh = cv_round(sh * fy);
}

// The source rows [sy0, sy1) that output rows [dy0, dy1) of resize_rows read.
void resize_src_rows(int sw, int sh, double fx, double fy, int dy0, int dy1, int &sy0, int &sy1) {
  const int dw = cv_round(sw * fx), dh = cv_round(sh * fy);
  sy0 = sh;
  sy1 = 0;
  if (dy1 <= dy0) {
    sy0 = sy1 = 0;
    return;
  }
  if (dw == sw && dh == sh) {
    sy0 = dy0, sy1 = dy1;
    return;
  }
  const double scale_x = 1. / fx, scale_y = 1. / fy;
  const int iscale_x = cv_round(scale_x), iscale_y = cv_round(scale_y);
  if (std::abs(scale_x - iscale_x) < DBL_EPSILON && std::abs(scale_y - iscale_y) < DBL_EPSILON &&
      iscale_x == 2 && iscale_y == 2) {
    sy0 = std::min(2 * dy0, sh);
    sy1 = std::min(2 * dy1, sh);
    if (sy1 <= sy0) sy0 = sy1 = 0;
    return;
  }
  for (int dy : {dy0, dy1 - 1}) {   // sy is monotonic in dy
    float f = (float)((dy + 0.5) * scale_y - 0.5);
    int sy = (int)std::floor(f);
    sy = std::max(0, std::min(sy, sh - 1));
    sy0 = std::min(sy0, sy);
    sy1 = std::max(sy1, std::min(sy + 1, sh - 1) + 1);
  }
}

void resize_u8(const Image8 &src, double fx, double fy, Image8 &dst) {
  Image8 out;
  resized_size(src.width, src.height, fx, fy, out.width, out.height);
  out.data.resize((size_t)out.width * out.height);
  resize_rows([&](int sy) { return src.row(sy); }, src.width, src.height, fx, fy, 0, out.height,
              out.data.data());
  dst = std::move(out);
}

// ------------------------------------------------------------------ row bands
// Strip-organised 8-bit gray TIFF read for only some rows: the header, the IFD and the strip
// tables by pread, then, for uncompressed strips, just the bytes of the rows asked for, and
// for compressed strips just the strips that hold them.  Returns 0 on success, 1 if the file
// is not such a TIFF (the caller decodes it whole), -1 on a read / format error.
namespace {
struct PFile {
  int fd = -1;
  uint64_t size = 0;
  ~PFile() {
    if (fd >= 0) close(fd);
  }
  bool read(uint64_t off, size_t n, void *dst) const {
    if (off > size || n > size - off) return false;
    uint8_t *d = (uint8_t *)dst;
    while (n) {
      const ssize_t r = pread(fd, d, n, (off_t)off);
      if (r <= 0) return false;
      d += r, off += (uint64_t)r, n -= (size_t)r;
    }
    return true;
  }
};
}  // namespace

static int tiff_rows(const std::string &path, int &W, int &H,
                     const std::vector<std::pair<int, int>> &ranges,   // source rows [a, b)
                     std::vector<std::vector<uint8_t>> &rows, std::string &err) {
  PFile f;
  f.fd = open(path.c_str(), O_RDONLY);
  if (f.fd < 0) {
    err = "cannot open " + path;
    return -1;
  }
  struct stat st;
  if (fstat(f.fd, &st) != 0) return 1;
  f.size = (uint64_t)st.st_size;
  uint8_t hdr[8];
  if (!f.read(0, 8, hdr)) return 1;
  const bool le = hdr[0] == 'I';
  if (memcmp(hdr, "II*\0", 4) && memcmp(hdr, "MM\0*", 4)) return 1;
  auto u16 = [&](const uint8_t *q) { return le ? (uint32_t)(q[0] | q[1] << 8) : (uint32_t)(q[0] << 8 | q[1]); };
  auto u32 = [&](const uint8_t *q) {
    return le ? (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24
              : (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | q[3];
  };
  const uint32_t ifd = u32(hdr + 4);
  uint8_t c2[2];
  if (!f.read(ifd, 2, c2)) return 1;
  const uint32_t nent = u16(c2);
  std::vector<uint8_t> ents((size_t)nent * 12);
  if (!f.read((uint64_t)ifd + 2, ents.size(), ents.data())) return 1;
  uint32_t w = 0, h = 0, bps = 8, comp = 1, photo = 1, spp = 1, rps = 0, planar = 1, pred = 1,
           fmt = 1;
  std::vector<uint32_t> offs, cnts;
  auto values = [&](const uint8_t *e, std::vector<uint32_t> &v) {
    const uint32_t type = u16(e + 2), cnt = u32(e + 4);
    const size_t sz = type == 3 ? 2 : 4;
    if ((uint64_t)cnt * sz > f.size) return false;
    std::vector<uint8_t> raw((size_t)cnt * sz);
    if (raw.size() <= 4) memcpy(raw.data(), e + 8, raw.size());
    else if (!f.read(u32(e + 8), raw.size(), raw.data())) return false;
    v.resize(cnt);
    for (uint32_t i = 0; i < cnt; ++i) v[i] = sz == 2 ? u16(&raw[i * 2]) : u32(&raw[i * 4]);
    return true;
  };
  for (uint32_t i = 0; i < nent; ++i) {
    const uint8_t *e = &ents[(size_t)i * 12];
    std::vector<uint32_t> v;
    if (!values(e, v)) return 1;
    const uint32_t v0 = v.empty() ? 0 : v[0];
    switch (u16(e)) {
      case 256: w = v0; break;
      case 257: h = v0; break;
      case 258: bps = v0; break;
      case 259: comp = v0; break;
      case 262: photo = v0; break;
      case 273: offs = v; break;
      case 277: spp = v0; break;
      case 278: rps = v0; break;
      case 279: cnts = v; break;
      case 284: planar = v0; break;
      case 317: pred = v0; break;
      case 339: fmt = v0; break;
      default: break;
    }
  }
  // only the layout this reader covers: 8-bit gray strips, uncompressed / LZW / deflate
  if (!w || !h || bps != 8 || spp != 1 || planar != 1 || fmt == 3 || offs.empty() ||
      offs.size() != cnts.size() || (photo != 0 && photo != 1) ||
      (comp != 1 && comp != 5 && comp != 8 && comp != 32946) || (uint64_t)w * h > kMaxPixels)
    return 1;
  if (!rps || rps > h) rps = h;
  if ((uint64_t)offs.size() * rps < h) return 1;   // whole decode reports the missing rows
  // every strip inside the file, not only the ones the bands need: a truncated or corrupt
  // file takes the whole decode, which reports it, as the per-pair path does
  for (size_t s = 0; s < offs.size(); ++s)
    if ((uint64_t)offs[s] + cnts[s] > f.size) return 1;
  W = (int)w, H = (int)h;
  rows.assign(h, {});
  std::vector<uint8_t> strip;
  long have_strip = -1;
  for (const auto &rg : ranges) {
    for (int y = rg.first; y < rg.second; ++y) {
      if (y < 0 || y >= (int)h || !rows[y].empty()) continue;
      const uint32_t s = (uint32_t)y / rps, r = (uint32_t)y % rps;
      const uint32_t srows = std::min<uint32_t>(rps, h - s * rps);
      std::vector<uint8_t> &o = rows[y];
      o.resize(w);
      if (comp == 1) {
        // uncompressed: the row's bytes where they lie (a short strip reads as zeros, as the
        // whole decode's padding does)
        const uint64_t at = (uint64_t)r * w;
        const uint64_t n = cnts[s] > at ? std::min<uint64_t>(w, cnts[s] - at) : 0;
        memset(o.data(), 0, w);
        if (n && !f.read((uint64_t)offs[s] + at, (size_t)n, o.data())) {
          err = "TIFF: strip out of range";
          return -1;
        }
        if (pred == 2)   // horizontal differencing, per row, as the whole decode applies it
          for (uint32_t i = 1; i < w; ++i) o[i] = (uint8_t)(o[i] + o[i - 1]);
      } else {
        if (have_strip != (long)s) {
          std::vector<uint8_t> src(cnts[s]);
          if (!f.read(offs[s], src.size(), src.data())) {
            err = "TIFF: strip out of range";
            return -1;
          }
          const size_t expect = (size_t)srows * w;
          strip.clear();
          if (comp == 5) {
            if (!lzw_decode(src.data(), src.size(), strip, expect)) {
              err = "TIFF: corrupt LZW strip";
              return -1;
            }
          } else {
            strip.resize(expect);
            uLongf dl = (uLongf)expect;
            if (uncompress(strip.data(), &dl, src.data(), src.size()) != Z_OK) {
              err = "TIFF: corrupt deflate strip";
              return -1;
            }
          }
          strip.resize(expect, 0);
          if (pred == 2)
            for (uint32_t k = 0; k < srows; ++k) {
              uint8_t *q = strip.data() + (size_t)k * w;
              for (uint32_t i = 1; i < w; ++i) q[i] = (uint8_t)(q[i] + q[i - 1]);
            }
          have_strip = (long)s;
        }
        memcpy(o.data(), strip.data() + (size_t)r * w, w);
      }
      if (photo == 0)
        for (auto &b : o) b = (uint8_t)(255 - b);
    }
  }
  return 0;
}

bool read_gray8_bands(const std::string &path, double scale,
                      const std::function<std::vector<std::pair<int, int>>(int, int)> &bands_of,
                      int &W, int &H, std::vector<Image8> &out, std::string &err, bool *partial) {
  out.clear();
  if (partial) *partial = false;
  try {
    // the source rows each band needs, for a source of sw x sh
    auto plan = [&](int sw, int sh, std::vector<std::pair<int, int>> &bands,
                    std::vector<std::pair<int, int>> &src) {
      resized_size(sw, sh, scale, scale, W, H);
      bands = bands_of(W, H);
      src.clear();
      for (auto &b : bands) {
        if (b.first < 0 || b.second > H || b.first >= b.second) {
          err = "row band [" + std::to_string(b.first) + ", " + std::to_string(b.second) +
                ") outside the " + std::to_string(W) + "x" + std::to_string(H) + " image";
          return false;
        }
        int a = 0, z = 0;
        resize_src_rows(sw, sh, scale, scale, b.first, b.second, a, z);
        src.emplace_back(a, z);
      }
      return true;
    };
    std::vector<std::pair<int, int>> bands, src;
    {
      // strip-organised TIFF: only the needed rows leave the file
      int sw = 0, sh = 0;
      std::vector<std::vector<uint8_t>> rows;
      // the header first (sizes), then the rows: tiff_rows is called twice only for the
      // sizes' sake when bands depend on them; one call with every row range would read
      // the strips twice, so the plan is made from the header pass
      std::string e2;
      const int r = tiff_rows(path, sw, sh, {}, rows, e2);
      if (r < 0) {
        err = e2;
        return false;
      }
      if (r == 0) {
        if (!plan(sw, sh, bands, src)) return false;
        if (tiff_rows(path, sw, sh, src, rows, err) != 0) return false;
        for (size_t i = 0; i < bands.size(); ++i) {
          Image8 im;
          im.width = W;
          im.height = bands[i].second - bands[i].first;
          im.data.resize((size_t)im.width * im.height);
          resize_rows([&](int sy) { return (const uint8_t *)rows[sy].data(); }, sw, sh, scale, scale,
                      bands[i].first, bands[i].second, im.data.data());
          out.push_back(std::move(im));
        }
        if (partial) *partial = true;
        return true;
      }
    }
    Image8 full;   // any other file: whole decode, then only the bands' rows are resized
    if (!decode_any(path, full, err)) return false;
    if (!plan(full.width, full.height, bands, src)) return false;
    for (auto &b : bands) {
      Image8 im;
      im.width = W;
      im.height = b.second - b.first;
      im.data.resize((size_t)im.width * im.height);
      resize_rows([&](int sy) { return full.row(sy); }, full.width, full.height, scale, scale,
                  b.first, b.second, im.data.data());
      out.push_back(std::move(im));
    }
    return true;
  } catch (const std::exception &e) {
    out.clear();
    err = "cannot decode " + path + ": " + e.what();
    return false;
  }
}

// ------------------------------------------------------------------ TIFF write
static bool write_tiff(const std::string &path, const void *data, int W, int H, size_t pitch,
                       int bps, int fmt, std::string &err) {
  FILE *f = fopen(path.c_str(), "wb");
  if (!f) {
    err = "cannot write " + path;
    return false;
  }
  const uint32_t rowb = (uint32_t)W * (bps / 8);
  const uint32_t img_bytes = rowb * (uint32_t)H;
  const uint16_t nent = 10;
  const uint32_t ifd_off = 8;
  const uint32_t data_off = ifd_off + 2 + nent * 12 + 4;
  std::vector<uint8_t> h;
  auto p16 = [&](uint16_t v) { h.push_back(v & 0xff); h.push_back(v >> 8); };
  auto p32 = [&](uint32_t v) { for (int i = 0; i < 4; ++i) h.push_back((v >> (8 * i)) & 0xff); };
  auto ent = [&](uint16_t tag, uint16_t type, uint32_t cnt, uint32_t val) {
    p16(tag); p16(type); p32(cnt);
    if (type == 3) { p16((uint16_t)val); p16(0); } else { p32(val); }
  };
  h.insert(h.end(), {'I', 'I', 42, 0});
  p32(ifd_off);
  p16(nent);
  ent(256, 4, 1, (uint32_t)W);        // ImageWidth
  ent(257, 4, 1, (uint32_t)H);        // ImageLength
  ent(258, 3, 1, (uint32_t)bps);      // BitsPerSample
  ent(259, 3, 1, 1);                  // Compression: none
  ent(262, 3, 1, 1);                  // Photometric: BlackIsZero
  ent(273, 4, 1, data_off);           // StripOffsets
  ent(277, 3, 1, 1);                  // SamplesPerPixel
  ent(278, 4, 1, (uint32_t)H);        // RowsPerStrip
  ent(279, 4, 1, img_bytes);          // StripByteCounts
  ent(339, 3, 1, (uint32_t)fmt);      // SampleFormat (1 uint, 3 IEEE float)
  p32(0);                             // next IFD
  bool ok = fwrite(h.data(), 1, h.size(), f) == h.size();
  for (int y = 0; y < H && ok; ++y)
    ok = fwrite((const char *)data + (size_t)y * pitch, 1, rowb, f) == rowb;
  ok = (fclose(f) == 0) && ok;
  if (!ok) err = "short write to " + path;
  return ok;
}

bool write_tiff_f32(const std::string &path, const float *data, int W, int H, size_t pitch,
                    std::string &err) {
  return write_tiff(path, data, W, H, pitch, 32, 3, err);
}

bool write_tiff_u8(const std::string &path, const Image8 &img, std::string &err) {
  return write_tiff(path, img.data.data(), img.width, img.height, (size_t)img.width, 8, 1, err);
}

}  // namespace ofio
