// imageio.hpp — host-side image I/O of the optflow CLI (no OpenCV, no libpng/libtiff).
//
// Restates what the reference gets from OpenCV's imgcodecs/imgproc on the host
// (/root/reference/src/optflow.cpp):
//   cv::imread(path, IMREAD_GRAYSCALE)            :106, :119  -> read_gray8()
//   cv::resize(frame, frame, Size(), scale, scale) :113, :125  -> resize_u8()
//   cv::imwrite(file, CV_32FC1 flow)               :482-483    -> write_tiff_f32()
// Formats: PNG (gray/RGB/RGBA/palette, 1-16 bit, non-interlaced), baseline TIFF
// (uncompressed, LZW or deflate; 8/16-bit; 1 or 3 samples), binary PGM (P5).
// OpenCV's exact colour-to-gray and 16->8-bit conversions are restated from its
// published sources and are NOT verifiable here (OpenCV is absent):
// FIB-SEM slices are 8-bit grayscale, for which decoding is exact.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <new>
#include <string>
#include <utility>
#include <vector>

namespace ofio {

// Host storage of images and flow fields.  By default operator new; the CLI installs a
// page-locked pool (hipHostMalloc) so that decoded slices are uploaded by one DMA straight
// from the buffer the decoder wrote, and flow fields download likewise (optflow.cpp:315-316
// GpuMat::upload).  Install before any image is allocated; release() gets
// back exactly the pointers alloc() returned.
struct HostAllocHooks {
  void *(*alloc)(size_t bytes);
  void (*release)(void *p, size_t bytes);
};
void set_host_alloc(const HostAllocHooks &h);
void *host_alloc(size_t bytes);
void host_release(void *p, size_t bytes);

template <class T>
struct HostAlloc {
  using value_type = T;
  HostAlloc() = default;
  template <class U>
  HostAlloc(const HostAlloc<U> &) {}
  T *allocate(size_t n) {
    if (n > (size_t)-1 / sizeof(T)) throw std::bad_alloc();
    void *p = host_alloc(n * sizeof(T));
    if (!p) throw std::bad_alloc();
    return static_cast<T *>(p);
  }
  void deallocate(T *p, size_t n) { host_release(p, n * sizeof(T)); }
  // resize() default-initialises (no zero fill): every decoder writes each pixel it sizes
  template <class U>
  void construct(U *p) noexcept {
    ::new (static_cast<void *>(p)) U;
  }
  template <class U, class... A>
  void construct(U *p, A &&...a) {
    ::new (static_cast<void *>(p)) U(std::forward<A>(a)...);
  }
  template <class U>
  bool operator==(const HostAlloc<U> &) const { return true; }
  template <class U>
  bool operator!=(const HostAlloc<U> &) const { return false; }
};
template <class T>
using HostVec = std::vector<T, HostAlloc<T>>;

struct Image8 {
  int width = 0, height = 0;
  HostVec<uint8_t> data;  // row-major, pitch == width
  uint8_t *row(int y) { return data.data() + (size_t)y * width; }
  const uint8_t *row(int y) const { return data.data() + (size_t)y * width; }
};

// Read a whole file; a ".gz" suffix is gunzipped (boost gzip_decompressor at
// optflow.cpp:43-52).  Returns false and sets err on failure.
bool read_file(const std::string &path, std::string &out, std::string &err, bool gunzip_if_gz);

// cv::imread(path, IMREAD_GRAYSCALE).  Returns false (empty image) on failure,
// which the caller reports like optflow.cpp:108-112.
bool read_gray8(const std::string &path, Image8 &img, std::string &err);

// cv::resize(src, dst, Size(), fx, fy, INTER_LINEAR) for CV_8UC1 on the CPU:
// dst size = round(src * f) (half-even); an exact 1/2 scale takes OpenCV's
// INTER_AREA fast path (2x2 mean), other scales half-pixel-centre bilinear with
// 11-bit fixed-point weights.
void resize_u8(const Image8 &src, double fx, double fy, Image8 &dst);

// Size of cv::resize's output (round half-even of src * f).
void resized_size(int sw, int sh, double fx, double fy, int &dw, int &dh);
// The source rows [sy0, sy1) that output rows [dy0, dy1) of resize_u8 read.
void resize_src_rows(int sw, int sh, double fx, double fy, int dy0, int dy1, int &sy0, int &sy1);

// Row bands of read_gray8 + resize_u8(scale) without decoding what they do not need (the
// production strip jobs solve two ~100-row ROIs of each slice).  bands_of gets
// the pre-scaled image size (W, H) and returns the bands [y0, y1) wanted; out[i] holds band
// i, byte-identical to those rows of the whole decoded and resized image.  Strip-organised
// 8-bit gray TIFF (uncompressed: only the rows' bytes; LZW / deflate: only their strips) is
// read by pread; any other file is decoded whole first.  *partial says which happened.
bool read_gray8_bands(const std::string &path, double scale,
                      const std::function<std::vector<std::pair<int, int>>(int, int)> &bands_of,
                      int &W, int &H, std::vector<Image8> &out, std::string &err,
                      bool *partial = nullptr);

// Single-channel float32 TIFF (uncompressed, SampleFormat=IEEE float).
bool write_tiff_f32(const std::string &path, const float *data, int width, int height,
                    size_t pitch_bytes, std::string &err);
// Single-channel 8-bit TIFF (uncompressed).
bool write_tiff_u8(const std::string &path, const Image8 &img, std::string &err);

}  // namespace ofio
