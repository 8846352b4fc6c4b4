// Host decode throughput of the optflow CLI's slice loader (cli/imageio.cpp), no GPU:
// read_gray8 (file read + PNG inflate + unfilter) and resize_u8 (the pre-scale), per slice
// and with T threads over distinct files, so the CLI's production rate can be compared
// with its decode bound.
//   g++ -O3 -std=c++17 -I fibsem-optflow_amd/cli tools/decode_bench.cpp \
//       fibsem-optflow_amd/cli/imageio.cpp -lz -ldl -lpthread -o tools/_bin/decode_bench
//   tools/_bin/decode_bench <threads> <scale> file.png ...
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "imageio.hpp"
#ifdef OFIO_TIMING
namespace ofio { extern double ofio_t_inflate, ofio_t_unfilter, ofio_t_chunks; }
using ofio::ofio_t_inflate; using ofio::ofio_t_unfilter; using ofio::ofio_t_chunks;
#endif

int main(int argc, char **argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s threads scale files...\n", argv[0]);
    return 2;
  }
  const int T = atoi(argv[1]);
  const double scale = atof(argv[2]);
  std::vector<std::string> files(argv + 3, argv + argc);
  using clk = std::chrono::steady_clock;
  // one thread, phase split over the first few files
  double t_dec = 0, t_rs = 0;
  const int n1 = std::min<int>(4, (int)files.size());
  for (int i = 0; i < n1; ++i) {
    ofio::Image8 img, out;
    std::string err;
    auto a = clk::now();
    if (!ofio::read_gray8(files[i], img, err)) {
      fprintf(stderr, "%s: %s\n", files[i].c_str(), err.c_str());
      return 1;
    }
    auto b = clk::now();
    if (scale != 1.0) ofio::resize_u8(img, scale, scale, out);
    auto c = clk::now();
    t_dec += std::chrono::duration<double>(b - a).count();
    t_rs += std::chrono::duration<double>(c - b).count();
  }
  printf("one thread: read_gray8 %.1f ms, resize %.1f ms per slice\n", 1e3 * t_dec / n1,
         1e3 * t_rs / n1);
#ifdef OFIO_TIMING
  printf("  of which: chunks + alloc %.1f ms, inflate %.1f ms, unfilter %.1f ms\n",
         1e3 * ofio_t_chunks / n1, 1e3 * ofio_t_inflate / n1, 1e3 * ofio_t_unfilter / n1);
#endif
  // T threads over every file (each file decoded once)
  std::atomic<size_t> next{0};
  auto a = clk::now();
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(1)) < files.size();) {
        ofio::Image8 img, out;
        std::string err;
        ofio::read_gray8(files[i], img, err);
        if (scale != 1.0) ofio::resize_u8(img, scale, scale, out);
      }
    });
  for (auto &t : th) t.join();
  const double s = std::chrono::duration<double>(clk::now() - a).count();
  printf("%d threads: %zu slices in %.2f s = %.1f slices/s\n", T, files.size(), s, files.size() / s);
  return 0;
}
