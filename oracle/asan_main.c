/* TEST INFRASTRUCTURE: drives the oracle under ASan + UBSan (`make -C oracle asan`,
 * tests/test_host_hardening_cpu.py::test_oracle_under_asan).  Solves small synthetic pairs
 * at odd sizes through every code path of the restatement: both profiles, gamma, median,
 * fixed work, a pyramid that bottoms out, and 1x1 / 16x16 edge sizes. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tvl1_oracle.h"

static void pair(int w, int h, unsigned seed, uint8_t *a, uint8_t *b) {
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      seed = seed * 1103515245u + 12345u;
      const int v = 40 + (int)((seed >> 16) % 160);
      a[y * w + x] = (uint8_t)v;
      b[y * w + (x + 1) % w] = (uint8_t)(v + ((seed >> 8) & 3));
    }
}

int main(void) {
  static const int sizes[][2] = {{1, 1}, {16, 16}, {17, 16}, {33, 19}, {61, 47}, {97, 40}};
  int fails = 0;
  for (size_t si = 0; si < sizeof sizes / sizeof sizes[0]; ++si) {
    const int w = sizes[si][0], h = sizes[si][1];
    uint8_t *a = malloc((size_t)w * h), *b = malloc((size_t)w * h);
    float *u = malloc(sizeof(float) * w * h), *v = malloc(sizeof(float) * w * h);
    pair(w, h, 7u + (unsigned)si, a, b);
    for (int variant = 0; variant < 6; ++variant) {
      tvl1_params p = {0.25, 0.05, 0.3, 10, 3, 0.01, 300, 0.8, 0.0, 0, 1, 0, 0, 30, 10};
      if (variant == 1) p.gamma = 0.2;
      if (variant == 2) p.median_filtering = 5;
      if (variant == 3) p.epsilon = 0.0, p.iterations = 7;
      if (variant == 4) p.profile = 1, p.lambda = 0.15, p.nscales = 3, p.inner_iterations = 5,
                        p.outer_iterations = 2, p.median_filtering = 5;
      if (variant == 5) p.scale_step = 0.5;
      int32_t wi[32 * 3];
      tvl1_stats st;
      memset(&st, 0, sizeof st);
      st.warp_iterations = wi;
      st.warp_iterations_capacity = 32 * 3;
      const int rc = orc_tvl1_calc(&p, a, (size_t)w, b, (size_t)w, w, h, u, v,
                                   sizeof(float) * (size_t)w, &st);
      if (rc != 0) {
        fprintf(stderr, "%dx%d variant %d: status %d\n", w, h, variant, rc);
        ++fails;
      }
      orc_postprocess(u, v, sizeof(float) * (size_t)w, b, (size_t)w, w, h, 1);
    }
    free(a);
    free(b);
    free(u);
    free(v);
  }
  printf("oracle asan driver: %d failures\n", fails);
  return fails != 0;
}
