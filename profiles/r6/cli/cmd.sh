#!/bin/bash
# r6: the 40,860-pair gen_cross-style strip job (401-slice uncompressed
# TIFF stack, strides 1-120, scale 0.5, top / bottom 100 rows, random_points) through the
# CLI with per-stage timing (timing_json), then the GPU-only rates on the same box.
#   cli_e2e_tiff_40860pairs_stages.txt   engine + CLI of commit d4007b3 (stages measured)
#   cli_e2e_tiff_40860pairs_overlap.txt  + point draws during the solve, parallel record writes
#   bench_strips_same_box.json / bench_c2_same_box.json: bench.py on the box of each run
set -o pipefail
timeout -k 10 300 python -u tools/cli_e2e.py --slices 401 --format tiff --jobs strips \
  --strides 1-120 --no-single-thread --out /tmp/cli_stack > gpurun_out/r6f/cli_e2e.txt 2>&1 &&
timeout -k 10 500 python bench.py > gpurun_out/r6f/bench_c2.json 2> gpurun_out/r6f/bench_c2.err
