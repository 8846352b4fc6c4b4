#!/bin/bash
# r5: the 40,860-pair production strip job (gen_cross shape: strides 1-120 over a 401-slice
# uncompressed-TIFF 6144x4096 stack, scale 0.5, top / bottom 100, random_points) through the
# CLI on the final r5 engine.  Expected: within a few % of r4's 1,544 pairs/s; the GPU side
# gained ~+3 % (strips 3,303 -> 3,387 in the evidence sets) and the CLI ran at ~94 % of it.
set -o pipefail
out=gpurun_out/r5cli
mkdir -p $out
timeout -k 10 1000 python -u tools/cli_e2e.py --slices 401 --format tiff --jobs strips --strides 1-120 --strip-batch 256 --no-single-thread --out /tmp/e2e_tiff > $out/cli_e2e_tiff_40860pairs.txt 2>&1 || { echo E2E_FAIL; tail -20 $out/cli_e2e_tiff_40860pairs.txt; exit 1; }
cat $out/cli_e2e_tiff_40860pairs.txt
