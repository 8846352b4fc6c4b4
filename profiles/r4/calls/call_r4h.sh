#!/bin/bash
# r4 GPU call: the CLI end to end on an uncompressed-TIFF 6144x4096 stack for >= 30 s --
# 40,860 gen_cross-style pairs (strides 1-120 over 401 slices), production strip jobs batched;
# then the same job on the per-pair path (strip_batch 0), and the PNG stack for comparison.
set -o pipefail
out=gpurun_out/r4h
mkdir -p $out
timeout -k 10 1000 python -u tools/cli_e2e.py --slices 401 --format tiff --jobs strips --strides 1-120 --strip-batch 256 --no-single-thread --out /tmp/e2e_tiff > $out/cli_e2e_tiff_long.txt 2>&1 || { echo E2E_FAIL; tail -20 $out/cli_e2e_tiff_long.txt; exit 1; }
cat $out/cli_e2e_tiff_long.txt
timeout -k 10 600 python -u tools/cli_e2e.py --slices 401 --format tiff --jobs strips --strides 1-20 --strip-batch 0 --no-single-thread --out /tmp/e2e_tiff > $out/cli_e2e_tiff_perpair.txt 2>&1 || { echo E2E_FAIL; tail -20 $out/cli_e2e_tiff_perpair.txt; exit 1; }
cat $out/cli_e2e_tiff_perpair.txt
rm -rf /tmp/e2e_tiff
echo ALL_DONE
