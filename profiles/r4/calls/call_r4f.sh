#!/bin/bash
# r4 GPU call: CLI end to end on an uncompressed-TIFF 6144x4096 stack, production strip jobs
# batched (strip_batch 256) against the per-pair path (0), then the C2 full-frame job.
set -o pipefail
out=gpurun_out/r4f
mkdir -p $out
timeout -k 10 900 python -u tools/cli_e2e.py --slices 201 --format tiff --jobs strips --strip-batch 256,0 --no-single-thread --out /tmp/e2e_tiff > $out/cli_e2e_tiff.txt 2>&1 || { echo E2E_FAIL; tail -20 $out/cli_e2e_tiff.txt; exit 1; }
cat $out/cli_e2e_tiff.txt
rm -rf /tmp/e2e_tiff
echo ALL_DONE
