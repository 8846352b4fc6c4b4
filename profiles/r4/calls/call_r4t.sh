#!/bin/bash
# r4: BASELINE's stack configs on the final r4 engine, one GPU: C3 (255 adjacent pairs of a
# 256-slice 6144x4096 stack) and C4 at full size (4095 pairs of 4096 slices), slices made on
# the device, progress on stderr every 30 s.
set -o pipefail
out=gpurun_out/r4t
mkdir -p $out
timeout -k 10 200 python bench.py --workload stack --slices 256 > $out/c3_stack256.json 2> $out/c3_progress.txt || { echo C3_FAIL; tail -5 $out/c3_progress.txt; exit 1; }
tail -1 $out/c3_stack256.json | cut -c1-200
timeout -k 10 600 python bench.py --workload stack --slices 4096 > $out/c4_full_1gpu.json 2> $out/c4_full_1gpu_progress.txt || { echo C4_FAIL; tail -5 $out/c4_full_1gpu_progress.txt; exit 1; }
tail -1 $out/c4_full_1gpu.json | cut -c1-200
echo ALL_DONE
