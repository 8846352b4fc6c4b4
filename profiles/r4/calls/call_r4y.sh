#!/bin/bash
# r4: C5 at full size on one GPU with the r4 engine: strides 1/4/16 over a 4096-slice
# 6144x4096 stack (12,267 pairs), slices made on the device, progress every 30 s.
set -o pipefail
out=gpurun_out/r4y
mkdir -p $out
timeout -k 10 1100 python bench.py --workload stack --slices 4096 --strides 1,4,16 > $out/c5_full_1gpu.json 2> $out/c5_full_1gpu_progress.txt || { echo C5_FAIL; tail -5 $out/c5_full_1gpu_progress.txt; exit 1; }
tail -1 $out/c5_full_1gpu.json | cut -c1-200
echo ALL_DONE
