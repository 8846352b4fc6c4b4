#!/bin/bash
# r5: the batched passes' minimum segment (TVL1_BATCH_SEG_MIN, default 128 rows: the strips'
# levels are never split) against roll_segment alone (=0), after the parity matrix of the
# batched kernels.  Expected: the +1.7 % of TVL1_ROLL_SEG=100 (profiles/r5/ab/strips_seg/).
set -o pipefail
mkdir -p gpurun_out/r5_seg
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py > gpurun_out/r5_seg/batch_tests.log 2>&1 || { tail -20 gpurun_out/r5_seg/batch_tests.log; exit 1; }
tail -1 gpurun_out/r5_seg/batch_tests.log
export BENCH_FLAGS="--workload strips --steps 3"
bash tools/ab_env.sh 3 "TVL1_BATCH_SEG_MIN=0" "TVL1_BATCH_SEG_MIN=128" > gpurun_out/r5_seg/ab.txt 2>&1
