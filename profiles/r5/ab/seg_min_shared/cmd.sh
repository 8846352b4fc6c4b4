#!/bin/bash
# r5 A/B (C2, 3 pairs in flight): level 3-4 long passes streamed with long segments while the
# other pairs fill the device (TVL1_ROLL_LONG_MIN=2000 streams levels 3 and 4;
# TVL1_SEG_MIN_SHARED=R keeps their segments >= R rows while other solves share the GPU)
# against the default (k_iterate_tb4 on levels 3-4).  Expected: level 4's long passes
# recompute 1.2x (64-row segments) or 1.1x (128) instead of tb4's 1.37x; if the other
# streams fill the slots those launches leave idle, C2 +1-2 %.  Two alternations.
set -o pipefail
export BENCH_FLAGS="--steps 6"
bash tools/ab_env.sh 2 "TVL1_SEG_MIN_SHARED=0" "TVL1_ROLL_LONG_MIN=2000 TVL1_SEG_MIN_SHARED=64" "TVL1_ROLL_LONG_MIN=2000 TVL1_SEG_MIN_SHARED=128" > gpurun_out/r5_seg_min_shared.txt 2>&1
