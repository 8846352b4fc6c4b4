#!/bin/bash
# r5 A/B (strips): the batched rolling passes in one segment per column band (TVL1_ROLL_SEG=100:
# a 100-row strip level is never split) against roll_segment's automatic split (level 0 of a
# 256-strip batch: 2 segments of 50 rows).  Expected: the long passes recompute 1.15x instead
# of 1.24x of their rows (-7 % of kb_iterate_roll<4,2>'s work, its PMC FETCH_SIZE likewise),
# at the price of a partly filled third round of wavefronts that the second batch in flight
# should cover; strips +2-3 % if so.  Three alternations, then 3 batches in flight with it.
set -o pipefail
export BENCH_FLAGS="--workload strips --steps 3"
bash tools/ab_env.sh 3 "TVL1_ROLL_SEG=0" "TVL1_ROLL_SEG=100" > gpurun_out/r5_strips_seg.txt 2>&1 || exit 1
export BENCH_FLAGS="--workload strips --steps 3 --inflight 3"
bash tools/ab_env.sh 1 "TVL1_ROLL_SEG=0" "TVL1_ROLL_SEG=100" >> gpurun_out/r5_strips_seg.txt 2>&1
