#!/bin/bash
# r5 A/B (strips, with the r5 segment minimum): batch sizes that quantise the big levels'
# launches better.  Level 0's K = 4 pass is 26 bands x B wavefronts on 3072 resident slots
# (B = 256: 2.17 rounds; 236: 2.00) and its kb_warp_iter 25 x B blocks on 1024 slots (256:
# 6.25 rounds; 236: 5.76).  Expected: 236 within +-1 % of 256 (the second batch in flight
# fills the partial rounds); 2 alternations of 224 / 236 / 248 / 256.
set -o pipefail
export BENCH_FLAGS="--workload strips --steps 3"
bash tools/ab_flags.sh 2 r5bs "--batch 224" "--batch 236" "--batch 248" "--batch 256" > gpurun_out/r5_strips_batch_size.txt 2>&1
