#!/bin/bash
# r5 A/B (strips): the fused warp + first pass (kb_warp_iter) only on levels of at least N px
# per pair (TVL1_BATCH_FUSE_MIN), below it kb_warp_ring + the 2-iteration pass.  On the tiny
# levels kb_warp_iter's window-ring prologue (2M = 12 rows) and 128-px bands cost 1.2-1.8x
# (41.9 ms per G px at level 8 against 16.7 at level 0, profiles/r5/strips_levels/).
# Expected: kb_warp_iter time of levels 7-8 (1.1 ms per batch) partly saved, strips +0-1 %.
# 0 (default) / 20000 (levels 7-8 unfused) / 60000 (4-8) / 100000 (3-8); three alternations.
set -o pipefail
export BENCH_FLAGS="--workload strips --steps 3"
bash tools/ab_env.sh 3 "TVL1_BATCH_FUSE_MIN=0" "TVL1_BATCH_FUSE_MIN=20000" "TVL1_BATCH_FUSE_MIN=60000" "TVL1_BATCH_FUSE_MIN=100000" > gpurun_out/r5_fuse_min.txt 2>&1
