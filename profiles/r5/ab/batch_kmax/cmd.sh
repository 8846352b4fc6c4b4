#!/bin/bash
# r5: batched passes longer than 4 iterations (TVL1_BATCH_KMAX; kb_iterate_roll<5..8, 1> on
# 64-px bands, <5..6, 2> on 128-px bands: <7, 2> and <8, 2> need > 256 VGPRs and gave wrong
# residuals, so 128-px bands cap at 6).  The kmax3 A/B showed the strips lose 19 % when passes
# are capped at 3: the pass count dominates.  The oracle's check schedules of the strips allow
# 10 rounds instead of 18 at level 0 with passes up to 8 (profiles/r5/strips_levels/
# schedule_model.txt).  Costs: <6,2> 240 VGPRs (2 waves/SIMD); <6,1> 123 (4), <8,1> 159 (3).
# Expected: strips -5 ... +10 % by cap.  Parity first (pass length never changes a result).
set -o pipefail
O=gpurun_out/r5_bkmax; mkdir -p $O
for k in 6 8; do
  TVL1_BATCH_KMAX=$k timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 250 --timeout-method thread > $O/parity_$k.log 2>&1 || { tail -30 $O/parity_$k.log; exit 1; }
  echo "kmax $k: $(tail -1 $O/parity_$k.log)"
done
export BENCH_FLAGS="--workload strips --steps 3"
bash tools/ab_env.sh 2 "TVL1_BATCH_KMAX=4" "TVL1_BATCH_KMAX=6" "TVL1_BATCH_KMAX=8" \
  "TVL1_BATCH_KMAX=8 TVL1_BATCH_PX1_W=4000" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
# (the knob this A/B used was removed after it; see the results beside this file and DESIGN 9)
