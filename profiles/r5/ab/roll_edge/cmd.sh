#!/bin/bash
# r5: the rolling passes skip the stage rows outside the image in the steps near its top and
# bottom (ab_edge: -DTVL1_ROLL_EDGE=1; wave-uniform branches per stage in those steps only)
# against HEAD.  Compile-time cost: <4,2> 164 -> 183 VGPRs (3 -> 2 waves/SIMD), kb <4,1> 95 ->
# 139 (5 -> 3).  Expected: strips -3 ... +3 % (VALU -4 % of a batch against the occupancy
# loss); C2 +-1 % (its segments rarely touch the border).  Parity subset on the variant first.
set -o pipefail
O=gpurun_out/r5_edge; mkdir -p $O
TVL1_ENGINE_SO=ab_edge/libtvl1_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -k "matches_oracle or benchmark_pair or batch or configs or fma or speculation" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
export BENCH_FLAGS="--workload strips --steps 3"
bash tools/ab_env.sh 3 "TVL1_AB_BASE=1" "TVL1_ENGINE_SO=ab_edge/libtvl1_hip.so" > $O/ab_strips.txt 2>&1 || { cat $O/ab_strips.txt; exit 1; }
cat $O/ab_strips.txt
export BENCH_FLAGS="--steps 4 --warmup 1"
bash tools/ab_env.sh 2 "TVL1_AB_BASE=1" "TVL1_ENGINE_SO=ab_edge/libtvl1_hip.so" > $O/ab_c2.txt 2>&1 || { cat $O/ab_c2.txt; exit 1; }
cat $O/ab_c2.txt
# (TVL1_ROLL_EDGE was removed after this A/B; see the results beside this file and DESIGN 9)
