#!/bin/bash
# r5: passes of at most 3 iterations (TVL1_KMAX=3) against 4.  The roll_edge A/B showed the
# rolling passes lose ~10 % per wavefront per SIMD they give up; <3,2> runs at 127 VGPRs
# (4 wavefronts per SIMD) where <4,2> needs 164 (3).  Expected: strips and C2 within -5 ... +5 %
# (a third more HBM passes per iteration and more launches, against the occupancy).  The
# pass length never changes a result: the parity subset runs with the cap first.
set -o pipefail
O=gpurun_out/r5_kmax; mkdir -p $O
TVL1_KMAX=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -k "matches_oracle or benchmark_pair or batch or configs or fma or speculation" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
export BENCH_FLAGS="--workload strips --steps 3"
bash tools/ab_env.sh 3 "TVL1_KMAX=4" "TVL1_KMAX=3" > $O/ab_strips.txt 2>&1 || { cat $O/ab_strips.txt; exit 1; }
cat $O/ab_strips.txt
export BENCH_FLAGS="--steps 4 --warmup 1"
bash tools/ab_env.sh 2 "TVL1_KMAX=4" "TVL1_KMAX=3" > $O/ab_c2.txt 2>&1 || { cat $O/ab_c2.txt; exit 1; }
cat $O/ab_c2.txt
# (the knob this A/B used was removed after it; see the results beside this file and DESIGN 9)
