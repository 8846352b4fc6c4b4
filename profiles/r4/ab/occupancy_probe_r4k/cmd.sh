#!/bin/bash
# r4 occupancy probe: k_iterate_roll with dynamic LDS padding that caps its residency
# (0: 2 wavefronts per SIMD from its VGPRs; 90000 B: 1 block per CU = 1 wavefront per SIMD),
# one C2 pair at a time, kernel trace.  Says whether the rolling passes are bound per wavefront
# (time doubles at 1 wave/SIMD) or by the SIMD (time barely moves).
set -o pipefail
out=gpurun_out/r4k
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for pad in 0 90000; do
  TVL1_PROBE_ROLL_LDS=$pad timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/pad$pad -o run -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > $out/bench_pad$pad.log 2>&1 || { echo TRACE_FAIL; tail -5 $out/bench_pad$pad.log; exit 1; }
  echo "pad $pad: $(tail -1 $out/bench_pad$pad.log | cut -c1-120)"
  find $out/pad$pad -name "*kernel_stats.csv" -exec grep -h "k_iterate_roll\|k_warp_iter\|k_iterate_tb4" {} \; | cut -c1-160
done
echo ALL_DONE
