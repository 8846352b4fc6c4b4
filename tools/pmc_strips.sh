#!/bin/bash
# The production-strip workload one batch at a time (--inflight 1: 256 strip pairs of
# 3072x100 per tvl1_calc_batch call, nothing else on the GPU): kernel trace + stats, the
# FETCH_SIZE and WRITE_SIZE passes (HBM bytes per dispatch) and the VALU issue pass, for the
# batched iteration class's roofline (bench.py production_strips.roofline).
# Usage (GPU box, repo root): bash tools/pmc_strips.sh <tag> [bench args]
set -o pipefail
tag=${1:-strips}; shift
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="bench.py --workload strips --width 3072 --height 100 --nscales 10 --warps 5 --batch 256 --steps 1 --warmup 1 --inflight 1 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 $B > $out/bench_trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $out/bench_trace.log; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $out/pmc_$ctr -o run -- python3 $B --no-kernel-timing > $out/bench_$ctr.log 2>&1 || { echo PMC_FAIL $ctr; tail -5 $out/bench_$ctr.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_valu -o run -- python3 $B --no-kernel-timing > $out/bench_valu.log 2>&1 || { echo PMC_FAIL; tail -5 $out/bench_valu.log; exit 1; }
python3 tools/pmc_summary.py $out --batch --emit-traffic $out/traffic_strips.json > $out/pmc_summary.txt
echo done
