# rocprofv3 evidence for the bench workload (run on the GPU box from the repo root):
#   1. kernel trace + stats (per-kernel average durations)
#   2. separate PMC passes: FETCH_SIZE, WRITE_SIZE, SQ wave/VALU counters
# Usage: bash tools/profile.sh <tag> [extra bench args]
set -o pipefail
tag=${1:-r1}; shift
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 $B > $out/bench_trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $out/bench_trace.log; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  name=$(echo $ctr | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $out/pmc_$name -o run -- python3 $B --no-kernel-timing > $out/bench_$name.log 2>&1 || { echo PMC_FAIL $ctr; tail -5 $out/bench_$name.log; exit 1; }
done
tail -1 $out/bench_trace.log | cut -c1-300
echo done
