# One pair alone on the GPU (--inflight 1): kernel trace + stats, FETCH_SIZE and WRITE_SIZE
# passes (HBM bytes per dispatch), and one PMC pass of VALU
# issue counters, so per-kernel VALU utilisation = SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x
# GRBM_GUI_ACTIVE / 8 XCDs) is not diluted by a second stream's kernels.
# Usage (GPU box, repo root): bash tools/pmc_single.sh <tag> [bench args]
set -o pipefail
tag=${1:-single}; shift
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-fast-math-line --no-strips-line $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 $B > $out/bench_trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $out/bench_trace.log; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $out/pmc_$ctr -o run -- python3 $B --no-kernel-timing > $out/bench_$ctr.log 2>&1 || { echo PMC_FAIL $ctr; tail -5 $out/bench_$ctr.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_valu -o run -- python3 $B --no-kernel-timing > $out/bench_valu.log 2>&1 || { echo PMC_FAIL; tail -5 $out/bench_valu.log; exit 1; }
echo done
