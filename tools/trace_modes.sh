# Kernel traces of one isolated pair per engine configuration, for tools/trace_breakdown.py.
# Usage: bash tools/trace_modes.sh "ENV=V ..." ...   (run on the GPU box from the repo root)
# Per configuration the breakdown lands in gpurun_out/tr_<tag>.txt (the raw trace is
# deleted: gpurun merges at most 64 MiB back).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in "$@"; do
  tag=$(echo "$cfg" | sed "s/[ =\/]/_/g")
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$tag -o run -- python3 bench.py --steps 1 --warmup 1 --inflight 1 --no-cpu-baseline --no-fast-math-line --no-strips-line $BENCH_ARGS > gpurun_out/tr_$tag.log 2>&1 || { echo TRACE_FAIL $cfg; tail -5 gpurun_out/tr_$tag.log; exit 1; }
  python3 tools/trace_breakdown.py gpurun_out/tr_$tag/run_kernel_trace.csv "${TRACE_FILTER:-}" > gpurun_out/tr_$tag.txt
  rm -rf gpurun_out/tr_$tag
  echo "== $cfg"; cat gpurun_out/tr_$tag.txt
done
