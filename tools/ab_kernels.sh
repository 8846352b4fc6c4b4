# Per-kernel average durations of the in-tree engine (A) and another build (B, dir $1) from
# rocprofv3 kernel-trace stats of one bench run each (one pair in flight).
# Usage (GPU box, repo root): bash tools/ab_kernels.sh <dir-with-B/libtvl1_hip.so> [bench args]
set -o pipefail
B=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for arm in A B; do
  if [ $arm = B ]; then export TVL1_ENGINE_SO=$B/libtvl1_hip.so; else unset TVL1_ENGINE_SO; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk_$arm -o run -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-fast-math-line --no-strips-line "$@" > gpurun_out/abk_$arm.log 2>&1 || { echo TRACE_FAIL $arm; tail -5 gpurun_out/abk_$arm.log; exit 1; }
  echo "== $arm"
  python3 - gpurun_out/abk_$arm/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0].replace("void ", "").replace("tvl1k::", "")
    if float(r["Percentage"]) > 0.5:
        print(f"  {n:45s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us  {float(r['Percentage']):5.1f} %")
PY
  rm -f gpurun_out/abk_$arm/run_kernel_trace.csv
done
unset TVL1_ENGINE_SO
