# Per-kernel average durations of several engine builds, one rocprofv3 kernel-trace run of
# one C2 pair in flight each (A = the in-tree build first and last).
# Usage (GPU box, repo root): bash tools/ab_kernels_multi.sh DIR1 DIR2 ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for d in . "$@" .; do
  if [ "$d" = "." ]; then unset TVL1_ENGINE_SO; else export TVL1_ENGINE_SO=$d/libtvl1_hip.so; fi
  tag=$(echo "$d" | tr '/.' '__')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abm_$tag -o run -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > gpurun_out/abm_$tag.log 2>&1 || { echo TRACE_FAIL $d; tail -5 gpurun_out/abm_$tag.log; exit 1; }
  echo "== $d  $(grep '^{' gpurun_out/abm_$tag.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("single_pair_ms", d.get("single_pair_ms"))')"
  python3 - gpurun_out/abm_$tag/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0].replace("void ", "").replace("tvl1k::", "")
    if float(r["Percentage"]) > 1.0:
        print(f"  {n:45s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us  {float(r['Percentage']):5.1f} %")
PY
  rm -f gpurun_out/abm_$tag/run_kernel_trace.csv
done
unset TVL1_ENGINE_SO
