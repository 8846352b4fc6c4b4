# r3 probe (record; the TVL1_SHORT_TB4 knob it sets was removed after this A/B, profiles/r3/ab_short_tb4.txt):
# 2-iteration passes on small levels in k_iterate_tb4 vs k_iterate_roll<2,2>
set -o pipefail
mkdir -p gpurun_out
TVL1_SHORT_TB4=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 200 \
  --timeout-method thread -k "matches_oracle or benchmark_pair or golden or batch" > gpurun_out/short_tb4_parity.log 2>&1 \
  || { echo PARITY_FAIL; tail -20 gpurun_out/short_tb4_parity.log; exit 1; }
echo "parity with TVL1_SHORT_TB4=1: $(tail -1 gpurun_out/short_tb4_parity.log)"
bash tools/ab_env.sh 3 "TVL1_SHORT_TB4=0" "TVL1_SHORT_TB4=1" || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 1; do
  TVL1_SHORT_TB4=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stb4_$v -o run -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > gpurun_out/stb4_$v.log 2>&1 || { echo TRACE_FAIL; exit 1; }
  echo "== TVL1_SHORT_TB4=$v $(grep '^{' gpurun_out/stb4_$v.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("single_pair_ms", d["single_pair_ms"])')"
  python3 - gpurun_out/stb4_$v/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0].replace("void ", "").replace("tvl1k::", "")
    if float(r["Percentage"]) > 1.0:
        print(f"  {n:45s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us  total {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
  rm -f gpurun_out/stb4_$v/run_kernel_trace.csv
done
