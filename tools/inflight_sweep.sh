set -o pipefail
mkdir -p gpurun_out
for F in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line --inflight $F > gpurun_out/inf_$F.log 2>&1 || { echo FAIL $F; tail -5 gpurun_out/inf_$F.log; exit 1; }
  echo "F=$F $(tail -1 gpurun_out/inf_$F.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("pairs/s", d["value"], "ms/step", d["ms_per_step"], "compulsory", r["compulsory_GBs"], d["pair_breakdown_ms"])')"
done
