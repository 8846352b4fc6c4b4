# A/B of kernel variants on the GPU box: parity first, then one bench per variant.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/t2.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/t2.log; exit 1; }
tail -3 gpurun_out/t2.log
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line $BENCH_ARGS > "gpurun_out/ab_$(echo $cfg | tr " " "_").log" 2>&1 || { echo BENCH_FAIL $cfg; tail -5 "gpurun_out/ab_$(echo $cfg | tr " " "_").log"; exit 1; }
  echo "$cfg $(tail -1 "gpurun_out/ab_$(echo $cfg | tr " " "_").log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("pairs/s", d["value"], "ms", d["ms_per_step"], "spec_miss", d["config"].get("speculation_misses"), "alg", r["achieved"], "compulsory", r["compulsory_GBs"], "us", r["avg_launch_us"], d["pair_breakdown_ms"], "inflight", d["config"]["pairs_in_flight_per_gpu"])')"
done
