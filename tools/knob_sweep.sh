# Knob sweep of the in-tree engine in ONE GPU call, two alternating rounds (box clock drift
# cancels): bash tools/knob_sweep.sh "ENV=V ..." ...   ("" = defaults).  BENCH_ARGS adds
# bench.py arguments (e.g. --inflight 1).
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for cfg in "$@"; do
    tag=$(echo "x$cfg" | tr " =" "__")
    env $cfg timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line $BENCH_ARGS > "gpurun_out/ks_$tag.log" 2>&1 || { echo BENCH_FAIL "$cfg"; tail -5 "gpurun_out/ks_$tag.log"; exit 1; }
    echo "r$round [$cfg] $(tail -1 "gpurun_out/ks_$tag.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("pairs/s", d["value"], "iter_us", d["roofline"]["avg_launch_us"], d["pair_breakdown_ms"])')"
  done
done
