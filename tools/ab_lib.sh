# A/B of two engine builds in ONE GPU call (box-to-box clock differences cancel).
# Usage (on the GPU box, repo root): bash tools/ab_lib.sh <dir-with-B/libtvl1_hip.so> [bench args]
# A = the in-tree build, B = the other; alternates A B A B, one bench each.
set -o pipefail
B=$1; shift
mkdir -p gpurun_out
for i in 1 2; do
  for arm in A B; do
    if [ $arm = B ]; then export TVL1_ENGINE_SO=$B/libtvl1_hip.so; else unset TVL1_ENGINE_SO; fi
    timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line "$@" > gpurun_out/ablib_$arm$i.log 2>&1 || { echo BENCH_FAIL $arm; tail -5 gpurun_out/ablib_$arm$i.log; exit 1; }
    echo "$arm$i $(tail -1 gpurun_out/ablib_$arm$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("pairs/s", d["value"], d.get("pair_breakdown_ms", d.get("ms_per_step")))')"
  done
done
unset TVL1_ENGINE_SO
