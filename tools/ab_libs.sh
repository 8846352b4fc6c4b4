# A/B/C... of engine builds in ONE GPU call (box-to-box clock differences cancel).
# Usage (on the GPU box, repo root): bash tools/ab_libs.sh ROUNDS DIR1 DIR2 ... [-- bench args]
# "." = the in-tree build; any other DIR holds a libtvl1_hip.so.  Each build first runs the
# parity subset (bitwise vs the oracle), then the builds alternate one C2 bench each.
set -o pipefail
rounds=$1; shift
dirs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do dirs+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p gpurun_out
for d in "${dirs[@]}"; do
  if [ "$d" = "." ]; then unset TVL1_ENGINE_SO; else export TVL1_ENGINE_SO=$d/libtvl1_hip.so; fi
  tag=$(echo "$d" | tr '/.' '__')
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 200 \
    --timeout-method thread -k "matches_oracle or benchmark_pair or golden or batch" > gpurun_out/abl_t$tag.log 2>&1 \
    || { echo "PARITY_FAIL $d"; tail -20 gpurun_out/abl_t$tag.log; exit 1; }
  echo "$d parity: $(tail -1 gpurun_out/abl_t$tag.log)"
done
for i in $(seq 1 "$rounds"); do
  for d in "${dirs[@]}"; do
    if [ "$d" = "." ]; then unset TVL1_ENGINE_SO; else export TVL1_ENGINE_SO=$d/libtvl1_hip.so; fi
    tag=$(echo "$d" | tr '/.' '__')
    timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line "$@" > gpurun_out/abl_$tag$i.log 2>&1 || { echo BENCH_FAIL $d; tail -5 gpurun_out/abl_$tag$i.log; exit 1; }
    echo "$d round $i $(tail -1 gpurun_out/abl_$tag$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("pairs/s", d["value"], "single_pair_ms", d.get("single_pair_ms"), d["pair_breakdown_ms"])')"
  done
done
unset TVL1_ENGINE_SO
