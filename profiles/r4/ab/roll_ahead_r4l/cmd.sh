#!/bin/bash
# r4 A/B: the 3- and 4-iteration rolling passes with one row of loads ahead (174 VGPRs) and
# with launch bounds for 3 wavefronts per SIMD (168 VGPRs, 5 spilled), against the in-tree
# build (2 rows ahead, 189 VGPRs, 2 wavefronts per SIMD).  Parity subset per build, then C2
# (3 alternations) and strips (2 alternations).
set -o pipefail
out=gpurun_out/r4l
mkdir -p $out
dirs=(. ab_r4l/A1W1 ab_r4l/A1W3)
for d in "${dirs[@]}"; do
  if [ "$d" = "." ]; then unset TVL1_ENGINE_SO; else export TVL1_ENGINE_SO=$d/libtvl1_hip.so; fi
  tag=$(echo "$d" | tr '/.' '__')
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 200 \
    --timeout-method thread -k "matches_oracle or benchmark_pair or golden" > $out/t$tag.log 2>&1 \
    || { echo "PARITY_FAIL $d"; tail -20 $out/t$tag.log; exit 1; }
  echo "$d parity: $(tail -1 $out/t$tag.log)"
done
for i in 1 2 3; do
  for d in "${dirs[@]}"; do
    if [ "$d" = "." ]; then unset TVL1_ENGINE_SO; else export TVL1_ENGINE_SO=$d/libtvl1_hip.so; fi
    tag=$(echo "$d" | tr '/.' '__')
    timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > $out/c2$tag$i.log 2>&1 || { echo BENCH_FAIL $d; tail -5 $out/c2$tag$i.log; exit 1; }
    echo "$d c2 round $i $(tail -1 $out/c2$tag$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("pairs/s", d["value"], "single_pair_ms", d.get("single_pair_ms"), d["pair_breakdown_ms"])')"
  done
done | tee $out/c2.txt
for i in 1 2; do
  for d in "${dirs[@]}"; do
    if [ "$d" = "." ]; then unset TVL1_ENGINE_SO; else export TVL1_ENGINE_SO=$d/libtvl1_hip.so; fi
    tag=$(echo "$d" | tr '/.' '__')
    timeout -k 10 200 python bench.py --workload strips --steps 3 --warmup 1 --no-cpu-baseline > $out/s$tag$i.log 2>&1 || { echo STRIPS_FAIL $d; tail -5 $out/s$tag$i.log; exit 1; }
    echo "$d strips round $i $(tail -1 $out/s$tag$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done | tee $out/strips.txt
echo ALL_DONE
