#!/bin/bash
# r4 A/B: the 1- and 2-iteration rolling passes on 128-px bands at more wavefronts per SIMD:
# W4 = launch bounds for 4 (128 VGPRs, 1 spilled), A1 = one row of loads ahead (99 VGPRs, 5
# per SIMD), against the in-tree build (129 VGPRs, 3 per SIMD).  Parity subset per build, a
# kernel trace of one C2 pair per build, then C2 and strips alternations.
set -o pipefail
out=gpurun_out/r4o
mkdir -p $out
dirs=(. ab_r4o/W4 ab_r4o/A1)
for d in "${dirs[@]}"; do
  if [ "$d" = "." ]; then unset TVL1_ENGINE_SO; else export TVL1_ENGINE_SO=$d/libtvl1_hip.so; fi
  tag=$(echo "$d" | tr '/.' '__')
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 200 \
    --timeout-method thread -k "matches_oracle or benchmark_pair or golden" > $out/t$tag.log 2>&1 \
    || { echo "PARITY_FAIL $d"; tail -20 $out/t$tag.log; exit 1; }
  echo "$d parity: $(tail -1 $out/t$tag.log)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for d in "${dirs[@]}"; do
  if [ "$d" = "." ]; then unset TVL1_ENGINE_SO; else export TVL1_ENGINE_SO=$d/libtvl1_hip.so; fi
  tag=$(echo "$d" | tr '/.' '__')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/k$tag -o run -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > $out/k$tag.log 2>&1 || { echo TRACE_FAIL; tail -5 $out/k$tag.log; exit 1; }
  echo "$d kernels:"; find $out/k$tag -name "*kernel_stats.csv" -exec grep -h "k_iterate_roll<false, [12], 2" {} \; | cut -d, -f1-4
done
for i in 1 2; do
  for d in "${dirs[@]}"; do
    if [ "$d" = "." ]; then unset TVL1_ENGINE_SO; else export TVL1_ENGINE_SO=$d/libtvl1_hip.so; fi
    tag=$(echo "$d" | tr '/.' '__')
    timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > $out/c2$tag$i.log 2>&1 || { echo BENCH_FAIL $d; exit 1; }
    echo "$d c2 round $i $(tail -1 $out/c2$tag$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("pairs/s", d["value"], "single_pair_ms", d.get("single_pair_ms"))')"
    timeout -k 10 200 python bench.py --workload strips --steps 3 --warmup 1 --no-cpu-baseline > $out/s$tag$i.log 2>&1 || { echo STRIPS_FAIL $d; exit 1; }
    echo "$d strips round $i $(tail -1 $out/s$tag$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done | tee $out/ab.txt
echo ALL_DONE
