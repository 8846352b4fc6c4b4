#!/bin/bash
# r4 A/B: k_warp_iter with a 4-px window margin (ab_wi4: 29,952 B of LDS, 5 blocks per CU)
# against the in-tree 6-px margin (39,936 B, 4 blocks per CU, LDS-limited).  Parity subset on
# the variant, kernel trace of one C2 pair each, C2 alternations.
set -o pipefail
out=gpurun_out/r4w
mkdir -p $out
export TVL1_ENGINE_SO=ab_wi4/libtvl1_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > $out/t_wi4.log 2>&1 || { echo "PARITY_FAIL"; tail -30 $out/t_wi4.log; exit 1; }
echo "wi4 parity: $(tail -1 $out/t_wi4.log)"
unset TVL1_ENGINE_SO
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for d in . ab_wi4; do
  if [ "$d" = "." ]; then unset TVL1_ENGINE_SO; else export TVL1_ENGINE_SO=$d/libtvl1_hip.so; fi
  tag=$(echo "$d" | tr '/.' '__')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/k$tag -o run -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > $out/k$tag.log 2>&1 || { echo TRACE_FAIL; tail -5 $out/k$tag.log; exit 1; }
  echo "$d: $(find $out/k$tag -name '*kernel_stats.csv' -exec grep -h 'k_warp_iter' {} \; | awk -F'",' '{print $2}' | cut -d, -f1-3)"
done
for i in 1 2 3; do
  for d in . ab_wi4; do
    if [ "$d" = "." ]; then unset TVL1_ENGINE_SO; else export TVL1_ENGINE_SO=$d/libtvl1_hip.so; fi
    tag=$(echo "$d" | tr '/.' '__')
    timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > $out/c2$tag$i.log 2>&1 || { echo BENCH_FAIL $d; exit 1; }
    echo "$d c2 round $i $(tail -1 $out/c2$tag$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("pairs/s", d["value"], "single_pair_ms", d.get("single_pair_ms"))')"
  done
done | tee $out/ab.txt
echo ALL_DONE
