#!/bin/bash
# r4: C2 pairs in flight re-checked on the final engine (2 / 3 / 4, three alternations).
set -o pipefail
out=gpurun_out/r4x
mkdir -p $out
for i in 1 2 3; do
  for f in 3 2 4; do
    timeout -k 10 200 python bench.py --steps 4 --warmup 1 --inflight $f --no-cpu-baseline --no-fast-math-line --no-strips-line > $out/c2_f${f}_$i.log 2>&1 || { echo BENCH_FAIL; exit 1; }
    echo "inflight $f round $i $(tail -1 $out/c2_f${f}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("pairs/s", d["value"])')"
  done
done | tee $out/ab.txt
echo ALL_DONE
