#!/bin/bash
# r4: strip batch size / batches in flight on the final engine (LDS-staged passes, 64-px bands
# on narrow levels): 256 x 2 (default), 256 x 3, 128 x 4, two alternations.
set -o pipefail
out=gpurun_out/r4aa
mkdir -p $out
for i in 1 2; do
  for cfg in "256 2" "256 3" "128 4"; do
    set -- $cfg
    timeout -k 10 200 python bench.py --workload strips --batch $1 --inflight $2 --steps 3 --warmup 1 --no-cpu-baseline > $out/s_$1_$2_$i.json 2>&1 || { echo STRIPS_FAIL; exit 1; }
    echo "strips batch $1 inflight $2 round $i $(tail -1 $out/s_$1_$2_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done | tee $out/sweep.txt
echo ALL_DONE
