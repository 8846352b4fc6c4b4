#!/bin/bash
# r4: the 64-px band cut-off of the batched passes re-checked with the LDS-staged 128-px
# passes (3 wavefronts per SIMD now): TVL1_BATCH_PX1_W 1700 (default) / 1100 / 2500 / 0,
# strips bench, three alternations.
set -o pipefail
out=gpurun_out/r4u
mkdir -p $out
for i in 1 2 3; do
  for w in 1700 1100 2500 0; do
    TVL1_BATCH_PX1_W=$w timeout -k 10 200 python bench.py --workload strips --steps 3 --warmup 1 --no-cpu-baseline > $out/s_${w}_$i.json 2>&1 || { echo STRIPS_FAIL; tail -5 $out/s_${w}_$i.json; exit 1; }
    echo "px1_w $w round $i $(tail -1 $out/s_${w}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done | tee $out/ab.txt
echo ALL_DONE
