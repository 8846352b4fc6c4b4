#!/bin/bash
# r4 GPU call: batched passes with 64-px bands (kb_iterate_roll<K, 1>) on narrow levels.
# Parity of the new instantiations first, then the strip workload at several width cut-offs
# (two alternations).
set -o pipefail
out=gpurun_out/r4j
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_batch.py > $out/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for i in 1 2; do
  for w in -1 1100 1700 2500 4000; do
    TVL1_BATCH_PX1_W=$w timeout -k 10 200 python bench.py --workload strips --steps 3 --warmup 1 --no-cpu-baseline > $out/s_${w}_$i.json 2>&1 || { echo STRIPS_FAIL; tail -5 $out/s_${w}_$i.json; exit 1; }
    echo "strips px1_w $w round $i $(tail -1 $out/s_${w}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done | tee $out/strips_px1.txt
echo ALL_DONE
