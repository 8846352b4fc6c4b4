#!/bin/bash
# r4 GPU call: strip batch size / batches in flight, and C2's shared-slot fill, re-checked on the
# r4 engine (two alternations each); plus the batched CLI test over two device workers.
set -o pipefail
out=gpurun_out/r4i
mkdir -p $out
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_cli_batch_gpu.py -k "two_device" > $out/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for i in 1 2; do
  for cfg in "256 2" "256 3" "128 3" "192 2"; do
    set -- $cfg
    timeout -k 10 200 python bench.py --workload strips --batch $1 --inflight $2 --steps 3 --warmup 1 --no-cpu-baseline > $out/s_$1_$2_$i.json 2>&1 || { echo STRIPS_FAIL; exit 1; }
    echo "strips batch $1 inflight $2 round $i $(tail -1 $out/s_$1_$2_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done | tee $out/strips_sweep.txt
for i in 1 2; do
  for f in 45 60 75; do
    TVL1_FILL_SHARED=$f timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > $out/c2_fill$f_$i.json 2>&1 || { echo C2_FAIL; exit 1; }
    echo "c2 fill_shared $f round $i $(tail -1 $out/c2_fill$f_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done | tee $out/c2_fill_sweep.txt
echo ALL_DONE
