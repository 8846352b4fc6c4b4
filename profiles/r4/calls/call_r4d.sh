#!/bin/bash
# r4 GPU call: the batched strip path of the CLI and kb_warp_iter's constants on demand.
set -o pipefail
out=gpurun_out/r4d
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cli_batch_gpu.py tests/test_gpu_batch.py > $out/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for i in 1 2; do
  for e in 0 1; do
    TVL1_BATCH_STORE=$e timeout -k 10 200 python bench.py --workload strips --steps 3 --warmup 1 --no-cpu-baseline > $out/strips_store$e_$i.json 2>&1 || { echo STRIPS_FAIL; exit 1; }
    echo "strips TVL1_BATCH_STORE=$e round $i $(tail -1 $out/strips_store$e_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"] if d["roofline"] else None)')"
  done
done | tee $out/ab_strips_store.txt
bash tools/pmc_strips.sh r4_ondemand > $out/pmc_strips.log 2>&1 || { echo PMC_FAIL; tail -5 $out/pmc_strips.log; exit 1; }
echo ALL_DONE
