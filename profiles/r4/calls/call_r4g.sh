#!/bin/bash
# r4 GPU call: batched short passes with 4 px per lane (opt-in) -- parity and strips A/B --
# then the CLI end to end on an uncompressed-TIFF 6144x4096 stack (strip jobs batched vs the
# per-pair path).
set -o pipefail
out=gpurun_out/r4g
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batch.py -k "PX4 or regather or larger_than" > $out/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for i in 1 2; do
  for arm in new px4; do
    unset TVL1_BATCH_PX4
    [ $arm = px4 ] && export TVL1_BATCH_PX4=1
    timeout -k 10 200 python bench.py --workload strips --steps 3 --warmup 1 --no-cpu-baseline > $out/strips_${arm}_$i.json 2>&1 || { echo STRIPS_FAIL; tail -5 $out/strips_${arm}_$i.json; exit 1; }
    echo "strips $arm round $i $(tail -1 $out/strips_${arm}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"] if d["roofline"] else None)')"
  done
done | tee $out/ab_strips_px4.txt
timeout -k 10 900 python -u tools/cli_e2e.py --slices 201 --format tiff --jobs strips --strip-batch 256,0 --no-single-thread --out /tmp/e2e_tiff > $out/cli_e2e_tiff.txt 2>&1 || { echo E2E_FAIL; tail -20 $out/cli_e2e_tiff.txt; exit 1; }
cat $out/cli_e2e_tiff.txt
rm -rf /tmp/e2e_tiff
echo ALL_DONE
