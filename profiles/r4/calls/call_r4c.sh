#!/bin/bash
# r4 GPU call: bank-conflict-free window rings (in-tree) against the same tree without them
# (ab_head/): parity, C2 A/B, strips A/B, PMC stall/LDS counters, then the residual-margin report.
set -o pipefail
out=gpurun_out/r4c
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_lifecycle.py tests/test_c1_cli_gpu.py > $out/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
bash tools/ab_libs.sh 3 . ab_head > $out/ab_c2.txt 2>&1 || { echo AB_FAIL; tail -20 $out/ab_c2.txt; exit 1; }
cat $out/ab_c2.txt
for i in 1 2; do
  for d in . ab_head; do
    if [ "$d" = "." ]; then unset TVL1_ENGINE_SO; else export TVL1_ENGINE_SO=$d/libtvl1_hip.so; fi
    timeout -k 10 200 python bench.py --workload strips --steps 3 --warmup 1 --no-cpu-baseline > $out/strips_$i$(echo $d | tr './' '__').json 2>&1 || { echo STRIPS_FAIL; exit 1; }
    echo "strips $d $i $(tail -1 $out/strips_$i$(echo $d | tr './' '__').json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"] if d["roofline"] else None)')"
  done
done | tee $out/ab_strips.txt
unset TVL1_ENGINE_SO
bash tools/pmc_stall.sh r4_new > $out/stall_new.log 2>&1 || { echo STALL_FAIL; exit 1; }
TVL1_ENGINE_SO=ab_head/libtvl1_hip.so bash tools/pmc_stall.sh r4_head > $out/stall_head.log 2>&1 || { echo STALL_FAIL; exit 1; }
OMP_NUM_THREADS=16 timeout -k 10 500 python -u tests/analysis/residual_margins.py --device --out $out/residual_margins > $out/margins.log 2>&1 || { echo MARGINS_FAIL; tail -5 $out/margins.log; exit 1; }
echo ALL_DONE
