#!/bin/bash
# r4 GPU call: stage-2 ring fill in k_warp_iter (in-tree) vs without (ab_nos2f/), the batched
# strip CLI path, kb_warp_iter constants on demand.
set -o pipefail
out=gpurun_out/r4e
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cli_batch_gpu.py tests/test_gpu_lifecycle.py tests/test_gpu_batch.py -k "not matches_oracle" > $out/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
# the point-to-point k_iterate_tb4 first on its own, short: a small parity subset under 90 s
TVL1_ENGINE_SO=ab_p2p/libtvl1_hip.so timeout -k 10 90 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_gpu_parity.py -k "golden" > $out/p2p_smoke.log 2>&1 || { echo P2P_FAIL; tail -20 $out/p2p_smoke.log; exit 1; }
tail -1 $out/p2p_smoke.log
bash tools/ab_libs.sh 3 . ab_nos2f ab_p2p > $out/ab_c2_s2f.txt 2>&1 || { echo AB_FAIL; tail -20 $out/ab_c2_s2f.txt; exit 1; }
cat $out/ab_c2_s2f.txt
for i in 1 2; do
  for arm in new nos2f store1 group0 segs0; do
    unset TVL1_ENGINE_SO TVL1_BATCH_STORE TVL1_BATCH_GROUP TVL1_BATCH_SEGS
    [ $arm = nos2f ] && export TVL1_ENGINE_SO=ab_nos2f/libtvl1_hip.so
    [ $arm = store1 ] && export TVL1_BATCH_STORE=1
    [ $arm = group0 ] && export TVL1_BATCH_GROUP=0
    [ $arm = segs0 ] && export TVL1_BATCH_SEGS=0
    timeout -k 10 200 python bench.py --workload strips --steps 3 --warmup 1 --no-cpu-baseline > $out/strips_${arm}_$i.json 2>&1 || { echo STRIPS_FAIL; tail -5 $out/strips_${arm}_$i.json; exit 1; }
    echo "strips $arm round $i $(tail -1 $out/strips_${arm}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_us"] if d["roofline"] else None)')"
  done
done | tee $out/ab_strips.txt
unset TVL1_ENGINE_SO TVL1_BATCH_STORE
bash tools/pmc_stall.sh r4e_s2f > $out/stall.log 2>&1 || { echo STALL_FAIL; exit 1; }
echo ALL_DONE
