#!/bin/bash
# r4 A/B in one call: strips on the r4-final engine (ab_old, commit 0dccc78) against the
# current tree (64-px bands on narrow levels + one-row lookahead in kb_iterate_roll), and the
# current tree with the 64-px bands off (TVL1_BATCH_PX1_W=0).  Three alternations.
set -o pipefail
out=gpurun_out/r4n
mkdir -p $out
for i in 1 2 3; do
  for v in old cur cur_px1off; do
    unset TVL1_ENGINE_SO TVL1_BATCH_PX1_W
    [ $v = old ] && export TVL1_ENGINE_SO=ab_old/libtvl1_hip.so
    [ $v = cur_px1off ] && export TVL1_BATCH_PX1_W=0
    timeout -k 10 200 python bench.py --workload strips --steps 3 --warmup 1 --no-cpu-baseline > $out/s_${v}_$i.json 2>&1 || { echo STRIPS_FAIL $v; tail -5 $out/s_${v}_$i.json; exit 1; }
    echo "$v round $i $(tail -1 $out/s_${v}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done | tee $out/strips_ab.txt
echo ALL_DONE
