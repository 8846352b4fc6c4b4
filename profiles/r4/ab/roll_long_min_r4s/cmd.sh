#!/bin/bash
# r4: with the LDS-staged rolling passes, where should long passes switch from
# k_iterate_tb4 to streaming?  TVL1_ROLL_LONG_MIN (56x32 tiles) default 4096 (levels 3-4 on
# tb4), 3000 (level 3 streams), 2000 (levels 3-4 stream).  Three alternations of the C2
# bench (in flight + one pair alone).
set -o pipefail
out=gpurun_out/r4s
mkdir -p $out
for i in 1 2 3; do
  for m in 4096 3000 2000; do
    TVL1_ROLL_LONG_MIN=$m timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > $out/c2_${m}_$i.log 2>&1 || { echo BENCH_FAIL $m; tail -5 $out/c2_${m}_$i.log; exit 1; }
    echo "long_min $m round $i $(tail -1 $out/c2_${m}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("pairs/s", d["value"], "single_pair_ms", d.get("single_pair_ms"))')"
  done
done | tee $out/ab.txt
echo ALL_DONE
