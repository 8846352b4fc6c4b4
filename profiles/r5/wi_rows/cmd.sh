#!/bin/bash
# r5: how much of a k_warp_iter launch is fixed cost (pipeline run-in / drain, launch, tail)
# rather than per-row work: the C2 level-0 geometry at 4096 rows against 2048 and 8192 rows
# (one round of segments each, so the segment length scales with H), and the level-1..3
# widths.  A two-warps-per-launch kernel can save at most the fixed part.
set -o pipefail
O=gpurun_out/r5_wi; mkdir -p $O
P=tools/_bin/wi_probe
for g in "6144 2048" "6144 4096" "6144 8192" "4915 3277" "3932 2621" "3146 2097" "2516 1678"; do
  echo "== $g" >> $O/wi_rows.txt
  timeout -k 10 60 $P $g 10 >> $O/wi_rows.txt 2>&1 || exit 1
done
echo "== 6144 4096 mode 2 (no HBM)" >> $O/wi_rows.txt
timeout -k 10 60 $P 6144 4096 10 0 2 >> $O/wi_rows.txt 2>&1
