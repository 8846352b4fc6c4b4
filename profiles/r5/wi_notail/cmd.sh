#!/bin/bash
# r5: timing bound for moving the gather's tail (1/wsum, the three products, rho_c: ~13 VALU
# + a reciprocal of the producers' ~250 per step) off k_warp_iter's producers, which set the
# pace (profiles/r5/wi_roles/).  wi_probe built with -DTVL1_PROBE_NO_TAIL skips the tail
# (results wrong, timing only) against the shipped body, alternating, C2 levels 0 / 2 / 4.
# Expected: if the producers alone set the pace, -4..-6 % per launch; integrate only if the
# bound is >= 4 %.
set -o pipefail
O=gpurun_out/r5_wi_notail; mkdir -p $O
for rep in 1 2; do
for g in "6144 4096" "3932 2621" "2516 1678"; do
  echo "== base $g" >> $O/notail.txt
  timeout -k 10 60 tools/_bin/wi_probe $g 10 2>&1 | grep -E "engine|^probe:" >> $O/notail.txt || exit 1
  echo "== notail $g" >> $O/notail.txt
  timeout -k 10 60 tools/_bin/wi_probe_notail $g 10 2>&1 | grep -E "engine|^probe:" >> $O/notail.txt || exit 1
done
done
