#!/bin/bash
# r5: which k_warp_iter role sets the pace on the final r4 engine?  Per-wave barrier-wait
# share by role (tools/wi_probe.hip built with -DWI_BARRIER: waves 0 / 1 = stage 1 / 2,
# 2-3 = producers), C2 levels 0, 2 and 4.  A role that waits least is the pace setter; work
# moves toward roles that wait most.
set -o pipefail
O=gpurun_out/r5_wi_roles; mkdir -p $O
for g in "6144 4096" "3932 2621" "2516 1678"; do
  echo "== $g" >> $O/roles.txt
  timeout -k 10 60 tools/_bin/wi_probe_bar $g 5 >> $O/roles.txt 2>&1 || exit 1
done
