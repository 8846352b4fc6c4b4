#!/bin/bash
# r6: k_warp_iter's one-round static launch against persistent blocks
# pulling (band, row range) items from a per-XCD atomic queue, on C2's level 0 and level 3.
# Expected (verdict): mean-life/span 0.889 -> >= 0.95, -5 ... -8 % per launch; integrate only
# at >= 4 %.  Build: see tools/wi_dyn.hip's header.
set -o pipefail
timeout -k 10 300 tools/_bin/wi_dyn 6144 4096 10 > gpurun_out/r6a/wi_dyn_l0.txt 2>&1 &&
timeout -k 10 300 tools/_bin/wi_dyn 3146 2097 10 > gpurun_out/r6a/wi_dyn_l3.txt 2>&1
