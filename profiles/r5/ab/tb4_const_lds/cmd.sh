#!/bin/bash
# r5: k_iterate_tb4 with the warp constants in LDS (TVL1_TB4_CLDS=1, in-tree) against the
# r5 engine's registers (ab_tb4c0: -DTVL1_TB4_CLDS=0): 102 -> 76 VGPRs, 2 -> 3 blocks per CU.
# Expected: one C2 pair alone -0.8 ... -1.5 ms (tb4 7.7 ms per pair, 0.33 of its wave cycles
# at barriers, 50 % more blocks to cover them); C2 in flight +1-3 % unless tb4's 160 KB of
# LDS per CU keeps the other pairs' kernels off the CUs.  Parity subset per build first.
set -o pipefail
bash tools/ab_libs.sh 3 . ab_tb4c0 > gpurun_out/r5_tb4c.txt 2>&1; rc=$?
cat gpurun_out/r5_tb4c.txt; exit $rc
# (TVL1_TB4_CLDS was removed after this A/B; see result.txt and DESIGN 9)
