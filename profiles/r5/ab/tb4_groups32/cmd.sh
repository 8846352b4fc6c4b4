#!/bin/bash
# r5 A/B (C2): k_iterate_tb4 with 1024-thread regions of 64 x 96 rows (32 row groups of 3
# rows; ab_tb4g32/, built by tools/build_variant.sh with -DTVL1_TB4_GROUPS=32) against the
# in-tree 512-thread 64 x 48 regions.  Level 4's 4-iteration passes recompute 1.25x instead
# of 1.37x of their output (-9 % work), at 16 waves per barrier instead of 8 and one block
# per CU.  Expected: k_iterate_tb4 -0..-8 % per pass; C2 within +-1 %.  Parity subset first.
set -o pipefail
bash tools/ab_libs.sh 3 . ab_tb4g32 > gpurun_out/r5_tb4g32.txt 2>&1
# (the knob this A/B used was removed after it; see result.txt and DESIGN 9)
