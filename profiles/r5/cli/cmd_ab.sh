#!/bin/bash
# r5: the same 40,860-pair CLI strip job, alternating the default engine with
# TVL1_BATCH_SMALL=0 (the r4 coarsest-level path) on one stack, to tell the engine's share of
# cmd.sh's 1,414 pairs/s (r4: 1,544) from the box's.  Expected: the two within +-1 %.
set -o pipefail
out=gpurun_out/r5cli
mkdir -p $out
timeout -k 10 1000 python -u tools/cli_e2e.py --slices 401 --format tiff --jobs strips --strides 1-120 --strip-batch 256 --ab-env TVL1_BATCH_SMALL=0 --out /tmp/e2e_tiff > $out/cli_e2e_ab_small.txt 2>&1 || { echo E2E_FAIL; tail -20 $out/cli_e2e_ab_small.txt; exit 1; }
cat $out/cli_e2e_ab_small.txt
