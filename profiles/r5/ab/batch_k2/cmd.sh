#!/bin/bash
# r5 A/B (strips): 2-iteration passes on the narrow levels (TVL1_BATCH_K2_W = width cut-off).
# A K-iteration pass on 64-px bands recomputes a K-px halo per side and drains K rows:
# work per useful px-iteration at level 8 (515 x 17) 1.41x for K = 4, 1.19x for K = 2;
# level 5 (1007 x 33) 1.27x / 1.13x; the passes are L2-resident there, so the doubled HBM
# passes cost little, but the launches double.  Expected: levels 5-8 pass work -15 %, strips
# +0-2 %.  Cut-offs 0 (default) / 700 (levels 7-8) / 1100 (4-8) / 1700 (3-8), parity first.
set -o pipefail
mkdir -p gpurun_out/r5_k2
TVL1_BATCH_K2_W=1700 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_batch.py::test_batch_matches_oracle" > gpurun_out/r5_k2/parity.log 2>&1 || { tail -20 gpurun_out/r5_k2/parity.log; exit 1; }
tail -1 gpurun_out/r5_k2/parity.log
export BENCH_FLAGS="--workload strips --steps 3"
bash tools/ab_env.sh 2 "TVL1_BATCH_K2_W=0" "TVL1_BATCH_K2_W=700" "TVL1_BATCH_K2_W=1100" "TVL1_BATCH_K2_W=1700" > gpurun_out/r5_k2/ab.txt 2>&1
# (the knob this A/B used was removed after it; see result.txt and DESIGN 9)
