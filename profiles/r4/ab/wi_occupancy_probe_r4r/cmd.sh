#!/bin/bash
# r4: k_warp_iter occupancy probe (dynamic LDS capping it at 5 / 4 / 3 blocks per CU, segments
# sized for that residency), one C2 pair at a time, kernel trace.
set -o pipefail
out=gpurun_out/r4r
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for pad in 0 8192 20000; do
  TVL1_PROBE_WI_LDS=$pad timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/wi$pad -o run -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-fast-math-line --no-strips-line > $out/wi$pad.log 2>&1 || { echo TRACE_FAIL; tail -5 $out/wi$pad.log; exit 1; }
  echo "pad $pad: $(find $out/wi$pad -name '*kernel_stats.csv' -exec grep -h 'k_warp_iter' {} \; | awk -F'",' '{print $2}' | cut -d, -f1-3)"
done
echo PROBE_DONE
