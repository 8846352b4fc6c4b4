#!/bin/bash
# r5: one 256-strip batch at a time under the kernel trace, for the per-level split of the
# production workload (tools/trace_levels.py --levels 9).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_strips_levels; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d $O -o run -- python3 bench.py --workload strips --steps 1 --warmup 1 --inflight 1 --no-cpu-baseline --no-kernel-timing > $O/bench.json 2> $O/bench.err
