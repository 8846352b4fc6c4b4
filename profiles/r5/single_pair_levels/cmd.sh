#!/bin/bash
# r5: one C2 pair at a time (one stream) under the kernel trace, for the per-level split
# (tools/trace_levels.py) beside the batched path's (profiles/r5/ab/batch_c2_trace/).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_single; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d $O -o run -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-fast-math-line --no-strips-line --no-kernel-timing > $O/bench.json 2> $O/bench.err
