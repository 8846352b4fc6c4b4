#!/bin/bash
# r5: the strips' coarsest level on chip (kb_small_level, one workgroup per pair) -- the
# whole batch parity matrix first (its strip-shaped cases' coarsest levels take the new
# kernel; TVL1_BATCH_SMALL=0 keeps the streaming path), then strips A/B against =0.
# Expected: level 8 (515 x 17, 204 iterations per pair) from ~4.7 ms per 256-strip batch
# (89 launches, ~45 host round trips) to ~1 ms; strips +2-4 %.  A one-batch kernel trace
# gives the level split (tools/trace_levels.py --levels 9).
set -o pipefail
O=gpurun_out/r5_small; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py > $O/batch_tests.log 2>&1 || { tail -30 $O/batch_tests.log; exit 1; }
tail -1 $O/batch_tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d $O/trace -o run -- python3 bench.py --workload strips --steps 1 --warmup 1 --inflight 1 --no-cpu-baseline --no-kernel-timing > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
export BENCH_FLAGS="--workload strips --steps 3"
bash tools/ab_env.sh 3 "TVL1_BATCH_SMALL=0" "TVL1_BATCH_SMALL=1" > $O/ab.txt 2>&1
