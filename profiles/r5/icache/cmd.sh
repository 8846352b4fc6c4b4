#!/bin/bash
# r5: is k_warp_iter (34.6 KB of code, 4 roles' loops live at once) instruction-fetch bound?
# SQ_WAIT_INST_ANY is 0.23 of its wave cycles.  Instruction-cache hits / misses and fetches
# of the kernel alone (tools/wi_probe.hip, level-0 geometry), of one C2 pair alone and of
# 3 pairs in flight (where k_iterate_roll / k_iterate_tb4 share the CUs' instruction caches).
# Expected if fetch-bound: misses a few % of requests, more in flight.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_icache; mkdir -p $O
C="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU"
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/probe -o run -- tools/_bin/wi_probe 6144 4096 3 > $O/probe.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $O/single -o run -- python3 bench.py --steps 1 --warmup 0 --inflight 1 --no-cpu-baseline --no-fast-math-line --no-strips-line --no-kernel-timing > $O/single.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $O/inflight -o run -- python3 bench.py --steps 1 --warmup 0 --inflight 3 --no-cpu-baseline --no-fast-math-line --no-strips-line --no-kernel-timing > $O/inflight.log 2>&1
