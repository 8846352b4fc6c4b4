#!/bin/bash
# r5: kernel traces of C2 pairs through the pair path (3 ctxs in flight) and through
# tvl1_calc_batch (3 pairs per launch), to see which kernels make the batched path slower
# at full-frame geometry (profiles/r5/ab/batch_c2: -4.5 % per iteration).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_trace; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d $O/pair -o pair -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fast-math-line --no-strips-line --no-kernel-timing > $O/pair.json 2> $O/pair.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d $O/batch -o batch -- python3 bench.py --workload strips --width 6144 --height 4096 --nscales 5 --warps 30 --batch 3 --inflight 1 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/batch.json 2> $O/batch.err
