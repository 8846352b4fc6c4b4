#!/bin/bash
# r5 A/B (strips): the two batch slots free-running and staggered by half a batch (--stagger;
# the CLI's batch workers are free-running) against both starting every step together.  In
# lock step both batches reach the launch-bound coarse levels (levels 3-8: 36 % of a batch's
# kernel time at 1.3-2.4x level 0's cost per px-iteration, profiles/r5/strips_levels/) at the
# same moment; staggered, one batch's fine levels fill the GPU meanwhile.  Expected: strips
# +3-8 %.  Three alternations of 4 steps.
set -o pipefail
export BENCH_FLAGS="--workload strips --steps 4"
bash tools/ab_flags.sh 3 r5st "" "--stagger"   # (--stagger: removed after this A/B, commit history) > gpurun_out/r5_strips_stagger.txt 2>&1
