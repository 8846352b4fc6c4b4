# One diagnostic run of the GPU suite with per-launch checks (TVL1_CHECK=1): a fault
# is reported with the kernel, level, warp and iteration it happened in.
set -o pipefail
mkdir -p gpurun_out
TVL1_CHECK=1 timeout -k 10 300 python -m pytest tests -x -q -m gpu > gpurun_out/diag.log 2>&1
rc=$?
grep -E "failed at|passed|failed|TVL1Error" gpurun_out/diag.log | head -8
exit $rc
