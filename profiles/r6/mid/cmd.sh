# r6: the mid-check pass (k_iterate_roll_mid) with TVL1_MID=1 against the same engine without
# it (then the default), in one call: its parity tests, two alternating bench rounds
# (tools/knob_sweep.sh), then the whole -m gpu suite.  Expected before it ran: +2-3 % C2 in
# flight (5 mid-check passes replace 10 two-iteration passes on the C2 pair, about 1.3 ms of
# iteration kernels per pair).
set -o pipefail
mkdir -p gpurun_out/r6m
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "mid or benchmark_pair_bit_exact" > gpurun_out/r6m/parity_mid.txt 2>&1 || { echo PARITY_FAIL; tail -30 gpurun_out/r6m/parity_mid.txt; exit 1; }
tail -3 gpurun_out/r6m/parity_mid.txt
bash tools/knob_sweep.sh "TVL1_MID=1" "" > gpurun_out/r6m/ab_mid.txt 2>&1 || { echo AB_FAIL; cat gpurun_out/r6m/ab_mid.txt; exit 1; }
cat gpurun_out/r6m/ab_mid.txt
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6m/gpu_tests.txt 2>&1 || { echo SUITE_FAIL; tail -30 gpurun_out/r6m/gpu_tests.txt; exit 1; }
tail -3 gpurun_out/r6m/gpu_tests.txt
