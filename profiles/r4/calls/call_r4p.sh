#!/bin/bash
# r4: the driver's multi-GPU command form on the default pair workload (2 gloo ranks on the
# one GPU), then the 40,860-pair TIFF strip job through the CLI on the final r4 engine.
set -o pipefail
out=gpurun_out/r4p
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_stack.py -k "plain_launch" > $out/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 1000 python -u tools/cli_e2e.py --slices 401 --format tiff --jobs strips --strides 1-120 --strip-batch 256 --no-single-thread --out /tmp/e2e_tiff > $out/cli_e2e_tiff_long.txt 2>&1 || { echo E2E_FAIL; tail -20 $out/cli_e2e_tiff_long.txt; exit 1; }
cat $out/cli_e2e_tiff_long.txt
echo ALL_DONE
