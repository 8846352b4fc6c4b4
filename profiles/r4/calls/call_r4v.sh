#!/bin/bash
# r4 end: the whole -m gpu suite and smoke() on the current tree, then the 40,860-pair TIFF
# strip job through the CLI on the final engine.
set -o pipefail
out=gpurun_out/r4v
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 1000 python -u tools/cli_e2e.py --slices 401 --format tiff --jobs strips --strides 1-120 --strip-batch 256 --no-single-thread --out /tmp/e2e_tiff > $out/cli_e2e_tiff_long.txt 2>&1 || { echo E2E_FAIL; tail -20 $out/cli_e2e_tiff_long.txt; exit 1; }
tail -1 $out/cli_e2e_tiff_long.txt
echo ALL_DONE
