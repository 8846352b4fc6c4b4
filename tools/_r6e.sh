set -o pipefail
mkdir -p gpurun_out/r6e
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6e/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6e/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/ab_lib.sh ab_B --workload strips --steps 3 > gpurun_out/r6e/ab_strips.txt 2>&1 || exit 1
cat gpurun_out/r6e/ab_strips.txt
bash tools/pmc_issue.sh strips6 --strips || exit 1
timeout -k 10 300 python -u tools/cli_e2e.py --slices 401 --format tiff --jobs strips --strides 1-120 --no-single-thread --out /tmp/cli_stack > gpurun_out/r6e/cli_e2e.txt 2>&1 || { tail -5 gpurun_out/r6e/cli_e2e.txt; exit 1; }
timeout -k 10 200 python bench.py --workload strips > gpurun_out/r6e/bench_strips.json 2> gpurun_out/r6e/bench_strips.err || exit 1
tail -c 600 gpurun_out/r6e/cli_e2e.txt
