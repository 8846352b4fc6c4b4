set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_ilp.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/gpu_tests_ilp.log; exit 1; }
tail -1 gpurun_out/gpu_tests_ilp.log
bash tools/ab_libs.sh 3 . ab_B ab_C > gpurun_out/ab_ilp_c2.txt 2>&1 || { cat gpurun_out/ab_ilp_c2.txt; exit 1; }
cat gpurun_out/ab_ilp_c2.txt
bash tools/ab_libs.sh 2 . ab_B ab_C -- --workload strips > gpurun_out/ab_ilp_strips.txt 2>&1 || { cat gpurun_out/ab_ilp_strips.txt; exit 1; }
cat gpurun_out/ab_ilp_strips.txt
bash tools/ab_kernels.sh ab_B > gpurun_out/ab_ilp_kernels.txt 2>&1 || { cat gpurun_out/ab_ilp_kernels.txt; exit 1; }
cat gpurun_out/ab_ilp_kernels.txt
bash tools/ab_kernels.sh ab_C > gpurun_out/ab_ilp_kernels_C.txt 2>&1 && cat gpurun_out/ab_ilp_kernels_C.txt
