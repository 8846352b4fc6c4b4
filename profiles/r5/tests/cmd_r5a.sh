#!/bin/bash
# r5: the GPU tests touched this round (bench rank records under gloo and nccl, gather_flow's
# bound, the batched CLI, the 3-pair full-frame-geometry batch).
set -o pipefail
mkdir -p gpurun_out/r5_tests
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_lifecycle.py tests/test_gpu_stack.py tests/test_cli_batch_gpu.py "tests/test_gpu_batch.py::test_batch_of_full_frame_geometry_pairs" > gpurun_out/r5_tests/r5a.log 2>&1
