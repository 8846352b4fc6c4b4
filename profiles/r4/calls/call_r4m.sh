#!/bin/bash
# r4: batched parity after kb_iterate_roll's one-row lookahead, then a strips kernel trace
# (per-level split) and the strips bench.
set -o pipefail
out=gpurun_out/r4m
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_batch.py tests/test_cli_batch_gpu.py > $out/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/strips_trace -o run -- python3 bench.py --workload strips --steps 3 --warmup 1 --no-cpu-baseline > $out/strips_trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $out/strips_trace.log; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload strips --steps 3 --warmup 1 --no-cpu-baseline > $out/s$i.json 2>&1 || { echo STRIPS_FAIL; exit 1; }
  echo "strips round $i $(tail -1 $out/s$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
done | tee $out/strips.txt
echo ALL_DONE
