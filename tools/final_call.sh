# Round-end GPU call: the whole -m gpu suite, smoke(), then the evidence set (tools/final_profile.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/gpu_tests_final.log; exit 1; }
tail -1 gpurun_out/gpu_tests_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -2 gpurun_out/smoke_final.log
bash tools/final_profile.sh ${TAG:-final} > gpurun_out/final_profile.log 2>&1 || { echo PROFILE_FAIL; tail -20 gpurun_out/final_profile.log; exit 1; }
grep '^{' gpurun_out/${TAG:-final}/bench_c2.json | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("C2", d["value"], "frac", d["roofline"]["frac"], "strips", d["production_strips"]["value"], d["production_strips"]["roofline"]["frac"])'
