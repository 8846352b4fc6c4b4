set -o pipefail
T=r6final2
mkdir -p gpurun_out/$T/issue
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "mid" > gpurun_out/$T/parity_mid.txt 2>&1 || { echo PARITY_FAIL; tail -30 gpurun_out/$T/parity_mid.txt; exit 1; }
tail -1 gpurun_out/$T/parity_mid.txt
bash tools/knob_sweep.sh "" "TVL1_MID=0" > gpurun_out/$T/ab_mid.txt 2>&1 || { echo AB_FAIL; cat gpurun_out/$T/ab_mid.txt; exit 1; }
cat gpurun_out/$T/ab_mid.txt
bash tools/pmc_issue.sh ${T}c2 > gpurun_out/$T/pmc_issue.log 2>&1 || { echo ISSUE_FAIL; tail -20 gpurun_out/$T/pmc_issue.log; exit 1; }
cp gpurun_out/issue_${T}c2/pmc_issue.csv profiles/r6/issue/pmc_issue_c2.csv && cp gpurun_out/issue_${T}c2/kernel_stats.csv profiles/r6/issue/kernel_stats_c2.csv || exit 1
python3 tools/issue_model.py --dump-isa profiles/r6/issue > gpurun_out/$T/isa_dump.log 2>&1 || { echo ISA_FAIL; tail gpurun_out/$T/isa_dump.log; exit 1; }
python3 tools/issue_model.py --model --json profiles/r6/issue/model.json > profiles/r6/issue/model.txt || { echo MODEL_FAIL; exit 1; }
cp profiles/r6/issue/model.json profiles/r6/issue/model.txt profiles/r6/issue/pmc_issue_c2.csv profiles/r6/issue/kernel_stats_c2.csv profiles/r6/issue/*.s gpurun_out/$T/issue/ || exit 1
TVL1_SPEC=0 bash tools/pmc_single.sh ${T}_pair > gpurun_out/$T/pmc_single.log 2>&1 || { echo SINGLE_FAIL; tail -20 gpurun_out/$T/pmc_single.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/prof_${T}_pair --emit-traffic profiles/traffic.json > gpurun_out/$T/pmc_summary_single_pair.txt || { echo SUMMARY_FAIL; exit 1; }
cp profiles/traffic.json gpurun_out/$T/traffic.json && cp gpurun_out/prof_${T}_pair/trace/run_kernel_stats.csv gpurun_out/$T/kernel_stats_single_pair.csv || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/gpu_tests.txt 2>&1 || { echo SUITE_FAIL; tail -30 gpurun_out/$T/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/$T/bench_c2.json 2> gpurun_out/$T/bench_c2.err || { echo BENCH_FAIL; tail -5 gpurun_out/$T/bench_c2.err; exit 1; }
tail -1 gpurun_out/$T/bench_c2.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("C2", d["value"], d["roofline"]["bound"], d["roofline"]["frac"], "strips", d["production_strips"]["value"])'
rocm-smi --showclocks --showproductname > gpurun_out/$T/box.txt 2>&1 || true
