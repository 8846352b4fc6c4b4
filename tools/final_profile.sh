#!/bin/bash
# The round's evidence set from ONE box (so the hand checks compare like with like): the
# default bench line, one C2 pair alone (kernel trace + stats, PMC bytes, VALU issue, SQ
# stall split) and one strip batch alone (kernel trace + PMC), summarised for profiles/.
# Usage (GPU box, repo root): bash tools/final_profile.sh <tag>
set -o pipefail
tag=${1:-final}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python bench.py > $out/bench_c2.json 2> $out/bench_c2.err || { echo BENCH_FAIL; tail -5 $out/bench_c2.err; exit 1; }
TVL1_SPEC=0 bash tools/pmc_single.sh ${tag}_pair || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_${tag}_pair --emit-traffic $out/traffic.json > $out/pmc_summary_single_pair.txt || exit 1
TVL1_SPEC=0 bash tools/pmc_stall.sh ${tag} || exit 1
bash tools/pmc_strips.sh ${tag}_strips || exit 1
cp gpurun_out/prof_${tag}_pair/trace/run_kernel_stats.csv $out/kernel_stats_single_pair.csv
cp gpurun_out/stall_${tag}/summary.txt $out/pmc_stall_single_pair.txt
cp gpurun_out/prof_${tag}_strips/trace/run_kernel_stats.csv $out/kernel_stats_strip_batch.csv
cp gpurun_out/prof_${tag}_strips/pmc_summary.txt $out/pmc_summary_strip_batch.txt
cp gpurun_out/prof_${tag}_strips/traffic_strips.json $out/traffic_strips.json
rocm-smi --showclocks --showproductname > $out/box.txt 2>&1 || true
echo done
