#!/bin/bash
# Instruction-class counters for the issue model (tools/issue_model.py): one C2 pair alone
# (--inflight 1, TVL1_SPEC=0 so no empty speculative launch enters the per-dispatch
# averages) or one production-strip batch alone (--strips), a kernel trace for durations
# and four --pmc passes of at most 8 SQ counters + GRBM_GUI_ACTIVE each:
#   a: VALU by class (all, transcendental f32, f64 add/mul/fma, cvt, int32) + SQ_WAVES
#   b: f32 add/mul/fma, LDS, SALU, SMEM, BRANCH, VMEM instruction counts
#   c: the wave-cycle split (WAVE_CYCLES, WAIT_ANY, WAIT_INST_ANY, ACTIVE_INST_*)
#   d: SQ_INSTS, dual VALU issue, LDS array cycles, busy cycles
# Usage (GPU box, repo root): bash tools/pmc_issue.sh <tag> [--strips] [bench args]
set -o pipefail
tag=${1:-issue}; shift
if [ "$1" = "--strips" ]; then
  shift
  LV="none:1:1"   # every strip level has its own grid size
  B="bench.py --workload strips --width 3072 --height 100 --nscales 10 --warps 5 --batch 256 --steps 1 --warmup 1 --inflight 1 --no-cpu-baseline $*"
else
  LV="k_warp_iter<:5:30"   # C2: 5 levels x 30 warps, one k_warp_iter per warp
  B="bench.py --steps 1 --warmup 1 --inflight 1 --no-cpu-baseline --no-fast-math-line --no-strips-line $*"
fi
out=gpurun_out/issue_$tag      # summaries (merged back)
raw=/tmp/issue_raw_$tag        # rocprofv3 output (tens of MB: stays on the box)
mkdir -p $out $raw
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export TVL1_SPEC=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $raw/trace -o run -- python3 $B > $out/bench_trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $out/bench_trace.log; exit 1; }
run_pass() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $raw/pmc_$name -o run -- python3 $B --no-kernel-timing > $out/bench_$name.log 2>&1 || { echo PMC_FAIL $name; tail -5 $out/bench_$name.log; exit 1; }
}
run_pass a SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_WAVES GRBM_GUI_ACTIVE || exit 1
run_pass b SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM GRBM_GUI_ACTIVE || exit 1
run_pass c SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE || exit 1
run_pass d SQ_INSTS SQ_ACTIVE_INST_VALU2 SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE || exit 1
python3 tools/issue_model.py --collect $raw --levels "$LV" > $out/pmc_issue.csv || exit 1
cp $raw/trace/run_kernel_stats.csv $out/kernel_stats.csv
echo done
