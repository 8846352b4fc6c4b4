#!/bin/bash
# One pair alone (--inflight 1): the SQ wave-cycle split per kernel (WAIT_ANY = parked on
# s_waitcnt / barrier, WAIT_INST_ANY = issue stalls, ACTIVE_INST_ANY = issuing) and the LDS
# counters, two --pmc passes; summarised by tools/pmc_probe.py.
# Usage (GPU box, repo root): bash tools/pmc_stall.sh <tag> [bench args]
set -o pipefail
tag=${1:-stall}; shift
out=gpurun_out/stall_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="bench.py --steps 1 --warmup 1 --inflight 1 --no-cpu-baseline --no-fast-math-line --no-strips-line --no-kernel-timing $*"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU --output-format csv -d $out/a -o run -- python3 $B > $out/a.log 2>&1 || { echo PMC_FAIL_A; tail -5 $out/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $out/b -o run -- python3 $B > $out/b.log 2>&1 || { echo PMC_FAIL_B; tail -5 $out/b.log; exit 1; }
python3 tools/pmc_probe.py $out/a $out/b > $out/summary.txt
echo done
