set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU --output-format csv -d gpurun_out/pmcp/a -o run -- tools/_bin/wi_probe 6144 4096 3 > gpurun_out/pmcp/a.log 2>&1 || { echo FAIL_A; tail -5 gpurun_out/pmcp/a.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAVES --output-format csv -d gpurun_out/pmcp/b -o run -- tools/_bin/wi_probe 6144 4096 3 > gpurun_out/pmcp/b.log 2>&1 || { echo FAIL_B; tail -5 gpurun_out/pmcp/b.log; exit 1; }
python3 tools/pmc_probe.py gpurun_out/pmcp/a gpurun_out/pmcp/b
