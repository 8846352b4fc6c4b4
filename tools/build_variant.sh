# Builds an engine library variant into DIR from the working tree: per-TU extra flags.
# Usage: bash tools/build_variant.sh DIR "<engine-TU extra flags>" "<passes-TU extra flags>"
# (the Makefile's flags otherwise; e.g. "-mllvm -amdgpu-sched-strategy=max-ilp -DTVL1_ROLL_LDS=0")
set -e
D=$1; EF=$2; PF=$3
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall --offload-arch=gfx950"
C=fibsem-optflow_amd/csrc
mkdir -p "$D"
/opt/rocm/bin/hipcc $F $EF -c $C/tvl1_engine.hip -o "$D/engine.o" &
/opt/rocm/bin/hipcc $F $PF -c $C/tvl1_passes.hip -o "$D/passes.o" &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o "$D/libtvl1_hip.so" "$D/engine.o" "$D/passes.o"
rm -f "$D/engine.o" "$D/passes.o"
