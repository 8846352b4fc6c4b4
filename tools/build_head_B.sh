# Builds the engine as committed at a git revision (default HEAD) into ab_B/, for
# tools/ab_lib.sh A/B runs of the working tree against it.
set -e
REV=${1:-HEAD}
T=$(mktemp -d)
git archive "$REV" fibsem-optflow_amd/csrc include | tar -x -C "$T"
mkdir -p ab_B
if [ -f "$T/fibsem-optflow_amd/csrc/tvl1_passes.hip" ]; then   # two translation units (r3)
  git archive "$REV" fibsem-optflow_amd/Makefile | tar -x -C "$T"
  make -C "$T/fibsem-optflow_amd" lib/libtvl1_hip.so >/dev/null
  cp "$T/fibsem-optflow_amd/lib/libtvl1_hip.so" ab_B/
else
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall --offload-arch=gfx950 \
    -shared -o ab_B/libtvl1_hip.so "$T/fibsem-optflow_amd/csrc/tvl1_engine.hip"
fi
rm -rf "$T"
