#!/bin/bash
# r6: why kb_iterate_roll<7,2> / <8,2> returned wrong residuals in r5.
# CPU only.  Builds probe.hip (the batched pass at K = 4, 6, 7, 8) against the headers as
# committed just before the early-clobber fix (d91c53a^) and at HEAD, with the passes' flags,
# and scans the ISA for LDS reads whose destination holds the address of a later read of the
# same run (tests/test_kernel_fence_cpu.py's scan).
set -e
T=$(mktemp -d)
mkdir -p $T/pre/fibsem-optflow_amd/csrc $T/pre/include
for f in fibsem-optflow_amd/csrc/tvl1_kernels.hpp fibsem-optflow_amd/csrc/tvl1_batch.hpp include/tvl1.h; do
  git show d91c53a^:$f > $T/pre/$f
done
for v in pre head; do
  if [ $v = pre ]; then I="-I $T/pre/include -I $T/pre/fibsem-optflow_amd/csrc"; else I="-I include -I fibsem-optflow_amd/csrc"; fi
  /opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 \
    -mllvm -amdgpu-sched-strategy=max-ilp --cuda-device-only -c $I profiles/r6/k7k8/probe.hip -o $T/$v.co
  /opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/$v.co \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/$v.o
  /opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn $T/$v.o > $T/$v.s
  python3 - $T/$v.o $T/$v.s $v <<'PY'
import sys
sys.path[:0] = ["tools", "tests"]
import kernel_resources as kr, test_kernel_fence_cpu as t
o, s, v = sys.argv[1:]
for k in kr.notes(o):
    print(v, k[".name"], "vgpr", k[".vgpr_count"], "agpr", k.get(".agpr_count"))
ov = t.lds_read_overlaps(open(s).read())
print(v, "overlapping LDS reads:", len(ov))
for kern, ins in ov:
    print("  ", kern, "|", ins)
PY
done
rm -rf $T
