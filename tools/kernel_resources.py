#!/usr/bin/env python3
"""Per-kernel register / spill / LDS figures of the gfx950 code object (the code-object
notes: .vgpr_count, .sgpr_count, .vgpr_spill_count, .sgpr_spill_count,
.group_segment_fixed_size), for every kernel the engine library holds.

    python tools/kernel_resources.py [--out profiles/r2/kernel_resources.txt]

Compiles csrc/tvl1_engine.hip and csrc/tvl1_passes.hip device-only with the Makefile's flags (about 25 s, no GPU
needed), unbundles the gfx950 object and reads its notes with llvm-readelf."""
import argparse
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
LLVM = Path("/opt/rocm/lib/llvm/bin")
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "--offload-arch=gfx950"]
PASSFLAGS = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]   # Makefile PASSFLAGS
FIELDS = (".vgpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
          ".group_segment_fixed_size", ".max_flat_workgroup_size")


def notes(obj):
    out = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(obj)], check=True,
                         capture_output=True, text=True).stdout
    kernels, cur = [], {}
    # each kernel's metadata map lists its fields in alphabetical order, after its .args
    # list (whose items also start with "- ."); a map that holds .sgpr_count is a kernel's
    for line in out.splitlines():
        s = line.strip()
        if s.startswith("- .args:") or s == "- .agpr_count:" or re.match(r"^- \.\w", s):
            if cur.get(".name") and ".sgpr_count" in cur:
                kernels.append(cur)
            cur = {}
            s = s[2:]
        m = re.match(r"^(\.[a-z_]+):\s+(\S+)$", s)
        if m and (m.group(1) in FIELDS or m.group(1) == ".name"):
            cur[m.group(1)] = m.group(2)
    if cur.get(".name") and ".sgpr_count" in cur:
        kernels.append(cur)
    return kernels


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), check=True,
                         capture_output=True, text=True).stdout.splitlines()
    return [re.sub(r"^tvl1k::", "", o) for o in out]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    args = ap.parse_args()
    ks = []
    with tempfile.TemporaryDirectory() as d:
        # the two translation units of lib/libtvl1_hip.so, each with its Makefile flags
        for src, extra in (("tvl1_engine.hip", []), ("tvl1_passes.hip", PASSFLAGS)):
            co, obj = Path(d) / f"{src}.co", Path(d) / f"{src}.950.o"
            subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "--cuda-device-only", "-c",
                            "-I", str(ROOT / "include"), "-I", str(ROOT / "fibsem-optflow_amd/csrc"),
                            str(ROOT / "fibsem-optflow_amd/csrc" / src), "-o", str(co)],
                           check=True)
            subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o",
                            f"--input={co}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                            f"--output={obj}"], check=True)
            ks += notes(obj)
    names = demangle([k[".name"] for k in ks])
    rows = sorted(zip(names, ks), key=lambda t: t[0])
    hdr = f"{'kernel':<90} {'VGPR':>5} {'SGPR':>5} {'Vspill':>6} {'Sspill':>6} {'LDS':>6} {'WG':>5}"
    lines = [f"# gfx950 code-object notes of csrc/tvl1_engine.hip + tvl1_passes.hip ({len(rows)} kernels; "
             f"hipcc {' '.join(FLAGS)}; passes + {' '.join(PASSFLAGS)})", hdr]
    for n, k in rows:
        lines.append(f"{n[:90]:<90} {k.get('.vgpr_count', '?'):>5} {k.get('.sgpr_count', '?'):>5} "
                     f"{k.get('.vgpr_spill_count', '?'):>6} {k.get('.sgpr_spill_count', '?'):>6} "
                     f"{k.get('.group_segment_fixed_size', '?'):>6} "
                     f"{k.get('.max_flat_workgroup_size', '?'):>5}")
    text = "\n".join(lines) + "\n"
    if args.out:
        Path(args.out).write_text(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
