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
          ".group_segment_fixed_size", ".max_flat_workgroup_size", ".agpr_count",
          ".private_segment_fixed_size")
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def so_objects(so, outdir):
    """The gfx950 code objects inside a built shared library (lib/libtvl1_hip.so): its
    .hip_fatbin section holds one offload bundle per translation unit; each is unbundled
    to outdir/tu<i>.o.  Returns the object paths."""
    outdir = Path(outdir)
    fat = outdir / "fatbin"
    # an explicit output file: given only the input, objcopy rewrites it in place -- the
    # library the calling process (or another) may have mapped, which then faulted at exit
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", str(so),
                    str(outdir / "so_copy")], check=True, capture_output=True)
    data = fat.read_bytes()
    starts = [m.start() for m in re.finditer(re.escape(BUNDLE_MAGIC), data)] + [len(data)]
    objs = []
    for i in range(len(starts) - 1):
        part = outdir / f"bundle{i}"
        part.write_bytes(data[starts[i]:starts[i + 1]])
        obj = outdir / f"tu{i}.o"
        subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o",
                        f"--input={part}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--output={obj}"], check=True)
        objs.append(obj)
    return objs


def notes(obj):
    """Per kernel, the code-object metadata fields in FIELDS (the AMDGPU metadata note,
    parsed as the YAML document it is)."""
    import yaml
    out = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(obj)], check=True,
                         capture_output=True, text=True).stdout
    lines = out.splitlines()
    i0 = next(i for i, l in enumerate(lines) if l.strip() == "---")
    i1 = next((i for i in range(i0 + 1, len(lines)) if lines[i].strip() == "..."), len(lines))
    meta = yaml.safe_load("\n".join(lines[i0 + 1:i1]))
    kernels = []
    for k in meta.get("amdhsa.kernels", []):
        kernels.append({f: str(k[f]) for f in FIELDS + (".name",) if f in k})
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
