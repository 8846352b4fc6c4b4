"""Register-allocation fence over the shipped kernels.

r5's probe of batched passes of 7 and 8 iterations (`kb_iterate_roll<7,2>`, `<8,2>`: 275 and
309 VGPRs, i.e. 256 architectural VGPRs plus 19 / 53 AGPRs used as spill space) returned
wrong residuals (`profiles/r5/ab/batch_kmax/probe_k7_k8_128px.txt`).  The cause, found on
the CPU from the ISA of that build (`profiles/r6/k7k8/`): at that register
pressure the allocator gave the first `ds_read_b64` of `roll_lds_read`'s inline asm a
destination pair that contains the address VGPR the eight following reads of the same asm
block still use (`ds_read_b64 v[2:3], v2` then `ds_read_b64 ..., v2 offset:512`), because the
outputs were not marked early-clobber.  Every K <= 6 build allocated them apart, which is why
only K = 7, 8 failed.  HEAD marks them `=&v`.

This test fences all three conditions on what is shipped:
  * every kernel in lib/libtvl1_hip.so: at most 256 VGPRs, no AGPRs, no VGPR spills and no
    scratch (private segment 0), from the code-object metadata of both translation units;
  * in the emitted ISA, no load of a run of LDS reads that share one address register writes
    that register while a later read of the run still uses it;
  * in the sources, every multi-instruction inline-asm block marks its write-only outputs
    early-clobber (`=&`).
CPU only: it reads the built library (hipcc cross-compiles it in `build()`)."""
import re
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
LIB = ROOT / "fibsem-optflow_amd" / "lib" / "libtvl1_hip.so"
CSRC = ROOT / "fibsem-optflow_amd" / "csrc"
sys.path.insert(0, str(ROOT / "tools"))
import kernel_resources as kr  # noqa: E402


@pytest.fixture(scope="module")
def objects(tmp_path_factory):
    if not LIB.exists():
        pytest.skip("lib/libtvl1_hip.so not built (run __graft_entry__.build())")
    return kr.so_objects(LIB, tmp_path_factory.mktemp("co"))


@pytest.fixture(scope="module")
def kernels(objects):
    ks = [k for o in objects for k in kr.notes(o)]
    assert len(ks) >= 100, f"expected the engine's kernels, found {len(ks)}"
    return ks


def test_reading_the_library_leaves_it_untouched(tmp_path):
    """so_objects must not write the library: objcopy given only an input rewrites it in place,
    which made a pytest process that had the engine loaded (tests/test_homography_cpu.py) die
    with SIGSEGV at exit after every test passed (r6)."""
    if not LIB.exists():
        pytest.skip("lib/libtvl1_hip.so not built")
    before = LIB.stat()
    kr.so_objects(LIB, tmp_path)
    after = LIB.stat()
    assert (after.st_mtime_ns, after.st_size) == (before.st_mtime_ns, before.st_size)


def test_two_translation_units(objects):
    # tvl1_engine.hip and tvl1_passes.hip: both bundles must be read
    assert len(objects) == 2


def test_register_ceiling_and_no_scratch(kernels):
    bad = []
    for k in kernels:
        name = k[".name"]
        v, a = int(k[".vgpr_count"]), int(k.get(".agpr_count", 0))
        spill, scratch = int(k.get(".vgpr_spill_count", 0)), int(k.get(".private_segment_fixed_size", 0))
        if v > 256 or a > 0 or spill > 0 or scratch > 0:
            bad.append((name, v, a, spill, scratch))
    assert not bad, f"kernels past the 256-VGPR / no-scratch fence: {bad}"


def _regs(op):
    op = op.rstrip(",")
    m = re.match(r"v\[(\d+):(\d+)\]$", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", op)
    return {int(m.group(1))} if m else set()


def lds_read_overlaps(text):
    """(kernel, instruction) for every LDS read whose destination holds the address register of
    a later read in the same run of consecutive LDS reads on that address."""
    out, kern = [], None
    lines = [l.split("//")[0].strip() for l in text.split("\n")]
    for i, l in enumerate(lines):
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", l)
        if m:
            kern = m.group(1)
            continue
        p = l.split()
        if len(p) < 3 or not p[0].startswith("ds_read"):
            continue
        addr = p[2].rstrip(",")
        dest = _regs(p[1])
        for j in range(i + 1, len(lines)):
            q = lines[j].split()
            if len(q) < 3 or not q[0].startswith("ds_read"):
                break
            if q[2].rstrip(",") == addr and dest & _regs(addr):
                out.append((kern, l))
                break
    return out


def test_self_test_of_the_overlap_scan():
    bad = ("0 <k>:\n ds_read_b64 v[2:3], v2\n ds_read_b64 v[4:5], v2 offset:512\n")
    good = ("0 <k>:\n ds_read_b64 v[4:5], v2\n ds_read_b64 v[6:7], v2 offset:512\n")
    last = ("0 <k>:\n ds_read_b64 v[4:5], v2\n ds_read_b64 v[2:3], v2 offset:512\n")
    assert lds_read_overlaps(bad) == [("k", "ds_read_b64 v[2:3], v2")]
    assert lds_read_overlaps(good) == []
    assert lds_read_overlaps(last) == []   # the last read of a run may reuse its address


def test_no_lds_read_overwrites_a_live_address(objects):
    found = []
    for o in objects:
        text = subprocess.run([str(kr.LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", str(o)],
                              check=True, capture_output=True, text=True).stdout
        found += lds_read_overlaps(text)
    assert not found, found


def asm_blocks(src):
    """(template, outputs) of every `asm volatile(...)` statement of a C++ source."""
    out = []
    for m in re.finditer(r"asm\s+volatile\s*\(", src):
        i, depth, instr, j = m.end(), 1, False, m.end()
        while depth:
            c = src[j]
            if instr:
                if c == "\\":
                    j += 1
                elif c == '"':
                    instr = False
            elif c == '"':
                instr = True
            elif c == "(":
                depth += 1
            elif c == ")":
                depth -= 1
            j += 1
        # drop // comments (outside string literals): they may hold ':'
        body = "\n".join(re.sub(r'^((?:[^"/]|"(?:[^"\\]|\\.)*")*)//.*$', r"\1", ln)
                         for ln in src[i:j - 1].split("\n"))
        parts, depth, instr, cur = [], 0, False, ""
        k = 0
        while k < len(body):   # split on top-level ':'
            c = body[k]
            if instr:
                cur += c
                if c == "\\":
                    cur += body[k + 1]
                    k += 1
                elif c == '"':
                    instr = False
            elif c == '"':
                instr = True
                cur += c
            elif c in "([":
                depth += 1
                cur += c
            elif c in ")]":
                depth -= 1
                cur += c
            elif c == ":" and depth == 0:
                parts.append(cur)
                cur = ""
            else:
                cur += c
            k += 1
        parts.append(cur)
        template = "".join(re.findall(r'"((?:[^"\\]|\\.)*)"', parts[0]))
        outputs = re.findall(r'"([^"]*)"\s*\(', parts[1]) if len(parts) > 1 else []
        out.append((template, outputs))
    return out


def test_multi_instruction_asm_outputs_are_early_clobber():
    checked, bad = 0, []
    for f in sorted(CSRC.glob("*.h*")) + sorted(CSRC.glob("*.inc")):
        for template, outputs in asm_blocks(f.read_text()):
            insts = [t for t in template.split("\\n") if t.strip()]
            if len(insts) < 2:
                continue
            checked += 1
            for c in outputs:
                if c.startswith("=") and not c.startswith("=&"):
                    bad.append((f.name, insts[0], c))
    assert checked >= 1, "the LDS row read (roll_lds_read) should be found"
    assert not bad, f"multi-instruction asm with non-early-clobber outputs: {bad}"


def test_parser_finds_the_row_read_constraints():
    src = (CSRC / "tvl1_kernels.hpp").read_text()
    blocks = [b for b in asm_blocks(src) if "ds_read_b64 %8, %9 offset:4608" in b[0]]
    assert len(blocks) == 1
    assert blocks[0][1] == ["=&v"] * 9


def test_no_waterfall_loops(objects):
    """A buffer descriptor the compiler cannot prove uniform is rebuilt per lane in a
    `v_readfirstlane_b32` x 4 / `v_cmp_eq_u64` / `s_and_saveexec` loop around every load
    (cdna_hip_programming.md T20).  r6 found kb_warp_iter (the strips' fused first pass) and
    kb_warp_ring doing that on every load of the gather -- 703 and 463 readfirstlanes, ~100
    extra instructions per producer step -- because the pair index read from the kernel
    arguments by blockIdx.y was not known uniform; it is now readfirstlane'd.  No shipped
    kernel may hold the pattern again."""
    bad = []
    for o in objects:
        text = subprocess.run([str(kr.LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", str(o)],
                              check=True, capture_output=True, text=True).stdout
        kern, rfl, cmp64 = None, 0, 0
        for line in text.split("\n") + ["0 <end>:"]:
            m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
            if m:
                if kern and (rfl > 16 or cmp64 > 8):
                    bad.append((kern, rfl, cmp64))
                kern, rfl, cmp64 = m.group(1), 0, 0
                continue
            rfl += "v_readfirstlane_b32" in line
            cmp64 += "v_cmp_eq_u64" in line
    assert not bad, f"waterfall loops (kernel, readfirstlanes, 64-bit compares): {bad}"
