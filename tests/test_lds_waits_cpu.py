"""The hand-written waits of the LDS-staged rolling passes (`roll_step_lds`):
each input row reaches LDS through 5 buffer-to-LDS loads, and the step that reads it waits
with a counted `s_waitcnt vmcnt(17)` that the compiler does not check.  vmcnt retires in
issue order, so the wait is right only if at least 17 vector-memory instructions were issued
after the row's 5 loads by the time of the wait.  This test compiles the passes' translation
unit for gfx950 with the Makefile's flags and checks that invariant on the code the compiler
emitted, for every kernel that stages rows in LDS (a change to the stores per step, or a
scheduler that moved them, fails here instead of as a rare wrong bit on the GPU).  CPU-only:
hipcc cross-compiles."""
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "fibsem-optflow_amd" / "csrc"
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "--offload-arch=gfx950",
         "-mllvm", "-amdgpu-sched-strategy=max-ilp"]   # Makefile HIPFLAGS + PASSFLAGS
PIECES, WAIT = 5, 17
# mangled-name fragments of the kernels with LDS-staged rows (G = 0, K = 3, 4, PX = 2; every
# arithmetic mode)
# (fragment, counted wait, stores per step)
LDS_KERNELS = [(f"k_iterate_rollILb0ELi{k}ELi2ELi{fm}E", WAIT, 6) for k in (3, 4) for fm in (0, 1, 2)] + \
              [(f"kb_iterate_rollILi{k}ELi2ELi{fm}E", WAIT, 6) for k in (3, 4) for fm in (0, 1, 2)] + \
              [(f"k_iterate_roll_midILi{fm}E", WAIT, 6) for fm in (0, 1, 2)]


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not Path(HIPCC).exists():
        pytest.skip("hipcc not present")
    out = tmp_path_factory.mktemp("isa") / "passes.s"
    subprocess.run([HIPCC, *FLAGS, "--cuda-device-only", "-S", "-I", str(ROOT / "include"),
                    str(CSRC / "tvl1_passes.hip"), "-o", str(out)], check=True,
                   capture_output=True)
    return out.read_text().split("\n")


def kernel_body(lines, frag):
    for i, ln in enumerate(lines):
        if re.match(r"^_Z\S+:", ln) and frag in ln.split(":")[0]:
            j = i + 1
            while not lines[j].startswith(".Lfunc_end"):
                j += 1
            return lines[i:j]
    raise AssertionError(f"kernel {frag} not found")


def vmem_events(body):
    """(kind, text) in program order: D = buffer load to LDS, S = store, L = load, W = a
    vmcnt wait."""
    ev = []
    for ln in body:
        t = ln.strip()
        if t.startswith("s_waitcnt") and "vmcnt" in t:
            ev.append(("W", t))
        elif re.match(r"^(buffer|global)_load", t) and t.endswith(" lds"):
            ev.append(("D", t))
        elif re.match(r"^(buffer|global)_store", t):
            ev.append(("S", t))
        elif re.match(r"^(buffer|global)_load", t):
            ev.append(("L", t))
    return ev


@pytest.mark.parametrize("frag,wait,stores", LDS_KERNELS)
def test_row_waits_cover_the_rows_pieces(asm, frag, wait, stores):
    ev = vmem_events(kernel_body(asm, frag))
    kinds = "".join("C" if k == "W" and t == f"s_waitcnt vmcnt({wait})" else k for k, t in ev)
    # C = the counted wait of a step.  The step loop is unrolled by 2 (one step per LDS
    # slot); the compiler may emit more than one copy of it (alternative paths), each entered
    # from the prologue.  Every step: the wait, the next row's PIECES loads, the stores.
    counted = [i for i, k in enumerate(kinds) if k == "C"]
    assert counted and len(counted) % 2 == 0, kinds
    prologue = kinds[kinds.index("D"):counted[0]]
    assert prologue.count("D") == 2 * PIECES and "C" not in prologue, kinds
    # after the loop(s): the refills land before the block's LDS is released
    assert ev[-1][1] == "s_waitcnt vmcnt(0)" or any(
        t == "s_waitcnt vmcnt(0)" for k, t in ev[counted[-1]:]), kinds
    for c in range(0, len(counted), 2):
        end = counted[c + 2] if c + 2 < len(counted) else len(kinds)
        body = kinds[counted[c]:end]
        steps = re.findall(r"C([^C]*)", body)
        assert len(steps) == 2, (frag, body)
        step = "D" * PIECES + "S" * stores
        for st in steps:
            assert st.replace("W", "").startswith(step), (frag, body)
        # Row k is the k-th group of PIECES loads (the prologue's rows r0, r0 + 1, then one
        # row per step) and is read after the k-th counted wait: count the VMEM instructions
        # issued between the end of its group and that wait, over three trips of the loop
        # (each step as the compiler ordered it; what follows the last step is the epilogue).
        seq = prologue + ("C" + step) * 6
        d_end, n_d = [], 0
        for i, k in enumerate(seq):
            if k == "D":
                n_d += 1
                if n_d % PIECES == 0:
                    d_end.append(i)
        for row, w in enumerate(i for i, k in enumerate(seq) if k == "C"):
            after = sum(1 for k in seq[d_end[row] + 1:w] if k in "DSL")
            assert after >= wait, (frag, row, after, seq)


def test_only_lds_kernels_stage_rows(asm):
    """The other rolling passes keep their register ring: no buffer load to LDS."""
    for frag in ("k_iterate_rollILb0ELi2ELi2ELi0E", "k_iterate_rollILb1ELi4ELi2ELi0E",
                 "k_iterate_rollILb0ELi2ELi4ELi0E", "kb_iterate_rollILi4ELi1ELi0E"):
        kinds = "".join(k for k, _ in vmem_events(kernel_body(asm, frag)))
        assert "D" not in kinds, (frag, kinds)
