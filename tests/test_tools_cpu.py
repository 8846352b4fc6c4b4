"""tools/ holds only scripts that run against HEAD: every shell script
parses (`bash -n`), every Python tool compiles, every engine knob a tool names exists in the
engine sources, and the probes that include the engine headers still compile for gfx950.
One-off GPU call scripts live beside the outputs they produced (profiles/rN/.../cmd.sh)."""
from __future__ import annotations

import py_compile
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
TOOLS = ROOT / "tools"
CSRC = ROOT / "fibsem-optflow_amd" / "csrc"


def _knobs_in(paths):
    out = set()
    for p in paths:
        out |= set(re.findall(r"TVL1_[A-Z0-9_]+", p.read_text(errors="replace")))
    return out


def test_shell_scripts_parse():
    scripts = sorted(TOOLS.glob("*.sh"))
    assert scripts
    for s in scripts:
        r = subprocess.run(["bash", "-n", str(s)], capture_output=True, text=True)
        assert r.returncode == 0, (s.name, r.stderr)


def test_python_tools_compile(tmp_path):
    for s in sorted(TOOLS.glob("*.py")):
        py_compile.compile(str(s), cfile=str(tmp_path / (s.stem + ".pyc")), doraise=True)


def test_no_one_off_call_scripts_in_tools():
    assert not list(TOOLS.glob("call_r*.sh")), "one-off GPU calls belong beside their outputs"


def test_tool_knobs_exist_in_engine():
    engine = _knobs_in(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.hpp")) +
                       [CSRC / "tvl1_passes.inc"])
    engine |= _knobs_in([ROOT / "fibsem-optflow_amd" / "optflow_amd" / "capi.py"])
    for s in sorted(list(TOOLS.glob("*.sh")) + list(TOOLS.glob("*.py"))):
        missing = _knobs_in([s]) - engine
        assert not missing, (s.name, sorted(missing))


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="no hipcc")
@pytest.mark.parametrize("probe", ["wi_probe.hip", "div_check.hip", "sqrt_check.hip"])
def test_engine_probes_compile(probe, tmp_path):
    """The probes that include the engine's headers build against HEAD (device code
    only, syntax and semantics: no link, so no GPU needed)."""
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O1", "--offload-arch=gfx950",
                        "-ffp-contract=off", "-I", "include", "-I", "fibsem-optflow_amd/csrc",
                        "-fsyntax-only", str(TOOLS / probe)],
                       capture_output=True, text=True, cwd=str(ROOT), timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
