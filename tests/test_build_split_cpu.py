"""The engine library's two translation units (fibsem-optflow_amd/Makefile):
the iteration passes are compiled once, in csrc/tvl1_passes.hip under the ILP scheduler, and
tvl1_engine.hip only references them (its `extern template` declarations).  CPU-only: reads
the built objects' symbol tables."""
import re
import subprocess
from pathlib import Path

import pytest

PKG = Path(__file__).resolve().parent.parent / "fibsem-optflow_amd"
LIB = PKG / "lib"


def _expected():
    ks = set()
    for k in (1, 2, 3, 4):
        ks.add(f"k_iterate_roll<true, {k}, 2, 0>(tvl1k::RollArgs)")
    for k in (1, 2):
        ks.add(f"k_iterate_roll<true, {k}, 4, 0>(tvl1k::RollArgs)")
    for fm in (0, 1, 2):   # kIEEE, kFast, kFma
        for k in (1, 2, 3, 4):
            ks.add(f"k_iterate_roll<false, {k}, 2, {fm}>(tvl1k::RollArgs)")
            ks.add(f"kb_iterate_roll<{k}, 2, {fm}>(tvl1k::BatchRoll)")
            ks.add(f"kb_iterate_roll<{k}, 1, {fm}>(tvl1k::BatchRoll)")
        for k in (1, 2):
            ks.add(f"k_iterate_roll<false, {k}, 4, {fm}>(tvl1k::RollArgs)")
        ks.add(f"k_iterate_tb4<{fm}, 3>(tvl1k::TBArgs)")
        ks.add(f"k_iterate_roll_mid<{fm}>(tvl1k::RollArgs)")
    return ks


def _kernels(obj, kinds):
    out = subprocess.run(["nm", "-C", str(obj)], check=True, capture_output=True, text=True).stdout
    found = {}
    for line in out.splitlines():
        # the kernel handle or its host launch stub (__device_stub__<kernel>)
        m = re.match(r"^\s*[0-9a-f]*\s+([A-Za-z])\s+void tvl1k::(?:__device_stub__)?"
                     r"((?:k|kb)_iterate_(?:roll|roll_mid|tb4)<.*)$", line)
        if m and m.group(1) in kinds:
            found[m.group(2)] = found.get(m.group(2), 0) + 1
    return found


@pytest.mark.skipif(not (LIB / "tvl1_passes.o").exists(), reason="engine not built (make -C fibsem-optflow_amd)")
def test_passes_defined_once_in_their_own_unit():
    exp = _expected()
    inc = (PKG / "csrc" / "tvl1_passes.inc").read_text()
    assert inc.count("TVL1_PASS_INSTANCE(") == 6 + 16   # 6 gamma forms, 16 per arithmetic mode
    defined = _kernels(LIB / "tvl1_passes.o", "VvWw")
    assert exp <= set(defined), sorted(exp - set(defined))
    assert all(n == 2 for k, n in defined.items() if k in exp)   # handle + stub, once each
    # the engine unit references them without instantiating any
    eng_defined = _kernels(LIB / "tvl1_engine.o", "VvWwTt")
    assert not (exp & set(eng_defined)), sorted(exp & set(eng_defined))
    eng_undef = set(_kernels(LIB / "tvl1_engine.o", "U"))
    hot = {"k_iterate_roll<false, 4, 2, 0>(tvl1k::RollArgs)", "k_iterate_roll<false, 2, 4, 0>(tvl1k::RollArgs)",
           "k_iterate_roll<false, 2, 2, 0>(tvl1k::RollArgs)", "k_iterate_tb4<0, 3>(tvl1k::TBArgs)",
           "kb_iterate_roll<4, 2, 0>(tvl1k::BatchRoll)", "k_iterate_roll_mid<0>(tvl1k::RollArgs)"}
    assert hot <= eng_undef, sorted(hot - eng_undef)


def test_passes_unit_is_ilp_scheduled():
    mk = (PKG / "Makefile").read_text()
    assert re.search(r"^PASSFLAGS \?= -mllvm -amdgpu-sched-strategy=max-ilp$", mk, re.M)
    assert "$(PASSFLAGS) -c -o $@ csrc/tvl1_passes.hip" in mk
