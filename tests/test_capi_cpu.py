"""The C-ABI library loads and exports every symbol include/tvl1.h declares
(no compute calls here: no GPU in the CPU suite)."""
import ctypes as C
import re
from pathlib import Path

import pytest

from optflow_amd import capi

HEADER = Path(__file__).resolve().parents[1] / "include" / "tvl1.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(tvl1_[a-z_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("tvl1_create", "tvl1_calc", "tvl1_calc_host", "tvl1_calc_batch", "tvl1_destroy",
                 "tvl1_last_error", "tvl1_postprocess", "tvl1_params_default"):
        assert must in names


def test_library_exports_every_declared_symbol(built):
    lib = C.CDLL(str(capi.ENGINE_SO))
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_abi_version_and_defaults(built):
    lib = capi.load_engine()
    assert lib.tvl1_abi_version() == 9
    p = capi.TVL1Params()
    lib.tvl1_params_default(C.byref(p))
    # generate_TV_args defaults, /root/reference/src/optflow.cpp:503-512
    assert (p.tau, p.lambda_, p.theta, p.nscales, p.warps, p.epsilon, p.iterations,
            p.scale_step, p.gamma) == (0.25, 0.05, 0.3, 10, 5, 0.01, 300, 0.8, 0.0)
    assert p.use_initial_flow == 0 and p.median_filtering == 1 and p.fast_math == 0


def test_struct_layout_matches_header(built, tmp_path):
    """ctypes mirror == C layout: compile a probe against include/tvl1.h."""
    import shutil
    import subprocess
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    src = tmp_path / "probe.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "tvl1.h"\n'
        "int main(void){printf(\"%zu %zu %zu %zu %zu %zu %zu\\n\","
        "sizeof(tvl1_params), sizeof(tvl1_stats), offsetof(tvl1_params, epsilon),"
        "offsetof(tvl1_params, outer_iterations), offsetof(tvl1_stats, warp_iterations),"
        "offsetof(tvl1_stats, kernel_ms), offsetof(tvl1_stats, kernel_hbm_bytes));return 0;}\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", str(HEADER.parent), str(src), "-o", str(exe)], check=True)
    got = [int(t) for t in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    P, S = capi.TVL1Params, capi.TVL1Stats
    assert got == [C.sizeof(P), C.sizeof(S), P.epsilon.offset, P.outer_iterations.offset,
                   S.warp_iterations.offset, S.kernel_ms.offset, S.kernel_hbm_bytes.offset]


def test_create_rejects_bad_params_and_missing_gpu(built):
    lib = capi.load_engine()
    ctx = C.c_void_p()
    bad = capi.make_params(nscales=0)
    assert lib.tvl1_create(C.byref(ctx), 0, C.byref(bad)) == 1        # TVL1_EINVAL
    assert b"nscales" in lib.tvl1_last_error(None)
    bad = capi.make_params(fast_math=3)   # 0 IEEE, 1 fast, 2 fma
    assert lib.tvl1_create(C.byref(ctx), 0, C.byref(bad)) == 1        # TVL1_EINVAL
    assert b"fastMath" in lib.tvl1_last_error(None)
    bad = capi.make_params(profile=2)
    assert lib.tvl1_create(C.byref(ctx), 0, C.byref(bad)) == 1        # TVL1_EINVAL
    assert b"profile" in lib.tvl1_last_error(None)
    if lib.tvl1_device_count() == 0:
        good = capi.make_params()
        assert lib.tvl1_create(C.byref(ctx), 0, C.byref(good)) == 5   # TVL1_ENODEV
        assert not ctx.value


def test_engine_has_no_cpu_fallback(built, monkeypatch):
    """The product path fails loudly when the HIP library is missing."""
    monkeypatch.setattr(capi, "ENGINE_SO", Path("/nonexistent/libtvl1_hip.so"))
    with pytest.raises(FileNotFoundError):
        capi.Engine(capi.make_params())
