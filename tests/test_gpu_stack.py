"""C4 / C5 at reduced scale under -m gpu (VERDICT r1 "next" item 1): the
stack workload of bench.py -- slices generated on the device (DeviceStack), contiguous
chunks of pairs pulled from one WorkQueue shared by every rank, strides {1, 4, 16} as
gen_cross_file_list.py enumerates long-range pairs (/root/reference/support_scripts/
gen_cross_file_list.py:26-27,102-142) -- launched as the driver launches a multi-GPU bench
(torch.distributed.run, one process per rank) with 2 gloo ranks sharing the one GPU.

Checks: every (z, z + s) pair is solved exactly once across ranks; each pair's flow is
bit-identical to tvl1_calc of that pair alone and to the oracle, with the oracle's per-warp
iteration counts."""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from optflow_amd import capi
from oracle import checker

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

ROOT = Path(__file__).resolve().parent.parent
Z, W, H, STRIDES = 24, 256, 192, (1, 4, 16)
KW = dict(nscales=5, warps=10)


def bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32),
                          np.ascontiguousarray(b).view(np.uint32))


@pytest.fixture(scope="module")
def stack_run(tmp_path_factory, built):
    d = tmp_path_factory.mktemp("stack")
    port = 29700 + os.getpid() % 200
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"),
           "--gpus", "2", "--workload", "stack", "--slices", str(Z), "--width", str(W),
           "--height", str(H), "--strides", ",".join(map(str, STRIDES)), "--chunk", "3",
           "--inflight", "2", "--nscales", str(KW["nscales"]), "--warps", str(KW["warps"]),
           "--dump", str(d)]
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    return d, json.loads(line)


def test_plain_launch_runs_n_ranks(built, tmp_path):
    """`bench.py --gpus 2` started plainly, as the driver's bench command is written (no
    torch.distributed.run in front): bench.py starts the 2 ranks itself,
    so the line says n_gpus 2 and every pair is solved exactly once across both ranks."""
    z, strides = 10, (1, 4)
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--workload", "stack",
           "--slices", str(z), "--width", "128", "--height", "96",
           "--strides", ",".join(map(str, strides)), "--chunk", "2", "--inflight", "2",
           "--nscales", "3", "--warps", "3", "--dump", str(tmp_path)]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(BENCH_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["config"]["process_group"] == "gloo"
    want = {(s, k) for s in strides for k in range(z - s)}
    assert out["config"]["pairs"] == len(want)
    got = [tuple(int(t[1:]) for t in f.name.split("_")[1:3])
           for f in tmp_path.glob("pair_s*_z*_r*.npz")]
    assert sorted(got) == sorted(want)
    assert {int(np.load(f)["rank"]) for f in tmp_path.glob("*.npz")} <= {0, 1}
    # one record per rank; under gloo both ranks share the one card
    rk = out["ranks"]
    assert [r["rank"] for r in rk] == [0, 1]
    assert len({r["pci"] for r in rk}) == 1
    assert sum(r["pairs"] for r in rk) == len(want)
    assert all(r["elapsed_s"] > 0 for r in rk)


def test_plain_launch_default_pair_line(built):
    """The driver's multi-GPU command as written (`bench.py --gpus N --steps K --warmup W`, no
    launcher, the default pair workload with its extra lines): 2 ranks (gloo, on the one GPU),
    every collective of the math-mode and production-strip legs reached by both ranks, one
    JSON line from rank 0 claiming both GPUs, no CPU baseline above one GPU."""
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--width", "320", "--height", "240", "--inflight", "2"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(BENCH_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=200, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["process_group"] == "gloo"
    assert out["value"] > 0 and out["cpu_baseline"] is None
    assert set(out["math_modes"]) == {"fast", "fma"}
    assert out["production_strips"]["value"] > 0
    for rk in (out["ranks"], out["production_strips"]["ranks"]):
        assert [r["rank"] for r in rk] == [0, 1] and len({r["pci"] for r in rk}) == 1
    assert [r["pairs"] for r in out["ranks"]] == [2 * 2, 2 * 2]   # steps x in flight


def expected_pairs():
    return {(s, z) for s in STRIDES for z in range(Z - s)}


def test_every_pair_exactly_once_across_ranks(stack_run):
    d, out = stack_run
    got = []
    for f in d.glob("pair_s*_z*_r*.npz"):
        s, z = f.name.split("_")[1:3]
        got.append((int(s[1:]), int(z[1:])))
    assert len(got) == len(set(got)), "a pair was solved twice"
    assert set(got) == expected_pairs()
    assert out["config"]["pairs"] == len(expected_pairs()) == 51
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"


def test_stack_flows_bit_identical_to_single_solves_and_oracle(stack_run):
    from optflow_amd.synth_device import DeviceStack
    d, _ = stack_run
    gen = DeviceStack(W, H, torch.device("cuda", 0))
    sl = {z: gen.slice(z).cpu().numpy() for z in range(Z)}
    p = capi.make_params(**KW)
    eng = capi.Engine(p)
    ranks = set()
    for f in sorted(d.glob("pair_s*_z*_r*.npz")):
        s, z = (int(t[1:]) for t in f.name.split("_")[1:3])
        rec = np.load(f)
        ranks.add(int(rec["rank"]))
        us, vs, ss, ws = eng.calc_host(sl[z], sl[z + s])
        assert bits_equal(rec["u"], us) and bits_equal(rec["v"], vs), f"(s={s}, z={z})"
        np.testing.assert_array_equal(rec["warp_iters"], ws, err_msg=f"(s={s}, z={z})")
        if s == 16 or z % 5 == 0:   # the oracle on a third of the pairs (every stride)
            ur, vr, sr, wr = checker.oracle_calc(sl[z], sl[z + s], p)
            np.testing.assert_array_equal(ws, wr, err_msg=f"oracle (s={s}, z={z})")
            assert bits_equal(us, ur) and bits_equal(vs, vr), f"oracle (s={s}, z={z})"
    eng.close()
    assert ranks <= {0, 1}
