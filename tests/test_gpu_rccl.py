"""The RCCL (nccl backend) path of bench.py, executed on the one GPU before the driver's
8-GPU node runs it (VERDICT r2 "next" item 3).  bench.py opens a process group whenever a
launcher set WORLD_SIZE, so `torch.distributed.run --nproc-per-node 1` with the default
backend runs init_process_group("nccl", device_id=...), the start / stop barriers and the
device-tensor all_reduce (max of the elapsed time; sums of the stack's pair and iteration
counts) -- the code the multi-GPU bench depends on, for both the pair and the stack
workloads.  The reference's scale-out it replaces is file sharding
(/root/reference/support_scripts/gen_cross_file_list.py:26-27, singularity/janelia_run.sh:3).
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent


def torchrun(args, timeout=110, gpus_flag=True):
    port = 29500 + os.getpid() % 150
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"),
           *(["--gpus", "1"] if gpus_flag else []), *args]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    env.pop("BENCH_DIST_BACKEND", None)   # the default: nccl (= RCCL)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env,
                       cwd=str(ROOT))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


def test_pair_bench_under_rccl(built):
    out = torchrun(["--width", "640", "--height", "480", "--steps", "2", "--warmup", "1",
                    "--inflight", "2", "--no-cpu-baseline", "--no-strips-line",
                    "--no-fast-math-line"])
    assert out["config"]["process_group"] == "nccl", out["config"]
    assert out["n_gpus"] == 1 and out["steps"] == 2
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert out["config"]["iterations_per_pair"] > 0
    # the per-rank records travel through all_gather_object on the nccl group
    assert [r["rank"] for r in out["ranks"]] == [0] and out["ranks"][0]["pairs"] == 2 * 2
    assert out["ranks"][0]["pci"].count(":") == 2


def test_torchrun_without_gpus_flag(built):
    """`torchrun --nproc-per-node 1 bench.py` with no --gpus takes WORLD_SIZE."""
    out = torchrun(["--width", "320", "--height", "240", "--steps", "1", "--warmup", "1",
                    "--inflight", "1", "--no-cpu-baseline", "--no-strips-line",
                    "--no-fast-math-line"], gpus_flag=False)
    assert out["n_gpus"] == 1 and out["config"]["process_group"] == "nccl"


def test_stack_bench_under_rccl(built):
    out = torchrun(["--workload", "stack", "--slices", "10", "--width", "256", "--height", "192",
                    "--strides", "1,4", "--chunk", "3", "--inflight", "2", "--nscales", "4",
                    "--warps", "5"])
    assert out["config"]["process_group"] == "nccl", out["config"]
    # every (z, z + s) pair once: 9 adjacent + 6 at stride 4, counted by the all_reduce
    assert out["config"]["pairs"] == 9 + 6
    assert out["value"] > 0
    assert len(out["ranks"]) == 1 and out["ranks"][0]["pairs"] == 9 + 6
