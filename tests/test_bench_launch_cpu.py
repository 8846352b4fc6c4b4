"""bench.py's launch contract on CPU (VERDICT r3 "next" item 2): a plain `bench.py --gpus N`
(no launcher, WORLD_SIZE unset) starts N ranks itself -- `torch.distributed.run
--nproc-per-node N` as a child process, before torch (or HIP) is imported, never an exec --
and a launcher whose WORLD_SIZE disagrees with --gpus is an error, so a line can only claim
n_gpus = N when N ranks ran.  The reference scales by one process per shard
(/root/reference/support_scripts/gen_cross_file_list.py:26-27, singularity/janelia_run.sh:3).
The GPU side (2 gloo ranks through the plain launch) is tests/test_gpu_stack.py."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def run(args, **env):
    e = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    e.update(env)
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True,
                          text=True, timeout=60, env=e, cwd=str(ROOT))


def test_plain_multi_gpu_launch_spawns_ranks_before_torch():
    r = run(["--gpus", "8", "--steps", "3", "--warmup", "1"], BENCH_LAUNCH_DRYRUN="1")
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["torch_imported"] is False
    cmd = out["launch"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    # the same arguments reach every rank
    i = cmd.index(str(ROOT / "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "3", "--warmup", "1"]


def test_one_gpu_does_not_spawn():
    # --gpus 1 runs in this process (no launcher needed): without a GPU it fails inside the
    # bench, but never prints a launch line
    r = run(["--gpus", "1", "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
             "--no-strips-line", "--no-fast-math-line", "--width", "64", "--height", "48"],
            BENCH_LAUNCH_DRYRUN="1")
    assert '"launch"' not in r.stdout


def test_launcher_world_size_must_match_gpus():
    r = run(["--gpus", "8"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "WORLD_SIZE 2" in r.stderr
    assert not r.stdout.strip()


def test_launcher_without_gpus_takes_world_size():
    """`torchrun --nproc-per-node 2 bench.py` without --gpus: --gpus defaults to
    the launcher's WORLD_SIZE, so the mismatch check does not fire; the dry-run switch stops
    after the argument handling (the test must not depend on the host's GPUs)."""
    # (tiny geometry, no side lines and the dry-run switch, so that on a host that does have a
    # GPU the run stays an argument check and cannot start the C2 workload: ADVICE r5)
    r = run(["--steps", "1", "--warmup", "0", "--width", "64", "--height", "48",
             "--no-cpu-baseline", "--no-strips-line", "--no-fast-math-line"],
            WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", BENCH_LAUNCH_DRYRUN="1")
    assert "but the launcher started" not in r.stderr
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["gpus"] == 2 and out["world"] == 2 and out["torch_imported"] is False


def test_cpu_allotment_records_the_share(monkeypatch):
    """cpu_baseline's thread count is the smallest of the affinity mask, the cgroup quota and
    OMP_NUM_THREADS, and every one of them is recorded."""
    sys.path.insert(0, str(ROOT))
    import bench
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    a = bench.cpu_allotment()
    assert a["affinity_cpus"] == len(os.sched_getaffinity(0))
    assert a["omp_num_threads_env"] == 3
    assert a["threads"] == min(x for x in (a["affinity_cpus"], a["cgroup_quota_cpus"], 3) if x)
    assert a["cgroup_source"] in (None, "cgroup v2 cpu.max", "cgroup v1 cpu.cfs_quota_us")
    if a["cgroup_quota_exact"] is not None:
        assert a["cgroup_quota_cpus"] == max(1, int(a["cgroup_quota_exact"]))
    monkeypatch.delenv("OMP_NUM_THREADS")
    b = bench.cpu_allotment()
    assert b["omp_num_threads_env"] is None and 1 <= b["threads"] <= b["affinity_cpus"]
