#!/usr/bin/env python3
"""bench.py — slice-pairs/s of the MI355X TV-L1 engine on BASELINE.json's workload.

Workload (BASELINE.json configs[1], SURVEY 8(d) "C2"): one synthetic 6144x4096 u8
slice pair, nscales 5, warps 30, iterations 300, epsilon 0.01 (other TV-L1
parameters at the reference defaults, optflow.cpp:503-512).  A "step" is one full
solve of that pair through the C-ABI (tvl1_calc on device buffers): pyramid,
30 warps per level, the data-dependent primal-dual iterations and the final flow.
Inputs are resident in HBM before the timed region starts.

Multi-GPU: slice pairs are independent, so each rank (one process
per GPU) solves its own pair every step: weak scaling, no data-path collective.
torch.distributed (nccl = RCCL) is used only for the start/stop barrier and the
max-over-ranks reduction of the elapsed time.

Prints ONE JSON line on rank 0 (contract in the task statement), with
  roofline: dominant kernel class = the iteration passes (k_iterate_roll, k_iterate_tb
            and k_warp_iter, warpBackward fused into each warp's first pass).
            achieved = the bytes those launches move (the engine's live per-launch
            accounting of its tiling, checked against rocprofv3 PMC bytes: `traffic`)
            / their average HIP-event launch duration on ONE pair alone, measured after
            the timed steps (no events inside them); peak = 8000 GB/s (MI355X HBM3E).
  cpu_baseline: the oracle (CPU restatement, oracle/) timed on this host on the
            benchmark pair itself (one full C2 solve, 10-20 s on the box's cores),
            compiled for this host's CPU at bench time when a compiler is present.
  production_strips: the production ROI-strip workload through
            tvl1_calc_batch, with its own roofline for the batched iteration class.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "fibsem-optflow_amd"))

HBM_PEAK_GBS = 8000.0


def _traffic(name="traffic.json"):
    """PMC-measured HBM bytes per iteration-pass launch (rocprofv3 FETCH_SIZE x 2 per the
    gfx950 correction + WRITE_SIZE, separate passes, one pair alone: tools/pmc_single.sh +
    tools/pmc_summary.py --emit-traffic) and the class's VALU utilisation, committed under
    profiles/ for the engine build the bench runs.  None if not measured."""
    p = ROOT / "profiles" / name
    try:
        return json.loads(p.read_text())
    except Exception:
        return None


TRAFFIC = _traffic()
TRAFFIC_STRIPS = _traffic("traffic_strips.json")
# The VALU issue model of the C2 iteration class (tools/issue_model.py --model): the cycles
# the class keeps its SIMDs busy issuing VALU per launch, every instruction priced at its
# measured gfx950 throughput cost (tools/issue_rate.hip), from the ISA mix and the PMC counts
# of one pair alone (profiles/r6/issue/).
ISSUE_MODEL = _traffic("r6/issue/model.json")
RED_CPU = False   # reductions on CPU tensors (gloo rehearsal, BENCH_DIST_BACKEND=gloo)
DIST_BACKEND = None   # the torch.distributed backend in use (None: no process group)
MATH = {0: "IEEE (bit-identical to oracle/)", 1: "fast (CUDA_FAST_MATH semantics)",
        2: "fma (nvcc -fmad=true contraction, IEEE division; bit-identical to oracle/'s fma mode)"}
METRIC = "slice-pairs/sec (6k×4k, 5 scales, 30 warps) at 1/2/4/8 GPUs; % HBM roofline"


PAIR_KERNEL = ("iteration passes: estimateU + estimateDualVariables + residual partials, <= 4 "
               "iterations per HBM pass (k_iterate_roll wavefront pipeline; long passes on levels "
               "too small to fill the GPU with streaming segments in k_iterate_tb4's 64x48 "
               "blocked regions; on levels >= 4 Mpx each warp's first pass is k_warp_iter, "
               "warpBackward fused in)")
STRIP_KERNEL = ("batched iteration passes of one tvl1_calc_batch call: kb_iterate_roll<K, 2> "
                "(<= 4 iterations per HBM pass, a pair index per launch) and kb_warp_iter "
                "(warpBackward fused with each warp's first pass)")


def roofline(k_bytes, k_hbm, k_ms, k_launch, traffic, kernel, issue=None, cls="iteration_class"):
    """The dominant kernel class against its two ceilings.

    hbm: achieved = the bytes these launches must move (the engine's per-launch accounting of
    its tiling: band loads with halos + interior stores, checked against the rocprofv3
    FETCH_SIZE / WRITE_SIZE passes in profiles/, see `traffic`) / their average HIP-event
    launch time.  SURVEY 8(d)'s one-pass-per-iteration model (64 B/px per iteration) does not
    describe a temporally blocked kernel (it would exceed the peak), so it is reported beside
    the fraction as `model_bytes_over_peak`, never as `frac`.

    valu (issue = the committed issue model, C2 class only): achieved = the SIMD cycles the
    class's VALU instructions occupy per launch (each priced at its measured throughput cost)
    x 1024 SIMDs / the live average launch time; peak = 1024 SIMDs x the clock the PMC run
    held.  `bound` names the larger fraction: the ceiling the kernels sit closer to (with every
    HBM access dropped, k_warp_iter takes the same time: DESIGN 10.1)."""
    achieved = k_hbm / (k_ms * 1e-3) / 1e9
    model = k_bytes / (k_ms * 1e-3) / 1e9
    hbm = {"achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4),
           "bytes_per_launch": round(k_hbm / k_launch),
           "bytes_basis": "engine accounting of the tiling's compulsory HBM bytes (live)",
           "model_bytes_per_launch": round(k_bytes / k_launch),
           "model": "SURVEY 8(d): 64 B/px per executed iteration (+ 40 B/px for a fused "
                    "warpBackward)",
           "model_bytes_over_peak": round(model / HBM_PEAK_GBS, 4)}
    r = {"bound": "hbm", "achieved": hbm["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": hbm["frac"],
         "traffic": traffic.get("iterate_hbm_bytes_per_launch") if traffic else None,
         "kernel": kernel,
         "launches": k_launch, "avg_launch_us": round(1e3 * k_ms / k_launch, 2),
         "hbm": hbm}
    if traffic:
        r["traffic_source"] = traffic.get("source")
        r["traffic_over_bytes"] = round(traffic["iterate_hbm_bytes_per_launch"] /
                                        (k_hbm / k_launch), 4)
        if traffic.get("iterate_valu_frac") is not None:
            # SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8), same class,
            # same workload alone (tools/pmc_single.sh + tools/valu_util.py)
            hbm["valu_frac_at_2_cycles"] = traffic["iterate_valu_frac"]
    if issue and cls in issue:
        ic = issue[cls]
        live_us = 1e3 * k_ms / k_launch
        clk = ic["class_clock_ghz"]
        v_ach = ic["class_busy_cycles_per_launch"] * 1024 / (live_us * 1e-6) / 1e9
        v_peak = 1024 * clk
        valu = {"achieved": round(v_ach, 1), "peak": round(v_peak, 1),
                "unit": "G SIMD-issue-cycles/s", "frac": round(v_ach / v_peak, 4),
                "busy_cycles_per_launch": ic["class_busy_cycles_per_launch"],
                "pmc_frac": ic["class_simd_valu_busy_frac"],
                "pmc_avg_launch_us": ic["class_avg_launch_us"],
                "frac_at_2_cycles_per_valu": ic["class_valu_frac_at_2_cycles"],
                "dominant_kernel": {k: v["simd_valu_busy_frac"] for k, v in ic["kernels"].items()},
                "model": "tools/issue_model.py: ISA mix x measured throughput cost per "
                         "instruction class x PMC VALU count, over GRBM_GUI_ACTIVE / 8",
                "source": f"profiles/r6/issue/model.json ({cls})"}
        r["valu"] = valu
        if valu["frac"] > hbm["frac"]:
            r.update({"bound": "valu", "achieved": valu["achieved"], "peak": valu["peak"],
                      "unit": valu["unit"], "frac": valu["frac"]})
    return r


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: WORLD_SIZE under a launcher, else 1")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    # defaults None: C2's 6144x4096 / 5 scales / 30 warps, or for --workload strips the
    # production strip's 3072x100 / 10 scales / 5 warps
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--nscales", type=int, default=None)
    ap.add_argument("--warps", type=int, default=None)
    ap.add_argument("--iterations", type=int, default=300)
    ap.add_argument("--epsilon", type=float, default=0.01)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fast-math", type=int, default=0, choices=(0, 1, 2), nargs="?", const=1,
                    help="headline arithmetic mode (tvl1_params.fast_math): 0 = IEEE, bit-identical "
                         "to oracle/ (default); 1 = the reference build's CUDA_FAST_MATH semantics "
                         "(tolerance parity); 2 = nvcc's -fmad=true contraction alone (bit-identical "
                         "to oracle/'s fma mode).  The other modes are measured after the headline "
                         "and reported under \"math_modes\" with their EPE against it")
    ap.add_argument("--profile", type=int, default=0, choices=(0, 1),
                    help="1 = OpenCV's CPU DualTVL1OpticalFlow schedule (SURVEY 8(f) N3; "
                         "BASELINE configs[0]), with --inner / --outer iterations")
    ap.add_argument("--inner", type=int, default=30)
    ap.add_argument("--outer", type=int, default=10)
    ap.add_argument("--lambda", dest="lam", type=float, default=0.05)
    ap.add_argument("--median", type=int, default=1)
    ap.add_argument("--no-strips-line", action="store_true",
                    help="skip the production ROI-strip measurement reported beside C2")
    ap.add_argument("--no-fast-math-line", action="store_true",
                    help="skip the other arithmetic modes' measurement (math_modes)")
    ap.add_argument("--cpu-sample", default="6144x4096",
                    help="WxH crop of the benchmark pair the CPU baseline solves (default: all of it)")
    ap.add_argument("--inflight", type=int, default=None,
                    help="slice pairs solved concurrently per GPU (one ctx + stream + host "
                         "thread each); a step = one batch of this many pairs")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="skip per-kernel HIP events (roofline fields become null)")
    ap.add_argument("--batch", type=int, default=256,
                    help="strips: pairs per tvl1_calc_batch call")
    ap.add_argument("--workload", choices=("pair", "stack", "strips"), default="pair",
                    help="pair: BASELINE configs[1] (C2, the headline); stack: adjacent / "
                         "strided pairs of a synthetic stack (C3: --slices 256; C4: --slices "
                         "4096 on 8 GPUs; C5: --strides 1,4,16), slices made on the device")
    ap.add_argument("--slices", type=int, default=256)
    ap.add_argument("--strides", default="1")
    ap.add_argument("--chunk", type=int, default=8,
                    help="stack: contiguous pairs per work item (slice reuse within it)")
    ap.add_argument("--dump", default=None,
                    help="stack: write every pair's flow, per-warp iterations and solving "
                         "rank to DIR/pair_s<s>_z<z>.npz (tests/test_gpu_stack.py; not timed "
                         "for the bench line)")
    args = ap.parse_args()
    # `torchrun --nproc-per-node N bench.py` without --gpus: the launcher's WORLD_SIZE (an
    # explicit --gpus that disagrees with it stays an error in main())
    args.gpus_explicit = args.gpus is not None
    if args.gpus is None:
        args.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    geo = (3072, 100, 10, 5) if args.workload == "strips" else (6144, 4096, 5, 30)
    for k, d in zip(("width", "height", "nscales", "warps"), geo):
        if getattr(args, k) is None:
            setattr(args, k, d)
    if args.inflight is None:   # pairs (or strip batches) in flight per GPU
        # pairs: 3 (+1.5 % over 2 on the C2 pair, 4 is slower); strip batches: 2
        args.inflight = 2 if args.workload == "strips" else 3
    return args


def cpu_allotment():
    """The host CPUs this process may use, and the oracle thread count taken from them
    (the CPU baseline runs on all the host cores it is given).  A gpurun box
    shows the whole machine to os.cpu_count() but allots a share through the cgroup CPU
    quota and OMP_NUM_THREADS; every figure is recorded so the line explains its `cores`."""
    aff = len(os.sched_getaffinity(0))
    quota, quota_exact, source = None, None, None
    try:   # cgroup v2: "<quota> <period>" or "max <period>"
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        source = "cgroup v2 cpu.max"
        if q != "max":
            quota_exact = int(q) / int(per)
    except (OSError, ValueError):
        try:   # cgroup v1: cpu.cfs_quota_us (-1: none) over cpu.cfs_period_us
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            source = "cgroup v1 cpu.cfs_quota_us"
            if q > 0 and per > 0:
                quota_exact = q / per
        except (OSError, ValueError):
            pass
    if quota_exact is not None:
        quota = max(1, int(quota_exact))   # whole threads; the fraction is recorded beside it
    env = os.environ.get("OMP_NUM_THREADS")
    omp = int(env) if env and env.isdigit() and int(env) > 0 else None
    threads = min(x for x in (aff, quota, omp) if x is not None)
    return {"affinity_cpus": aff, "cgroup_quota_cpus": quota,
            "cgroup_quota_exact": None if quota_exact is None else round(quota_exact, 3),
            "cgroup_source": source, "omp_num_threads_env": omp,
            "machine_cpus": os.cpu_count(), "threads": threads}


def rank_records(dist, local_rank, pairs, iterations, elapsed):
    """One record per rank, gathered after the timed region: the device
    each rank solved on (PCI domain:bus:device, which must be N distinct GPUs on an N-GPU
    line under nccl; ranks share the one card under the gloo rehearsal), the pairs it solved
    and its own elapsed time, so the line shows placement and balance, not only the
    max-over-ranks time."""
    import torch
    pr = torch.cuda.get_device_properties(local_rank)
    rec = {"rank": int(os.environ.get("RANK", "0")), "local_rank": local_rank,
           "pci": f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}",
           "device": pr.name or pr.gcnArchName, "pairs": pairs, "iterations": iterations,
           "elapsed_s": round(elapsed, 4)}
    if not dist:
        return [rec]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, rec)
    return out


_NATIVE_ORACLE = None


def native_oracle():
    """SURVEY 8(d)'s CPU-baseline recipe: the oracle compiled on the bench host for its own
    CPU (-O3 -march=native -fopenmp; -ffp-contract=off keeps the float32 operation order,
    so the bits do not change) into a temp dir.  Falls back to the portable in-tree build
    (no -march=native: it travels between hosts) when no compiler is present.  Returns
    (path or None, description of the build)."""
    global _NATIVE_ORACLE
    if _NATIVE_ORACLE is not None:
        return _NATIVE_ORACLE
    import platform
    import subprocess
    import tempfile
    cpu = platform.processor() or "unknown CPU"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                cpu = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    flags = ["-O3", "-march=native", "-std=c11", "-fPIC", "-fopenmp", "-ffp-contract=off",
             "-fno-fast-math"]
    d = Path(tempfile.mkdtemp(prefix="orc_native_"))
    so = d / "liboracle_tvl1_native.so"
    src = ROOT / "oracle"
    try:
        subprocess.run(["gcc", *flags, "-shared", "-o", str(so), str(src / "tvl1_oracle.c"),
                        str(src / "tvl1_oracle_dualtvl1.c"), str(src / "tvl1_oracle_align.c"),
                        "-lm"], check=True,
                       capture_output=True, timeout=120)
        _NATIVE_ORACLE = (str(so), f"gcc {' '.join(flags)} on the bench host ({cpu}, "
                                   f"{os.cpu_count()} logical CPUs)")
    except Exception as e:   # no compiler: the portable build
        _NATIVE_ORACLE = (None, f"portable in-tree build (oracle/Makefile, no -march=native; "
                                f"host build failed: {type(e).__name__}) on {cpu}, "
                                f"{os.cpu_count()} logical CPUs")
    return _NATIVE_ORACLE


def cpu_baseline(I0, I1, params, sample: str):
    """Oracle (CPU restatement of OpenCV 3.4.1 CUDA TV-L1) on the benchmark pair itself (or
    a crop of it, extrapolated by pixel count, with --cpu-sample)."""
    import numpy as np
    from oracle import checker   # cpu_baseline leg: the oracle is timed, never the product
    sw, sh = (int(t) for t in sample.lower().split("x"))
    H, W = I0.shape
    sw, sh = min(sw, W), min(sh, H)
    a = np.ascontiguousarray(I0[:sh, :sw])
    b = np.ascontiguousarray(I1[:sh, :sw])
    so, build = native_oracle()
    lib = checker.load_oracle(so)
    allot = cpu_allotment()
    lib.orc_set_num_threads(allot["threads"])
    threads = int(lib.orc_num_threads())
    t0 = time.perf_counter()
    _, _, st, _ = checker.oracle_calc(a, b, params, warp_iters=False, so=so)
    dt = time.perf_counter() - t0
    scale = (W * H) / float(sw * sh)
    return {
        "value": 1.0 / (dt * scale),
        "unit": "slice-pairs/s",
        "cores": threads,
        "allotment": allot,
        "kind": "port",
        "build": build,
        "sample": ((f"oracle/ CPU restatement, {threads} OpenMP threads, one {sw}x{sh} crop of "
                    f"the benchmark pair, same TV-L1 parameters ({st['iterations_total']} "
                    f"iterations over {st['levels']} levels) in {dt:.2f} s, extrapolated "
                    f"x{scale:.2f} by pixel count to one {W}x{H} pair") if scale != 1.0 else
                   (f"oracle/ CPU restatement, {threads} OpenMP threads, the whole benchmark "
                    f"pair ({W}x{H}, {st['iterations_total']} iterations over {st['levels']} "
                    f"levels, the same as the GPU's) in {dt:.2f} s")),
    }


def run_stack(args, rank, world, local_rank, dist):
    """C3/C4/C5: every pair (z, z + s) of a synthetic Z-slice stack for each stride s,
    in contiguous chunks of --chunk pairs pulled from one work queue shared by all
    ranks; each rank keeps --inflight chunks in flight (one engine ctx + stream + host
    thread each).  Slices are generated on the device per chunk and reused by the
    chunk's pairs (slice z is I1 of (z - s, z) and I0 of (z, z + s))."""
    import threading
    import torch
    from optflow_amd import capi
    from optflow_amd.stack import WorkQueue
    from optflow_amd.synth_device import DeviceStack

    W, H, Z = args.width, args.height, args.slices
    strides = [int(t) for t in args.strides.split(",")]
    params = capi.make_params(nscales=args.nscales, warps=args.warps,
                              iterations=args.iterations, epsilon=args.epsilon,
                              fast_math=int(args.fast_math))
    dev = torch.device("cuda", local_rank)
    gen = DeviceStack(W, H, dev)
    items = []
    for s_ in strides:
        for z0 in range(0, Z - s_, args.chunk):
            items.append((s_, z0, min(z0 + args.chunk, Z - s_)))
    npairs = sum(z1 - z0 for _, z0, z1 in items)
    F = max(1, args.inflight)
    engines = [capi.Engine(params, device=local_rank) for _ in range(F)]
    u = [torch.empty((H, W), dtype=torch.float32, device=dev) for _ in range(F)]
    v = [torch.empty((H, W), dtype=torch.float32, device=dev) for _ in range(F)]
    # warm-up: one pair per slot (kernels loaded, arenas sized)
    a0, a1 = gen.slice(0), gen.slice(1)
    torch.cuda.synchronize(dev)
    for j in range(F):
        engines[j].calc_device(a0.data_ptr(), W, a1.data_ptr(), W, W, H, u[j].data_ptr(),
                               v[j].data_ptr(), 4 * W, stream=engines[j].stream)
    torch.cuda.synchronize(dev)
    del a0, a1
    store = None
    if dist:
        store = dist.distributed_c10d._get_default_store()
        if rank == 0:
            store.set("stack_q", "0")
        dist.barrier()
    q = WorkQueue(len(items), store)
    done = [0] * F
    iters = [0] * F
    errors = []

    def worker(j):
        eng, st = engines[j], engines[j].stream
        torch_stream = torch.cuda.ExternalStream(st, device=dev)
        try:
            while True:
                i = q.pop()
                if i is None:
                    return
                s_, z0, z1 = items[i]
                with torch.cuda.stream(torch_stream):
                    sl = {z: gen.slice(z) for z in range(z0, z1 + s_)}
                for z in range(z0, z1):
                    r = eng.calc_device(sl[z].data_ptr(), W, sl[z + s_].data_ptr(), W, W, H,
                                        u[j].data_ptr(), v[j].data_ptr(), 4 * W, stream=st,
                                        warp_iters=bool(args.dump))
                    iters[j] += r["iterations_total"]
                    done[j] += 1
                    if args.dump:   # correctness runs only (tests/test_gpu_stack.py)
                        import numpy as np
                        torch_stream.synchronize()
                        np.savez(Path(args.dump) / f"pair_s{s_}_z{z}_r{rank}_{j}.npz",
                                 u=u[j].cpu().numpy(), v=v[j].cpu().numpy(),
                                 warp_iters=r["warp_iters"], rank=rank, slot=j, item=i)
                torch_stream.synchronize()
                del sl
        except Exception as e:   # surfaced below, after the other workers finish
            errors.append(repr(e))

    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    threads = [threading.Thread(target=worker, args=(j,)) for j in range(F)]
    for t in threads:
        t.start()
    # a progress line on stderr every 30 s (a full C4/C5 stack runs for minutes)
    while True:
        alive = [t for t in threads if t.is_alive()]
        if not alive:
            break
        alive[0].join(timeout=30.0)
        if alive[0].is_alive():
            print(f"[rank {rank}] {sum(done)} pairs in {time.perf_counter() - t0:.0f} s",
                  file=sys.stderr, flush=True)
    for t in threads:
        t.join()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if errors:
        raise RuntimeError("; ".join(errors))
    ranks = rank_records(dist, local_rank, sum(done), sum(iters), elapsed)
    mine = torch.tensor([float(sum(done)), float(sum(iters)), elapsed], dtype=torch.float64,
                        device="cpu" if RED_CPU else dev)
    if dist:
        tot = mine[:2].clone()
        dist.all_reduce(tot)
        t = mine[2:].clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        pairs_done, iters_done, elapsed = float(tot[0]), float(tot[1]), float(t[0])
    else:
        pairs_done, iters_done = float(mine[0]), float(mine[1])
    if dist:
        dist.destroy_process_group()
    if rank != 0:
        return
    assert int(pairs_done) == npairs, (pairs_done, npairs)
    name = {1: "C3" if Z <= 512 else "C4"}.get(len(strides) == 1 and strides[0], "C5")
    out = {
        "metric": METRIC,
        "value": round(pairs_done / elapsed, 4),
        "unit": "slice-pairs/s",
        "n_gpus": world,
        "steps": 1,
        "warmup": 1,
        "ms_per_step": round(1e3 * elapsed, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "math": MATH[args.fast_math],
        "data": "synthetic (slices generated on the device)",
        "config": {
            "workload": (f"{name}: {npairs} pairs (z, z+s), s in {strides}, of a {Z}-slice "
                         f"{W}x{H} stack, nscales {args.nscales}, warps {args.warps}, "
                         f"iterations {args.iterations}, epsilon {args.epsilon}"),
            "parallelism": (f"{world} rank(s), {F} chunk(s) in flight per GPU, chunks of "
                            f"{args.chunk} pairs from one shared work queue"),
            "step": "the whole stack",
            "process_group": DIST_BACKEND,
            "pairs": int(pairs_done),
            "iterations_per_pair": round(iters_done / max(1.0, pairs_done), 1),
        },
        "ranks": ranks,
    }
    print(json.dumps(out), flush=True)


def run_strips(args, rank, world, local_rank, dist, standalone=True):
    """The production workload: per slice pair, two ROI strips of the
    half-scale slice (gen_cross_file_list.py top/bottom 100 rows at scale 0.5 -> 3072x100),
    nscales 10 (-> 9 levels), warps 5, the reference's other defaults.  A step = --inflight
    batches of --batch strip pairs, each batch one tvl1_calc_batch call on its own ctx +
    stream + host thread.  value = strip solves/s; slice pairs/s = value / 2."""
    import numpy as np
    import torch
    from concurrent.futures import ThreadPoolExecutor
    from optflow_amd import capi, synth

    W, H, B, F = args.width, args.height, args.batch, max(1, args.inflight)
    params = capi.make_params(nscales=args.nscales, warps=args.warps,
                              iterations=args.iterations, epsilon=args.epsilon,
                              fast_math=int(args.fast_math))
    from optflow_amd.synth_device import DeviceStack
    dev = torch.device("cuda", local_rank)
    slots = []
    for j in range(F):
        # slices 0..B of a synthetic stack, made on the device (synth_device, the SURVEY 8(d)
        # recipe); pair b = (slice 0, slice b + 1), as the C2 pair is (base, slice z): I0
        # pair stride 0, I1 strided through the stack
        gen = DeviceStack(W, H, dev, seed=0x5EED + 977 * (rank * F + j))
        stack = torch.stack([gen.slice(z) for z in range(B + 1)])
        eng = capi.Engine(params, device=local_rank)
        slots.append(dict(eng=eng, stack=stack,
                          ts=torch.cuda.ExternalStream(eng.stream, device=dev),
                          u=torch.empty((B, H, W), dtype=torch.float32, device=dev),
                          v=torch.empty((B, H, W), dtype=torch.float32, device=dev)))
    torch.cuda.synchronize(dev)

    def solve(sl):
        base = sl["stack"].data_ptr()
        st = sl["eng"].calc_batch_device(B, base, W, 0, base + W * H, W, W * H, W, H,
                                         sl["u"].data_ptr(), sl["v"].data_ptr(),
                                         4 * W, 4 * W * H, stream=sl["eng"].stream)
        sl["ts"].synchronize()   # this slot's stream only: the other slots keep running
        return st

    pool = ThreadPoolExecutor(max_workers=F)

    def step():
        return list(pool.map(solve, slots))

    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    iters = 0
    for _ in range(args.steps):
        for st in step():
            iters += sum(s["iterations_total"] for s in st)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ranks = rank_records(dist, local_rank, args.steps * F * B, iters, elapsed)
    # one batch alone on the GPU after the timed steps, with HIP events around every launch
    # (tvl1_set_profiling): the batched iteration class's roofline
    roof = None
    if not args.no_kernel_timing:
        slots[0]["eng"].set_profiling(True)
        s0 = solve(slots[0])[0]
        slots[0]["eng"].set_profiling(False)
        if s0["kernel_ms"][0] > 0:
            prod = (W, H, args.nscales, args.warps, B, args.fast_math) == (3072, 100, 10, 5, 256, 0)
            roof = roofline(s0["kernel_bytes"][0], s0["kernel_hbm_bytes"][0], s0["kernel_ms"][0],
                            s0["kernel_launches"][0], TRAFFIC_STRIPS, STRIP_KERNEL,
                            ISSUE_MODEL if prod else None, "strips_class")
            roof["timing"] = f"one batch of {B} strip pairs alone on the GPU, after the timed steps"
            if s0["kernel_launches"][3] > 0:   # kb_small_level: on chip, outside the HBM class
                roof["coarsest_level_on_chip"] = {"launches": s0["kernel_launches"][3],
                                                  "ms": round(s0["kernel_ms"][3], 3)}
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if RED_CPU else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        if standalone:
            dist.destroy_process_group()
    for sl in slots:
        sl["eng"].close()
    pool.shutdown()
    if rank != 0:
        return None
    solves = world * args.steps * F * B
    value = solves / elapsed
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        from oracle import checker   # cpu_baseline leg only
        st0 = slots[0]["stack"]
        a, c = st0[0].cpu().numpy(), st0[1].cpu().numpy()
        so, build = native_oracle()
        lib = checker.load_oracle(so)
        allot = cpu_allotment()
        lib.orc_set_num_threads(allot["threads"])
        t1 = time.perf_counter()
        n_rep = 4
        for _ in range(n_rep):
            checker.oracle_calc(a, c, params, warp_iters=False, so=so)
        dt = (time.perf_counter() - t1) / n_rep
        cpu = {"value": round(1.0 / dt, 3), "unit": "strip solves/s",
               "cores": int(lib.orc_num_threads()), "allotment": allot, "kind": "port",
               "build": build,
               "sample": f"oracle/ CPU restatement, {n_rep} solves of one {W}x{H} strip pair"}
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "strip solves/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "math": MATH[args.fast_math],
        "data": "synthetic (slice 0 vs slices 1..B of a device-generated stack)",
        "config": {"workload": (f"production ROI strips (SURVEY 3.2): {W}x{H} pairs, nscales "
                                f"{args.nscales}, warps {args.warps}, epsilon {args.epsilon}; "
                                f"2 strips per slice pair"),
                   "slice_pairs_per_s": round(value / 2, 2),
                   "batch": B, "batches_in_flight_per_gpu": F,
                   "iterations_per_strip": round(iters / (args.steps * F * B), 1)},
        "roofline": roof,
        "cpu_baseline": cpu,
        "ranks": ranks,
    }
    if standalone:
        print(json.dumps(out), flush=True)
    return out


def strips_line(args, rank, world, local_rank, dist):
    """The production-strip figure reported beside the C2 headline: 3072x100
    ROI strip pairs, nscales 10, warps 5, batches of 256, 2 batches in flight, 2 steps."""
    import copy
    a = copy.copy(args)
    a.width, a.height, a.nscales, a.warps = 3072, 100, 10, 5
    a.iterations, a.epsilon = 300, 0.01
    a.batch, a.inflight, a.steps, a.warmup = 256, 2, 2, 1
    o = run_strips(a, rank, world, local_rank, dist, standalone=False)
    if o is None:
        return None
    return {"workload": o["config"]["workload"], "value": o["value"], "unit": o["unit"],
            "slice_pairs_per_s": o["config"]["slice_pairs_per_s"],
            "ms_per_step": o["ms_per_step"], "batch": a.batch, "batches_in_flight_per_gpu": a.inflight,
            "iterations_per_strip": o["config"]["iterations_per_strip"],
            "roofline": o["roofline"],
            "cpu_baseline": o["cpu_baseline"],
            "ranks": o["ranks"],
            "api": "tvl1_calc_batch (DESIGN.md 4.6)"}


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` (N > 1) started plainly, without a launcher: start
    `torch.distributed.run --nproc-per-node N bench.py <same args>` as a CHILD process (one
    rank per GPU, as the reference runs one process per shard: gen_cross_file_list.py:26-27,
    janelia_run.sh:3) and return its exit code.  Called before torch is imported, so this
    process never touches the GPU (no exec from a GPU-initialised process).  Rank 0's JSON
    line reaches our stdout through the inherited descriptor."""
    import signal
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           str(ROOT / "bench.py"), *sys.argv[1:]]
    if os.environ.get("BENCH_LAUNCH_DRYRUN") == "1":   # tests/test_bench_launch_cpu.py
        print(json.dumps({"launch": cmd, "torch_imported": "torch" in sys.modules}), flush=True)
        return 0
    print(f"[bench] --gpus {n} without a launcher: starting {n} ranks via "
          f"torch.distributed.run", file=sys.stderr, flush=True)
    child = subprocess.Popen(cmd, cwd=str(ROOT))

    def forward(sig, _frame):   # a driver's SIGTERM / Ctrl-C reaches the ranks too
        child.send_signal(sig)
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, forward)
    return child.wait()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # a line claiming N GPUs must come from N ranks (n_gpus is WORLD_SIZE)
        sys.exit(f"[bench] --gpus {args.gpus} but the launcher started WORLD_SIZE {world} "
                 f"ranks")
    if os.environ.get("BENCH_LAUNCH_DRYRUN") == "1":   # argument handling only (tests)
        print(json.dumps({"rank": rank, "world": world, "gpus": args.gpus,
                          "torch_imported": "torch" in sys.modules}), flush=True)
        return
    import numpy as np
    import torch

    dist = None
    # nccl (= RCCL) by default; BENCH_DIST_BACKEND=gloo rehearses the N > 1 path on fewer
    # GPUs than ranks (ranks share devices round-robin; the collectives here are only the
    # barrier and the max / sum of a few scalars, never on the data path)
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local_rank = local_rank % max(1, torch.cuda.device_count())
    # a process group whenever a launcher (torch.distributed.run) set WORLD_SIZE, N = 1
    # included: the RCCL init, barrier and device-tensor reductions then run on every
    # torchrun launch, not first on the driver's 8-GPU node (tests/test_gpu_rccl.py)
    if "WORLD_SIZE" in os.environ:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(local_rank)
    global RED_CPU, DIST_BACKEND
    RED_CPU = backend == "gloo"
    DIST_BACKEND = dist.get_backend() if dist else None
    if args.workload == "stack":
        return run_stack(args, rank, world, local_rank, dist)
    if args.workload == "strips":
        return run_strips(args, rank, world, local_rank, dist)

    from optflow_amd import capi, synth

    W, H = args.width, args.height
    params = capi.make_params(nscales=args.nscales, warps=args.warps,
                              iterations=args.iterations, epsilon=args.epsilon,
                              fast_math=int(args.fast_math), profile=args.profile,
                              inner_iterations=args.inner, outer_iterations=args.outer,
                              lambda_=args.lam, median_filtering=args.median)
    if args.profile == 1:
        args.no_fast_math_line = True   # fast_math does not apply to profile 1
    # each rank gets its own slice pair(s) of the synthetic stack (z = rank*F + j + 1 vs base)
    F = max(1, args.inflight)
    dev = torch.device("cuda", local_rank)
    slots = []
    for j in range(F):
        I0h, I1h = synth.gen_pair(W, H, seed=0x5EED, z=1 + rank * F + j)
        eng = capi.Engine(params, device=local_rank)
        eng.set_profiling(False)   # no per-launch events in the timed steps (they cost time)
        # F == 1: torch's current stream; F > 1: each ctx on its own non-blocking stream
        st = eng.stream if F > 1 else torch.cuda.current_stream(dev).cuda_stream
        slots.append(dict(I0h=I0h, I1h=I1h, eng=eng, stream=st,
                          I0=torch.from_numpy(I0h).to(dev), I1=torch.from_numpy(I1h).to(dev),
                          u=torch.empty((H, W), dtype=torch.float32, device=dev),
                          v=torch.empty((H, W), dtype=torch.float32, device=dev)))
    torch.cuda.synchronize(dev)

    def solve(sl):
        return sl["eng"].calc_device(sl["I0"].data_ptr(), W, sl["I1"].data_ptr(), W, W, H,
                                     sl["u"].data_ptr(), sl["v"].data_ptr(), 4 * W,
                                     stream=sl["stream"])

    pool = None
    if F > 1:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(max_workers=F)   # ctypes releases the GIL in tvl1_calc

    def step():
        if pool is None:
            return [solve(slots[0])]
        return list(pool.map(solve, slots))

    def timed(warmup, steps):
        """W untimed warmup steps, then exactly K timed steps bracketed by a barrier and a
        device sync on both sides; the max over ranks."""
        for _ in range(warmup):
            step()
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        stats = []
        for _ in range(steps):
            stats.extend(step())
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        own = elapsed = time.perf_counter() - t0
        if dist:
            t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if RED_CPU else dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed, stats, own

    elapsed, stats, own = timed(args.warmup, args.steps)
    ranks = rank_records(dist, local_rank, len(stats), sum(s["iterations_total"] for s in stats),
                         own)
    I0h, I1h = slots[0]["I0h"], slots[0]["I1h"]
    # one pair alone on the GPU, twice (not timed): with HIP events around every launch for
    # clean per-kernel-class durations (the roofline; no interleaving with other pairs), then
    # without them for the wall time -- the events themselves cost ~2.7 ms per C2 pair
    iso = None
    single_pair_instr_ms = None
    if not args.no_kernel_timing:
        slots[0]["eng"].set_profiling(True)
        t_iso = time.perf_counter()
        iso = solve(slots[0])
        torch.cuda.synchronize(dev)
        single_pair_instr_ms = 1e3 * (time.perf_counter() - t_iso)
        slots[0]["eng"].set_profiling(False)
    t_iso = time.perf_counter()
    solve(slots[0])
    torch.cuda.synchronize(dev)
    single_pair_ms = 1e3 * (time.perf_counter() - t_iso)

    # secondary measurement in the other math mode (same pairs, same K): the IEEE run is
    # the headline unless --fast-math; its flow is the reference for the EPE figures
    # the other arithmetic modes on the same pairs and K: pairs/s and the
    # per-pixel EPE of pair 0 against the headline run's flow -- the tolerance table
    modes = None
    if not args.no_fast_math_line:
        u_ref, v_ref = slots[0]["u"].clone(), slots[0]["v"].clone()
        modes = {}
        names = {0: "ieee", 1: "fast", 2: "fma"}
        for m in (0, 1, 2):
            if m == args.fast_math:
                continue
            mp = capi.make_params(nscales=args.nscales, warps=args.warps,
                                  iterations=args.iterations, epsilon=args.epsilon,
                                  fast_math=m, lambda_=args.lam, median_filtering=args.median)
            for sl in slots:
                sl["eng"].set_params(mp)
                sl["eng"].set_profiling(False)
            m_elapsed, m_stats, _ = timed(1, args.steps)
            solve(slots[0])
            torch.cuda.synchronize(dev)
            e = torch.sqrt((slots[0]["u"] - u_ref) ** 2 + (slots[0]["v"] - v_ref) ** 2).flatten()
            k = max(1, int(round(0.001 * e.numel())))
            modes[names[m]] = {
                "fast_math": m,
                "value": round(world * args.steps * F / m_elapsed, 4),
                "ms_per_step": round(1e3 * m_elapsed / args.steps, 3),
                "iterations_per_pair": m_stats[0]["iterations_total"],
                "same_iterations": m_stats[0]["iterations_total"] == stats[0]["iterations_total"],
                "epe_vs_headline_px": {"mean": float(e.mean()),
                                       "p99.9": float(torch.topk(e, k).values.min()),
                                       "max": float(e.max())}}

    # aggregate per-kernel timing of this rank (rank 0 reports its own kernel roofline)
    pair_bytes = sum(s["algorithmic_bytes"] for s in stats) / len(stats)
    iters = [s["iterations_total"] for s in stats]

    # the production workload beside the C2 headline, every rank taking part
    strips = None
    if not args.no_strips_line and args.profile == 0:
        for sl in slots:
            sl["eng"].close()
        strips = strips_line(args, rank, world, local_rank, dist)

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    value = world * args.steps * F / elapsed
    ms_per_step = 1e3 * elapsed / args.steps
    # the roofline is measured on ONE stream: with F > 1 in flight the launch durations
    # interleave with the other pair's kernels, so they come from the isolated solve
    src = iso if iso is not None else None
    roof = None
    if src is not None and src["kernel_ms"][0] > 0:
        roof = roofline(src["kernel_bytes"][0], src["kernel_hbm_bytes"][0], src["kernel_ms"][0],
                        src["kernel_launches"][0], TRAFFIC, PAIR_KERNEL,
                        ISSUE_MODEL if (W, H, args.nscales, args.warps, args.fast_math,
                                        args.profile) == (6144, 4096, 5, 30, 0, 0) else None)
        roof["timing"] = "one pair alone on the GPU (the isolated solve after the timed steps)"
    out = {
        "metric": METRIC,
        "value": round(value, 4),
        "unit": "slice-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "single_pair_ms": round(single_pair_ms, 3),
        "single_pair_ms_with_events": None if single_pair_instr_ms is None else round(single_pair_instr_ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "math": MATH[args.fast_math],
        "data": "synthetic",
        "config": {
            "workload": ((("C2" if (W, H, args.nscales, args.warps) == (6144, 4096, 5, 30)
                           else "pair") + f": one {W}x{H} u8 slice pair per GPU per step, nscales "
                          f"{args.nscales}, warps {args.warps}, iterations {args.iterations}, "
                          f"epsilon {args.epsilon} (reference defaults otherwise)")
                         if args.profile == 0 else
                         (f"profile 1 (CPU DualTVL1OpticalFlow schedule): one {W}x{H} u8 pair "
                          f"per GPU per step, nscales {args.nscales}, warps {args.warps}, "
                          f"inner {args.inner} x outer {args.outer}, lambda {args.lam}, median "
                          f"{args.median}, epsilon {args.epsilon}")),
            "pair": f"{W}x{H}",
            "parallelism": f"pairs sharded over {world} GPU(s), no data-path collective",
            "process_group": DIST_BACKEND,
            "pairs_in_flight_per_gpu": F,
            "step": f"one batch of {F} pair(s) solved concurrently per GPU (one ctx + stream each)",
            "iterations_per_pair": iters[0],
            "checks_per_pair": stats[0]["checks_total"],
            "pair_algorithmic_GB": round(pair_bytes / 1e9, 2),
            # SURVEY 8(d) whole-pair byte model / step time, per GPU
            "pair_roofline_frac": round(pair_bytes * args.steps * F / elapsed / 1e9 / HBM_PEAK_GBS, 4),
        },
        "roofline": roof,
        # per-pair breakdown of one solve alone on the GPU (F > 1: the isolated solve;
        # F == 1: the timed steps)
        # kernel classes from the instrumented solve, host syncs and gaps against the wall
        # time of the uninstrumented one
        "pair_breakdown_ms": None if iso is None else
            {"iterate": round(iso["kernel_ms"][0], 2), "warp": round(iso["kernel_ms"][1], 2),
             "other_kernels": round(iso["kernel_ms"][2], 2),
             "host_sync_and_gaps": round(single_pair_ms - sum(iso["kernel_ms"][:3]), 2)},
        "cpu_baseline": None,
        "math_modes": modes,
        "production_strips": strips,
        # per rank: device (PCI id), pairs solved, own elapsed time of the timed steps
        "ranks": ranks,
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(I0h, I1h, params, args.cpu_sample)
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
