"""End-to-end throughput of the optflow CLI on a slice stack ("a separate run
includes PNG decode"; 8(f) N2): decode + pre-scale + upload + solve + point-match output,
timed around the whole CLI process.

    python tools/cli_e2e.py [--slices 17] [--width 6144 --height 4096] [--out DIR]
                            [--format png|tiff|tiff_deflate] [--jobs c2,strips]
                            [--strip-batch 256,0] [--no-single-thread]

--format tiff writes uncompressed one-strip TIFFs (the strip jobs then read only the ROIs'
rows of each slice), tiff_deflate deflate TIFFs of 64-row strips (only the strips holding
them).  --strip-batch runs the strip job once per value of the CLI's build-only
"strip_batch" key (0 = one tvl1_calc per strip, the r3 path).

Writes the slices once (device-generated synthetic texture, PNG), then runs two job
configurations, each with the decode-ahead pool and with one decode thread:
  * "C2 full frame": scale 1, one custom full-frame ROI, nscales 5, warps 30;
  * "production strips": scale 0.5, top/bottom 100-row ROIs, reference defaults
    (gen_cross_file_list.py's job shape).
Output type random_points (the production output) keeps TIFF writes out of the timing.
Every default run also asks the CLI for its per-stage host timing (the build-only
"timing_json" key) and prints it beside the rate as `stages`: band reads on the decode pool
(thread-seconds), and per batch worker the wait for its chunk's bands, packing, upload (GPU
clock), the batched solve, point sampling, flow read-back and output writes; the stage that
sets the rate is the one whose thread-seconds per pair, over the threads doing it, come
closest to the wall time per pair.
--ab-pinned instead runs each job with the decode pool twice with page-locked slices and
flows and twice pageable (OPTFLOW_PINNED=1/0, alternating).
Prints one JSON line per run."""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "fibsem-optflow_amd"))
OPTFLOW = ROOT / "fibsem-optflow_amd" / "bin" / "optflow"


def make_stack(d: Path, Z: int, W: int, H: int, fmt: str = "png"):
    import torch
    from PIL import Image

    from optflow_amd.synth_device import DeviceStack
    st = DeviceStack(W, H, torch.device("cuda", 0), seed=0x5EED)
    ext = "png" if fmt == "png" else "tif"
    paths = [d / f"s{z:04d}.{ext}" for z in range(Z)]

    def save(z):
        a = st_slices[z]
        if fmt == "png":
            Image.fromarray(a).save(paths[z], compress_level=6)
        elif fmt == "tiff":
            Image.fromarray(a).save(paths[z])   # uncompressed, one strip
        else:
            Image.fromarray(a).save(paths[z], compression="tiff_adobe_deflate",
                                    tiffinfo={278: 64})
    # generated and written in groups (a 6144x4096 slice is 25 MB of host memory)
    for g in range(0, Z, 32):
        st_slices = {z: st.slice(z).cpu().numpy() for z in range(g, min(Z, g + 32))}
        with ThreadPoolExecutor(8) as ex:
            list(ex.map(save, st_slices))
    return paths


def run(cfg, d: Path, name: str, skip: int = 4, env=None):
    """Wall time of the whole CLI process, and the steady rate: the CLI prints "p q" as it
    starts each pair, so pairs after the first `skip` starts over the time from that start to
    the process end leave out process start, device init and the first decodes."""
    p = d / f"{name}.json"
    p.write_text(json.dumps(cfg))
    t0 = time.perf_counter()
    proc = subprocess.Popen([str(OPTFLOW), str(p)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                            text=True, env=env)
    starts = []
    for line in proc.stdout:
        if line.strip() and not line.startswith("{"):
            starts.append(time.perf_counter())
    err = proc.stderr.read()
    rc = proc.wait(timeout=900)
    t1 = time.perf_counter()
    if rc != 0:
        raise RuntimeError(err[-2000:])
    for line in err.splitlines():
        if line.startswith("pinned pool:"):
            print(line, flush=True)
    steady = None
    if len(starts) > skip + 1:
        steady = (len(starts) - skip) / (t1 - starts[skip])
    return t1 - t0, steady


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slices", type=int, default=17)
    ap.add_argument("--width", type=int, default=6144)
    ap.add_argument("--height", type=int, default=4096)
    ap.add_argument("--out", default=None)
    ap.add_argument("--ab-pinned", action="store_true")
    ap.add_argument("--format", choices=("png", "tiff", "tiff_deflate"), default="png")
    ap.add_argument("--jobs", default="c2,strips")
    ap.add_argument("--strip-batch", default=None,
                    help="comma list of strip_batch values for the strip job (default: the CLI's)")
    ap.add_argument("--no-single-thread", action="store_true",
                    help="skip the one-decode-thread runs")
    ap.add_argument("--strides", default="1",
                    help="pairs (z, z + s) for each s: a comma list, or A-B for every s in it "
                         "(gen_cross-style long-range pairs; long jobs over one stack)")
    ap.add_argument("--ab-env", default=None,
                    help="KEY=VAL[,KEY=VAL]: run each job twice with and twice without these "
                         "environment settings, alternating, on the same stack")
    args = ap.parse_args()
    d = Path(args.out or tempfile.mkdtemp(prefix="cli_e2e_"))
    d.mkdir(parents=True, exist_ok=True)
    t0 = time.perf_counter()
    paths = make_stack(d, args.slices, args.width, args.height, args.format)
    print(json.dumps({"stack": f"{args.slices} x {args.width}x{args.height} {args.format}",
                      "bytes": sum(os.path.getsize(p) for p in paths),
                      "write_s": round(time.perf_counter() - t0, 1)}), flush=True)
    if "-" in args.strides:
        lo, hi = (int(t) for t in args.strides.split("-"))
        strides = list(range(lo, hi + 1))
    else:
        strides = [int(t) for t in args.strides.split(",")]
    pairs = [{"p": str(paths[z]), "q": str(paths[z + s]), "output_name": f"z{z}_s{s}",
              "pId": f"{z}", "qId": f"{z + s}", "pGroupId": f"{z}.0", "qGroupId": f"{z + s}.0"}
             for s in strides for z in range(args.slices - s)]
    W, H = args.width, args.height
    jobs = {}
    if "c2" in args.jobs:
        jobs["c2_full_frame"] = {"scale": 1, "nscales": 5, "warps": 30,
                                 "rois": {"custom": [0, 0, W, H]}}
    if "strips" in args.jobs:
        for sb in (args.strip_batch.split(",") if args.strip_batch else [None]):
            key = "production_strips" + (f"_batch{sb}" if sb is not None else "")
            jobs[key] = {"scale": 0.5, "rois": {"top": 100, "bottom": 100}}
            if sb is not None:
                jobs[key]["strip_batch"] = int(sb)
    if args.ab_pinned:
        for name, extra in jobs.items():
            for rep, pinned in enumerate((1, 0, 1, 0)):
                cfg = {"output_dir": str(d / name), "output_type": "random_points",
                       "matches_file": str(d / name / "pm"), "images": pairs, **extra}
                (d / name).mkdir(exist_ok=True)
                env = dict(os.environ, OPTFLOW_PINNED=str(pinned), OPTFLOW_PINNED_TRACE="1")
                dt, steady = run(cfg, d, f"{name}_pin{pinned}_{rep}", env=env)
                n = len(pairs)
                print(json.dumps({"job": name, "pinned": pinned, "pairs": n,
                                  "wall_s": round(dt, 3), "pairs_per_s": round(n / dt, 2),
                                  "steady_pairs_per_s": steady and round(steady, 2)}), flush=True)
        return
    if args.ab_env:
        ab = dict(kv.split("=", 1) for kv in args.ab_env.split(","))
        for name, extra in jobs.items():
            for rep in range(4):
                env = dict(os.environ, **ab) if rep % 2 else None
                cfg = {"output_dir": str(d / name), "output_type": "random_points",
                       "matches_file": str(d / name / "pm"), "images": pairs, **extra}
                (d / name).mkdir(exist_ok=True)
                dt, steady = run(cfg, d, f"{name}_ab{rep}", env=env)
                n = len(pairs)
                print(json.dumps({"job": name, "env": args.ab_env if env else "default",
                                  "pairs": n, "wall_s": round(dt, 3),
                                  "pairs_per_s": round(n / dt, 2),
                                  "steady_pairs_per_s": steady and round(steady, 2)}), flush=True)
        return
    for name, extra in jobs.items():
        for threads in ((None,) if args.no_single_thread else (None, 1)):
            cfg = {"output_dir": str(d / name), "output_type": "random_points",
                   "matches_file": str(d / name / "pm"), "images": pairs, **extra}
            if threads:
                cfg["decode_threads"] = threads
            (d / name).mkdir(exist_ok=True)
            for f in (d / name).glob("pm_*.json"):
                f.unlink()
            tj = d / f"{name}_{threads or 'pool'}_timing.json"
            cfg["timing_json"] = str(tj)
            dt, steady = run(cfg, d, f"{name}_{threads or 'pool'}")
            n = len(pairs)
            stages = stage_summary(json.loads(tj.read_text()), dt) if tj.exists() else None
            # every pair's point-match record was written (random_points output)
            recs = sum(len(json.loads(f.read_text())) for f in (d / name).glob("pm_*.json"))
            print(json.dumps({"job": name, "decode_threads": threads or "default (pool)",
                              "pairs": n, "point_match_records": recs, "wall_s": round(dt, 3),
                              "pairs_per_s": round(n / dt, 2),
                              "steady_pairs_per_s": steady and round(steady, 2),
                              "stages": stages}), flush=True)


def stage_summary(t, wall):
    """The CLI's timing_json folded into per-stage seconds and the share of the wall time each
    stage's threads were busy: the decode pool's band reads over its threads, each batch-worker
    stage summed over the workers and divided by their number (workers run concurrently)."""
    out = {"wall_s": round(wall, 3), "cli_wall_s": round(t["wall_s"], 3),
           "point_match_records_s": round(t["point_match_records_s"], 3),
           "band_reads": t["decode"]["band_reads"],
           "band_read_s": round(t["decode"]["band_read_s"], 3),
           "decode_threads": t["decode"]["threads"],
           "band_read_busy_frac": round(t["decode"]["band_read_s"] / t["decode"]["threads"] / wall, 3)}
    ws = t.get("batch_workers") or []
    if ws:
        tot = {}
        for w in ws:
            for k, v in w.get("stage_s", {}).items():
                tot[k] = tot.get(k, 0.0) + v
        out["batch_workers"] = len(ws)
        out["worker_stage_s"] = {k: round(v, 3) for k, v in sorted(tot.items())}
        out["worker_stage_busy_frac"] = {k: round(v / len(ws) / wall, 3) for k, v in sorted(tot.items())}
        out["worker_s"] = round(max(w["worker_s"] for w in ws), 3)
    return out


if __name__ == "__main__":
    main()
