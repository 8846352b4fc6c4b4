#!/usr/bin/env python3
"""TEST INFRASTRUCTURE (analysis; runs the oracle, so it lives under tests/).
How robust is the iteration schedule to the residual's accumulation?  (DESIGN 2.2,
VERDICT r3 "next" item 3.)

OpenCV 3.4.1's procOneScale decides when a warp stops from cuda::sum of the float diff
buffer (behind /root/reference/src/optflow.cpp:518-519); its accumulation type and order
are not restated exactly here [OCV].  For each input this tool runs the oracle twice:
  * residual mode 0 (the engine's: rows in double, in order), recording error / scaledEps
    at every check and the relative margin of each decision to its nearest threshold
    (oracle.checker.check_margins: t in {1, 2, 4, 6, ...});
  * residual mode 1 (float rows, float total, rows reversed),
and reports whether the per-warp iteration counts are unchanged, and how far the two
residuals differ at the same checks (same schedule => same u, p trajectory).

Cases: the golden fixtures, the C2 bench pair (synth.gen_pair 6144x4096, z = 1), an
adjacent C3-style pair of the host stack recipe, and with --device the device-generated C3
pair of tests/test_gpu_c3_full.py (slices 0, 1) and 4 production strips (3072x100 at
nscales 10, warps 5; bench.py's strip batch: slice 0 vs slices 1..4).
Writes a JSON and a text table (--out PREFIX)."""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fibsem-optflow_amd")]
from optflow_amd import capi, synth  # noqa: E402
from oracle import checker  # noqa: E402


def case(name, I0, I1, params):
    t0 = time.perf_counter()
    _, _, st, wi, tr = checker.oracle_check_trace(I0, I1, params)
    _, _, st1, wi1, tr1 = checker.oracle_check_trace(I0, I1, params, residual_mode=1)
    dt = time.perf_counter() - t0
    same = bool(np.array_equal(wi, wi1))
    rec = {"case": name, "size": f"{I0.shape[1]}x{I0.shape[0]}", "checks": int(len(tr)),
           "iterations": st["iterations_total"], "float_residual_same_schedule": same,
           "seconds": round(dt, 1)}
    if len(tr):
        m = checker.check_margins(tr, params.iterations)
        order = np.argsort(m)[:5]
        rec["min_margin"] = float(m.min())
        rec["closest"] = [{"level": int(tr[i, 0]), "warp": int(tr[i, 1]), "n": int(tr[i, 2]),
                           "ratio": float(tr[i, 3]), "margin": float(m[i])} for i in order]
        rec["margin_quantiles"] = {q: float(np.quantile(m, float(q))) for q in ("0.01", "0.5")}
        if same:
            dev = np.abs(tr1[:, 3] / tr[:, 3] - 1.0)
            rec["float_vs_double_max_rel"] = float(dev.max())
            rec["safety_factor"] = float(m.min() / max(dev.max(), 1e-300))
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", action="store_true", help="add the device-generated cases")
    ap.add_argument("--no-c2", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    recs = []
    for f in sorted((ROOT / "tests" / "golden").glob("*.npz")):
        d = np.load(f)
        pj = json.loads(str(d["params"]))
        p = capi.make_params(**{k: v for k, v in pj.items() if k in capi.DEFAULTS})
        recs.append(case("golden " + f.stem, d["I0"], d["I1"], p))
        print(recs[-1], flush=True)
    c2 = capi.make_params(nscales=5, warps=30)
    if not a.no_c2:
        I0, I1 = synth.gen_pair(6144, 4096, seed=0x5EED, z=1)
        recs.append(case("C2 bench pair (synth.gen_pair z=1)", I0, I1, c2))
        print(recs[-1], flush=True)
        st = synth.gen_stack(6144, 4096, 2, seed=0x5EED ^ 3)
        recs.append(case("C3-style adjacent pair (host stack recipe, z=0,1)", st[0], st[1], c2))
        print(recs[-1], flush=True)
    if a.device:
        import torch
        from optflow_amd.synth_device import DeviceStack
        dev = torch.device("cuda", 0)
        g = DeviceStack(6144, 4096, dev)
        recs.append(case("C3 device pair (DeviceStack slices 0,1)", g.slice(0).cpu().numpy(),
                         g.slice(1).cpu().numpy(), c2))
        print(recs[-1], flush=True)
        gs = DeviceStack(3072, 100, dev, seed=0x5EED)
        s0 = gs.slice(0).cpu().numpy()
        sp = capi.make_params(nscales=10, warps=5)
        for z in range(1, 5):
            recs.append(case(f"production strip (slice 0 vs {z})", s0, gs.slice(z).cpu().numpy(), sp))
            print(recs[-1], flush=True)
    lines = ["| case | size | checks | min margin | closest check (level, warp, n, ratio) | "
             "float residual: same schedule | float vs double, max rel | safety |",
             "|---|---|---|---|---|---|---|---|"]
    for r in recs:
        c = r.get("closest", [{}])[0]
        lines.append(
            f"| {r['case']} | {r['size']} | {r['checks']} | "
            f"{r.get('min_margin', float('nan')):.2e} | "
            + (f"({c['level']}, {c['warp']}, {c['n']}, {c['ratio']:.6f})" if c else "-")
            + f" | {r['float_residual_same_schedule']} | "
            f"{r.get('float_vs_double_max_rel', float('nan')):.2e} | "
            f"{r.get('safety_factor', float('nan')):.0f} |")
    table = "\n".join(lines)
    print(table)
    if a.out:
        Path(a.out + ".json").write_text(json.dumps(recs, indent=1))
        Path(a.out + ".md").write_text(table + "\n")


if __name__ == "__main__":
    main()
