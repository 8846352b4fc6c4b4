#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.npz) with the oracle.

The reference ships no tests or golden outputs and OpenCV 3.4.1 is absent (SURVEY
8c), so these vectors are produced by oracle/ (the CPU restatement of OpenCV 3.4.1
CUDA TV-L1) from seeded synthetic inputs: they pin the restatement against drift
and give the GPU tests a fixed target.  PARITY UNPINNED w.r.t. OpenCV itself.

Each fixture holds: I0, I1 (u8), u, v (f32), warp_iters (int32 [levels, warps]),
levels, params (json string), seed.
Run:  python tests/golden/make_golden.py
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "fibsem-optflow_amd"))
sys.path.insert(0, str(ROOT))
from optflow_amd import capi, synth
from oracle import checker  # noqa: E402

CASES = {
    "pair_64x48_s5w3": (64, 48, 101, dict(nscales=5, warps=3)),
    "pair_128x96_defaults": (128, 96, 102, dict()),
    "pair_160x120_bench_params": (160, 120, 103, dict(nscales=5, warps=30)),
    "pair_97x61_gamma": (97, 61, 104, dict(nscales=4, warps=3, gamma=0.2)),
    "pair_96x64_fixed_work": (96, 64, 105, dict(nscales=3, warps=2, epsilon=0.0, iterations=9)),
    "pair_96x64_median5": (96, 64, 106, dict(nscales=4, warps=3, median_filtering=5)),
}


def main():
    out = Path(__file__).resolve().parent
    for name, (W, H, seed, kw) in CASES.items():
        I0, I1 = synth.gen_pair(W, H, seed=seed)
        p = capi.make_params(**kw)
        u, v, st, wi = checker.oracle_calc(I0, I1, p)
        params = {f: getattr(p, f) for f, _ in capi.TVL1Params._fields_}
        np.savez_compressed(out / f"{name}.npz", I0=I0, I1=I1, u=u, v=v,
                            warp_iters=wi.astype(np.int32), levels=st["levels"],
                            params=json.dumps(params), seed=seed)
        print(name, st["levels"], st["iterations_total"])


if __name__ == "__main__":
    main()
