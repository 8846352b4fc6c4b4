"""Wall time of the feature pre-alignment on device slices: find_alignment
(ORB detect + describe on both frames, 2-NN match, host homography) and the u8 warpAffine
of frame1, at the benchmark size and at the half-scale production size.

    python tools/align_timing.py [--reps 5] [--env-timing]

Prints one JSON line per size.  With TVL1_ALIGN_TIMING=1 in the environment the engine
also prints its own per-stage split to stderr."""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "fibsem-optflow_amd"))
from optflow_amd import capi  # noqa: E402
from optflow_amd.synth_device import DeviceStack  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sizes", default="6144x4096,3072x2048")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    eng = capi.Engine(capi.make_params())
    for sz in args.sizes.split(","):
        W, H = (int(t) for t in sz.split("x"))
        st = DeviceStack(W, H, dev, seed=11)
        f0, f1 = st.slice(0), st.slice(1)
        out = torch.empty_like(f0)
        torch.cuda.synchronize()
        eng.find_alignment(f1.data_ptr(), W, W, H, f0.data_ptr(), W, W, H)   # warm-up
        t_find, t_warp = [], []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            A, ng, oc = eng.find_alignment(f1.data_ptr(), W, W, H, f0.data_ptr(), W, W, H)
            t1 = time.perf_counter()
            eng.warp_affine_u8(f1.data_ptr(), W, W, H, out.data_ptr(), W, W, H, A)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            t_find.append(t1 - t0)
            t_warp.append(t2 - t1)
        print(json.dumps({"size": sz, "find_alignment_ms": round(1e3 * float(np.median(t_find)), 3),
                          "warp_affine_u8_ms": round(1e3 * float(np.median(t_warp)), 3),
                          "n_good": ng, "outcome": oc,
                          "affine": [round(float(x), 5) for x in A.ravel()]}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
