"""Compare the engine at TVL1_ENGINE_SO (e.g. an experimental build) against the in-tree
engine on synthetic C2-shaped pairs: iteration schedule and EPE.  Run on the GPU box:
  python tools/fm_check.py dump /tmp/ref.npz   (in-tree engine)
  TVL1_ENGINE_SO=ab_B/libtvl1_hip.so python tools/fm_check.py cmp /tmp/ref.npz
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "fibsem-optflow_amd"))
import numpy as np
from optflow_amd import capi, synth

mode, path = sys.argv[1], sys.argv[2]
W, H = int(os.environ.get("W", 6144)), int(os.environ.get("H", 4096))
eng = capi.Engine(capi.make_params(nscales=5, warps=30))
out = {}
for z in (1, 2, 3):
    I0, I1 = synth.gen_pair(W, H, seed=0x5EED, z=z)
    u, v, sd, wi = eng.calc_host(I0, I1)
    out[f"u{z}"], out[f"v{z}"], out[f"w{z}"] = u, v, wi
if mode == "dump":
    np.savez(path, **out)
    print("dumped", path)
else:
    ref = np.load(path)
    for z in (1, 2, 3):
        e = capi.epe(out[f"u{z}"], out[f"v{z}"], ref[f"u{z}"], ref[f"v{z}"])
        same = bool((out[f"w{z}"] == ref[f"w{z}"]).all())
        d = (out[f"w{z}"].astype(int) - ref[f"w{z}"].astype(int))
        print(f"z={z} iters_equal={same} total {int(out[f'w{z}'].sum())} vs {int(ref[f'w{z}'].sum())}"
              f" nz_diff_levels={np.nonzero(d.any(axis=1))[0].tolist()} EPE max {e.max():.3g}"
              f" mean {e.mean():.3g} p99.9 {np.quantile(e, 0.999):.3g}")
