"""Per-warp iteration counts of one synthetic C2 pair (6144x4096, 5 scales, 30 warps):
the pass schedule the host derives from them (2-iteration passes end at a check)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "fibsem-optflow_amd"))
import numpy as np
from optflow_amd import capi, synth

W, H = int(os.environ.get("W", 6144)), int(os.environ.get("H", 4096))
eng = capi.Engine(capi.make_params(nscales=5, warps=30))
for z in (1, 2):
    I0, I1 = synth.gen_pair(W, H, seed=0x5EED, z=z)
    _, _, sd, wi = eng.calc_host(I0, I1)
    print(f"pair z={z} levels={sd['levels']}")
    for s in range(wi.shape[0]):
        row = wi[s]
        print(f"  level {s}: total {int(row.sum()):4d}  hist {dict(zip(*np.unique(row, return_counts=True)))}")
        print("    ", " ".join(str(int(x)) for x in row))
