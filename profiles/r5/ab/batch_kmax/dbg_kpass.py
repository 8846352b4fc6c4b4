"""Debug probe (r5): batched solves with passes capped at KMAX (TVL1_BATCH_KMAX), PX = 2
everywhere (TVL1_BATCH_PX1_W=0), against the oracle: per KMAX, whether the per-warp counts
and the flow match, and where the flow first differs."""
import os, sys
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "fibsem-optflow_amd"),
                os.path.join(os.path.dirname(__file__), "..")]
import torch
from optflow_amd import capi, synth
from oracle import checker

w, h, nscales, warps = (int(x) for x in sys.argv[1:5])
eps = float(sys.argv[6]) if len(sys.argv) > 6 else 0.01
for K in [int(k) for k in sys.argv[5].split(",")]:
    os.environ["TVL1_BATCH_KMAX"] = str(K)
    p = capi.make_params(nscales=nscales, warps=warps, epsilon=eps)
    eng = capi.Engine(p)
    a, c = synth.gen_pair(w, h, seed=106, z=1)
    dev = torch.device("cuda", 0)
    d0 = torch.from_numpy(a[None].copy()).to(dev); d1 = torch.from_numpy(c[None].copy()).to(dev)
    du = torch.zeros((1, h, w), dtype=torch.float32, device=dev); dv = torch.zeros_like(du)
    torch.cuda.synchronize()
    st = eng.calc_batch_device(1, d0.data_ptr(), w, w * h, d1.data_ptr(), w, w * h, w, h,
                               du.data_ptr(), dv.data_ptr(), 4 * w, 4 * w * h, warp_iters=True)
    torch.cuda.synchronize()
    eng.close()
    u = du.cpu().numpy()[0]
    ur, vr, sr, wr = checker.oracle_calc(a, c, p)
    wi = st[0]["warp_iters"]
    same = np.array_equal(wi, wr)
    bad = u.view(np.uint32) != ur.view(np.uint32)
    print(f"KMAX={K}: warp counts {'equal' if same else 'DIFFER'}; {bad.sum()} px differ")
    if not same:
        for s in range(wi.shape[0] - 1, -1, -1):
            if not np.array_equal(wi[s], wr[s]):
                print(f"   first differing level {s}: engine {wi[s].tolist()} oracle {wr[s].tolist()}")
                break
