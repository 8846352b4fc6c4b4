import sys, os, numpy as np
sys.path.insert(0, "fibsem-optflow_amd")
from optflow_amd import capi, synth
W, H = int(sys.argv[1]), int(sys.argv[2])
kw = eval(sys.argv[3]) if len(sys.argv) > 3 else {}
p = capi.make_params(**kw)
I0, I1 = synth.gen_pair(W, H, seed=7)
eng = capi.Engine(p)
u, v, st, wi = eng.calc_host(I0, I1)
print("checks", st["checks_total"], "misses", st["speculation_misses"], "iters", st["iterations_total"], flush=True)
