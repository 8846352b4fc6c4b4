"""TEST INFRASTRUCTURE (analysis; runs the oracle, so it lives under tests/).
Per level of the production strip (3072x100, nscales 10, warps 5): iterations per pair and
the unchecked run lengths between residual checks, over the oracle's check schedules of N
host-recipe strips, with the rounds of grouped batched passes at most 4 (shipped) or 8
iterations long.  Output: profiles/r5/strips_levels/schedule_model.txt."""
import sys, numpy as np, collections
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / 'fibsem-optflow_amd')]
from optflow_amd import capi, synth
from oracle import checker
p=capi.make_params(nscales=10, warps=5)
W,H,N=3072,100,8
st=synth.gen_stack(W,H,N+1,seed=0x5EED)
pairs=[]
for b in range(N):
    u,v,s,wi,tr=checker.oracle_check_trace(st[0],st[b+1],p)
    pairs.append((wi,tr))
L=pairs[0][0].shape[0]
def segs(wi,tr,l,w):
    ns=[int(r[2]) for r in tr if int(r[0])==l and int(r[1])==w]
    tot=int(wi[l,w]); pts=[]; prev=-1
    for n in ns: pts.append(n-prev); prev=n
    if tot-1>prev: pts.append(tot-1-prev)
    return pts
for l in range(L):
    it=0; r4=0; r8=0; segl=[]
    for w in range(5):
        m4=m8=0
        for wi,tr in pairs:
            sg=segs(wi,tr,l,w)
            sg[0]-=2
            if sg[0]==0: sg.pop(0)
            it+=int(wi[l,w]); segl+=sg
            m4=max(m4,sum(-(-s//4) for s in sg)); m8=max(m8,sum(-(-s//8) for s in sg))
        r4+=m4; r8+=m8
    c=collections.Counter(min(s,9) for s in segl)
    print(f"level {l}: iterations/pair {it/N:6.1f}  rounds kmax4 {r4:4d} kmax8 {r8:4d}  segment lengths {dict(sorted(c.items()))}")
