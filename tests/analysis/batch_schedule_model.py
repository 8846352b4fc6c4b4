"""TEST INFRASTRUCTURE (analysis; runs the oracle, so it lives under tests/).
Model of the batched pass schedule: lock step (every active pair runs the
shortest pass any of them allows) against passes grouped by length (each pair runs its own),
over the oracle's check schedules of N host-recipe 3072x100 production strips.  Pass cost
model: max(K, a) units per pair-pass (a = the memory-bound floor of a short pass, in
iteration units).  Prints both costs and pair-pass counts."""
import sys, numpy as np
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / 'fibsem-optflow_amd')]
from optflow_amd import capi, synth
from oracle import checker
p=capi.make_params(nscales=10, warps=5)
W,H,N=3072,100,48
st=synth.gen_stack(W,H,N+1,seed=0x5EED)
pairs=[]
for b in range(N):
    u,v,s,wi,tr=checker.oracle_check_trace(st[0],st[b+1],p)
    pairs.append((wi,tr))
L=pairs[0][0].shape[0]
def segs(wi,tr,l,w):
    # list of check iterations (n) for this warp, and total iterations
    ns=[int(r[2]) for r in tr if int(r[0])==l and int(r[1])==w]
    tot=int(wi[l,w])
    # segment lengths between checks; after last check, remaining (if stopped at iterations cap)
    pts=[]; prev=-1
    for n in ns:
        pts.append(n-prev); prev=n
    if tot-1>prev: pts.append(tot-1-prev)  # trailing iterations without check (cap)
    return pts  # iterations to each check
def f(K,a): return max(K,a)
for a in (2.5,3.4):
    lock=0; grp=0; lock_passes=0; grp_passes=0
    for l in range(L):
        for w in range(5):
            sg=[segs(wi,tr,l,w) for wi,tr in pairs]
            # first pass (2 iterations) fused separately for all; drop first segment's 2 iterations
            rem=[list(s) for s in sg]
            for r in rem:
                r[0]-=2
                if r[0]==0: r.pop(0)
            # grouped: each pair passes greedy <=4 per segment
            for r in rem:
                for s_ in r:
                    x=s_
                    while x>0:
                        k=min(4,x); grp+=f(k,a); grp_passes+=1; x-=k
            # lock-step
            cur=[r[0] if r else 0 for r in rem]; idx=[0]*N
            while True:
                act=[b for b in range(N) if cur[b]>0]
                if not act: break
                K=min(4,min(cur[b] for b in act))
                lock+=f(K,a)*len(act); lock_passes+=len(act)
                for b in act:
                    cur[b]-=K
                    if cur[b]==0:
                        idx[b]+=1
                        cur[b]=rem[b][idx[b]] if idx[b]<len(rem[b]) else 0
    print(f"a={a}: lock-step cost {lock:.0f} ({lock_passes} pair-passes), grouped {grp:.0f} ({grp_passes}), ratio {lock/grp:.3f}")
