"""Lockstep replay of the lane walk (scripts/sim_wave_order.py model): per wave, the med3 insertion
networks a wave runs (ballot-gated), their cost under split networks (a uniform ballot starts the
network at the lowest insertion position of the inserting lanes) and under deferred insertion
(pending slots per lane). usage: python scripts/sim_topk_insertion.py K xsub ntiles"""
# lockstep replay: per wave, count med3-network invocations and their cost under split gating
import numpy as np, sys
sys.argv=[sys.argv[0]]+sys.argv[1:]
import os
exec(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'sim_wave_order.py')).read().split("tiles = []")[0].replace("def walk(q):","def walk_old(q):"))
def walk_ev(q):
    qcx=int(q[0]*xs); qcy=int(q[1]); qcz=int(q[2]); Hx=H*xs
    best=np.full(KM,np.inf); ev={}
    def span(y,z,it):
        dyz2=slab(q[1],y)**2+slab(q[2],z)**2; tau=best[-1]
        if dyz2>tau: return
        if np.isinf(tau): x0,x1=qcx-Hx,qcx+Hx
        else:
            rr=np.sqrt(tau-dyz2); x0=max(qcx-Hx,int(np.floor((q[0]-rr)*xs))); x1=min(qcx+Hx,int(np.floor((q[0]+rr)*xs)))
        if x0>x1: return
        base=(z*G+y)*(G*xs); s0=start[base+x0]; s1=start[base+x1+1]
        d=((Ps[s0:s1]-q)**2).sum(1)
        for st,v in enumerate(d):
            if v<best[-1]:
                p=int(np.searchsorted(best,v)); best[-1]=v; best.sort(); ev[(it,st)]=p
            else: ev[(it,st)]=-1
    for t,(dy,dz) in enumerate(inner): span(qcy+dy,qcz+dz,t)
    fy=q[1]-qcy; fz=q[2]-qcz; sgy=-1 if fy<0.5 else 1; sgz=-1 if fz<0.5 else 1; tau0=best[-1]
    marked=[(oy,oz) for (oy,oz) in outer if slab(q[1],qcy+sgy*oy)**2+slab(q[2],qcz+sgz*oz)**2<=tau0]
    for i,(oy,oz) in enumerate(marked): span(qcy+sgy*oy,qcz+sgz*oz,9+i)
    return ev
trng=np.random.default_rng(7); tiles=[tuple(int(v) for v in trng.integers(3,G-7,3)) for _ in range(NT)]
splits={'none':[],'half':[KM//2],'quart':[KM//4,KM//2,3*KM//4],'tail':[KM//2,3*KM//4]}
tot={k:0.0 for k in splits}; steps=0; nets=0; nw=0
for (tx,ty,tz) in tiles:
    sel=np.where((P[:,0]>=tx)&(P[:,0]<tx+4)&(P[:,1]>=ty)&(P[:,1]<ty+4)&(P[:,2]>=tz)&(P[:,2]<tz+4))[0]
    Q=P[sel]; k2=(np.floor(Q[:,2])*G+np.floor(Q[:,1]))*G*xs+np.floor(Q[:,0]*xs); Q=Q[np.lexsort((sel,k2))]
    E=[walk_ev(q) for q in Q]
    for c0 in range(0,len(Q),64):
        W=E[c0:c0+64]; keys=set().union(*[set(e) for e in W]); nw+=1
        for kk in keys:
            steps+=1
            ps=[e[kk] for e in W if kk in e and e[kk]>=0]
            if not ps: continue
            nets+=1; pm=min(ps)
            for name,sp in splits.items():
                # cost in med3 slots + gating compares: find the largest split <= pm
                lo=0
                for s in sp:
                    if pm>=s: lo=s
                tot[name]+=(KM-lo)+len([s for s in sp if True])*0  # compares counted below
                tot[name]+=len(sp)  # one compare per split level evaluated (upper bound)
print(f"K={K} KM={KM} steps/wave {steps/nw:.1f} networks/wave {nets/nw:.1f} ({nets/steps:.2f} of steps)")
for k,v in tot.items(): print(f"  split {k:6s} med3+cmp per wave {v/nw:7.1f}")
# distribution of inserting lanes per network step + per-lane insertions
hist=np.zeros(65); lane_ins=[]; maxl=[]
for (tx,ty,tz) in tiles[:3]:
    sel=np.where((P[:,0]>=tx)&(P[:,0]<tx+4)&(P[:,1]>=ty)&(P[:,1]<ty+4)&(P[:,2]>=tz)&(P[:,2]<tz+4))[0]
    Q=P[sel]; k2=(np.floor(Q[:,2])*G+np.floor(Q[:,1]))*G*xs+np.floor(Q[:,0]*xs); Q=Q[np.lexsort((sel,k2))]
    E=[walk_ev(q) for q in Q]
    for c0 in range(0,len(Q),64):
        W=E[c0:c0+64]; keys=set().union(*[set(e) for e in W])
        li=[sum(1 for v in e.values() if v>=0) for e in W]; lane_ins+=li; maxl.append(max(li))
        for kk in keys:
            n=sum(1 for e in W if kk in e and e[kk]>=0)
            hist[n]+=1
print("lane insertions mean %.1f, wave max mean %.1f"%(np.mean(lane_ins),np.mean(maxl)))
h=hist[1:]; print("inserting lanes per network: ", {i+1:int(v) for i,v in enumerate(h) if v})
def order_key(kk): return kk
res={0:0,1:0,2:0,3:0}; nw=0
for (tx,ty,tz) in tiles:
    sel=np.where((P[:,0]>=tx)&(P[:,0]<tx+4)&(P[:,1]>=ty)&(P[:,1]<ty+4)&(P[:,2]>=tz)&(P[:,2]<tz+4))[0]
    Q=P[sel]; k2=(np.floor(Q[:,2])*G+np.floor(Q[:,1]))*G*xs+np.floor(Q[:,0]*xs); Q=Q[np.lexsort((sel,k2))]
    E=[walk_ev(q) for q in Q]
    for c0 in range(0,len(Q),64):
        W=E[c0:c0+64]; keys=sorted(set().union(*[set(e) for e in W])); nw+=1
        for Pn in (0,1,2,3):
            pend=np.zeros(len(W),int); nets=0
            for kk in keys:
                ps=np.array([kk in e and e[kk]>=0 for e in W])
                if Pn==0:
                    nets+=ps.any(); continue
                if (ps & (pend>=Pn)).any():
                    nets+=pend.max(); pend[:]=0
                pend+=ps
            nets+=pend.max()
            res[Pn]+=nets
for Pn,v in res.items(): print(f"pending slots {Pn}: networks/wave {v/nw:.1f}")
