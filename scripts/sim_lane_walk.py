"""numpy replay of the lane walk (csrc/kernels/query.hip, knn_tile_kernel LANE) on a uniform cloud at
3.4 points/cell: per-lane row spans with the evolving K+M+1-th bound, then the wave's candidate
steps for the row-synchronous loop (v0: unroll-3 + remainder, as shipped), a masked tail (v1) and a
flattened per-lane loop (v2), plus schedule costs of flattened variants (row setup = crow units).
usage: ORDER=fixed|inner|dist python scripts/sim_lane_walk.py K xsub [crow]
Used for DESIGN.md section 3 (row-synchronous waste; x sub-cells; row orders)."""
import numpy as np, sys
rng=np.random.default_rng(2)
G=28; rho=3.4; N=int(G**3*rho)
P=rng.random((N,3))*G
K=int(sys.argv[1]) if len(sys.argv)>1 else 16
xs=int(sys.argv[2]) if len(sys.argv)>2 else 1
M=2; KM=K+M+1; H=2
cx=np.floor(P[:,0]*xs).astype(int); cy=np.floor(P[:,1]).astype(int); cz=np.floor(P[:,2]).astype(int)
key=(cz*G+cy)*(G*xs)+cx
o=np.lexsort((np.arange(N), key)); ks=key[o]; Ps=P[o]
start=np.searchsorted(ks, np.arange(G*G*G*xs+1))
offs=[0,1,-1,2,-2]
import os
ORDER=os.environ.get('ORDER','fixed')
rows=[(dy,dz) for dz in offs for dy in offs]
if ORDER=='inner': rows=[r for r in rows if max(abs(r[0]),abs(r[1]))<=1]+[r for r in rows if max(abs(r[0]),abs(r[1]))==2]
if ORDER=='dist':
    E={0:0,1:0.5,-1:0.5,2:1.5,-2:1.5}
    rows=sorted(rows,key=lambda r:(E[r[0]]**2+E[r[1]]**2))
def lane_spans(q):
    qcx=int(q[0]*xs); qcy=int(q[1]); qcz=int(q[2]); Hx=H*xs
    best=np.full(KM,np.inf); sp=[]
    for (dy,dz) in rows:
        y,z=qcy+dy,qcz+dz
        dzb=max(0,z-q[2],q[2]-(z+1)); dyb=max(0,y-q[1],q[1]-(y+1)); dyz2=dyb*dyb+dzb*dzb
        tau=best[-1]
        if dyz2>tau: sp.append(0); continue
        if np.isinf(tau): x0,x1=qcx-Hx,qcx+Hx
        else:
            rr=np.sqrt(tau-dyz2); x0=max(qcx-Hx,int(np.floor((q[0]-rr)*xs))); x1=min(qcx+Hx,int(np.floor((q[0]+rr)*xs)))
        if x0>x1: sp.append(0); continue
        base=(z*G+y)*(G*xs); s0=start[base+x0]; s1=start[base+x1+1]
        sp.append(s1-s0)
        for s in range(s0,s1):
            d=((Ps[s]-q)**2).sum()
            if d<best[-1]: best[-1]=d; best.sort()
    return sp
# tiles of 4x4x4 y/z-cells: queries ordered by tile row (y,z) then x
tot={'v0':0,'v1':0,'v2':0,'cand':0,'rows':0}; nw=0
for (tx,ty,tz) in [(8,8,8),(12,8,16),(16,12,8),(8,16,12)]:
    sel=np.where((P[:,0]>=tx)&(P[:,0]<tx+4)&(P[:,1]>=ty)&(P[:,1]<ty+4)&(P[:,2]>=tz)&(P[:,2]<tz+4))[0]
    Q=P[sel]; k2=(np.floor(Q[:,2])*G+np.floor(Q[:,1]))*G*xs+np.floor(Q[:,0]*xs)
    Q=Q[np.lexsort((sel,k2))]
    for c in range(0,len(Q),64):
        W=Q[c:c+64]; S=np.array([lane_spans(q) for q in W])  # lanes x 25
        act=(S>0).any(0)
        v0=sum(3*(S[:,t]//3).max()+ (S[:,t]%3).max() for t in range(25) if act[t])
        v1=sum(3*((S[:,t]+2)//3).max() for t in range(25) if act[t])
        v2=(3*((S+2)//3)).sum(1).max()
        tot['v0']+=v0; tot['v1']+=v1; tot['v2']+=v2; tot['cand']+=S.sum(1).mean(); tot['rows']+=act.sum(); nw+=1
print(f"K={K} xs={xs} per wave: mean lane cand {tot['cand']/nw:.1f}  active rows {tot['rows']/nw:.1f}  steps v0(cur) {tot['v0']/nw:.1f}  v1(masked tail) {tot['v1']/nw:.1f}  v2(flat) {tot['v2']/nw:.1f}")

def costs(S, crow=0.6, theta=16):
    L=S.shape[0]
    # A: row-synchronous (current): every active row iteration: setup + unroll-3 loop + remainder
    act=(S>0).any(0)
    A=sum(crow + (S[:,t]//3).max() + (S[:,t]%3).max()/3.0 for t in range(25) if act[t])
    # per-lane list of (rows examined, span) for each non-empty span
    seqs=[]
    for l in range(L):
        q=[]; skip=0
        for t in range(25):
            if S[l,t]>0: q.append((skip+1, S[l,t])); skip=0
            else: skip+=1
        seqs.append(q)
    def sim(theta):
        idx=[0]*L; rem=[0]*L; cost=0.0
        # initial refill
        while True:
            need=[l for l in range(L) if rem[l]<=0 and idx[l]<len(seqs[l])]
            active=[l for l in range(L) if rem[l]>0]
            if need and (len(need)>=theta or not active):
                cost+=crow*max(seqs[l][idx[l]][0] for l in need)
                for l in need: rem[l]=seqs[l][idx[l]][1]; idx[l]+=1
                continue
            if not active: break
            cost+=1.0
            for l in active: rem[l]-=3
        return cost
    return A, sim(1), sim(16), sim(32)
tot=np.zeros(4); nw=0
for (tx,ty,tz) in [(8,8,8),(12,8,16),(16,12,8),(8,16,12)]:
    sel=np.where((P[:,0]>=tx)&(P[:,0]<tx+4)&(P[:,1]>=ty)&(P[:,1]<ty+4)&(P[:,2]>=tz)&(P[:,2]<tz+4))[0]
    Q=P[sel]; k2=(np.floor(Q[:,2])*G+np.floor(Q[:,1]))*G*xs+np.floor(Q[:,0]*xs)
    Q=Q[np.lexsort((sel,k2))]
    for c in range(0,len(Q),64):
        W=Q[c:c+64]; S=np.array([lane_spans(q) for q in W])
        tot+=np.array(costs(S,crow=float(sys.argv[3]) if len(sys.argv)>3 else 0.6)); nw+=1
print("cost units (1 = one 3-candidate iteration): A(row-sync) %.1f  B(immediate) %.1f  C16 %.1f  C32 %.1f" % tuple(tot/nw))
