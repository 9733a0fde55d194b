import numpy as np, time
from libpointmatcher_amd.synth import reference_cloud, reading_cloud
M=1_000_000
ref,_=reference_cloud(M); rd=reading_cloud(M)
m=ref[:,:3].astype(np.float64).mean(0)
P=(ref[:,:3]-m).astype(np.float32); Q=(rd[:,:3]-m).astype(np.float32)
lo=P.min(0).astype(np.float64)-1e-6; hi=P.max(0).astype(np.float64)
# pick h so that ppc ~ 8
def occ(h):
    c=np.floor((P-lo)/h).astype(np.int64); g=np.floor((hi-lo)/h).astype(np.int64)+1
    key=(c[:,2]*g[1]+c[:,1])*g[0]+c[:,0]; return key,g,c
for h in np.geomspace(0.01,0.2,40):
    key,g,c=occ(h); u=np.unique(key).size
    if M/u>=8: break
print("h",h,"g",g,"ppc",M/u)
order=np.argsort(key,kind='stable'); key_s=key[order]; Ps=P[order]; cs=c[order]
first=np.r_[True,key_s[1:]!=key_s[:-1]]
starts=np.nonzero(first)[0]; ends=np.r_[starts[1:],M]
cc=cs[starts]
def spread(v):
    v=v.astype(np.uint64)&0x3ff
    v=(v|(v<<16))&0x030000ff; v=(v|(v<<8))&0x0300f00f; v=(v|(v<<4))&0x030c30c3; v=(v|(v<<2))&0x09249249; return v
mort=spread(cc[:,0])|(spread(cc[:,1])<<1)|(spread(cc[:,2])<<2)
lo_ord=np.argsort(mort,kind='stable')
ls,le=starts[lo_ord],ends[lo_ord]
n=ls.size
bmin=np.array([Ps[a:b].min(0) for a,b in zip(ls,le)]); bmax=np.array([Ps[a:b].max(0) for a,b in zip(ls,le)])
levels=[(bmin,bmax)]
while levels[-1][0].shape[0]>1:
    mn,mx=levels[-1]; R=(mn.shape[0]+3)//4
    pm=np.full((R*4,3),np.inf,np.float32); pM=np.full((R*4,3),-np.inf,np.float32)
    pm[:mn.shape[0]]=mn; pM[:mx.shape[0]]=mx
    levels.append((pm.reshape(R,4,3).min(1),pM.reshape(R,4,3).max(1)))
top=len(levels)-1
print("leaves",n,"top",top)
def boxd2(mn,mx,q):
    g=np.maximum(np.maximum(mn-q,q-mx),0).astype(np.float64); return (g*g).sum(-1)
def search(q):
    best=np.inf; enters=0; pts=0
    # levels[l] are boxes of nodes at level l (0=leaves); record (l,r) has children (l-1, 4r..4r+3)
    def enter(l,r):
        nonlocal enters; enters+=1
        ch=np.arange(4*r,4*r+4); mn,mx=levels[l-1]; ok=ch<mn.shape[0]
        d=np.full(4,np.inf); d[ok]=boxd2(mn[ch[ok]],mx[ch[ok]],q)
        mask=[(c,d[c]) for c in range(4) if d[c]*(1-1e-5)<=min(best,1e300)]
        mask.sort(key=lambda c:c[1]); return mask
    stack=[(top,0,enter(top,0))]
    while stack:
        l,r,mask=stack[-1]
        if not mask: stack.pop(); continue
        c,dc=mask.pop(0); ch=4*r+c
        if RETEST and dc*(1-1e-5)>best: continue
        if l==1:
            a,b=ls[ch],le[ch]; pts+=b-a
            d=((Ps[a:b].astype(np.float64)-q)**2).sum(-1).min(); best=min(best,d); continue
        stack.append((l-1,ch,enter(l-1,ch)))
    return best,enters,pts
import sys
RETEST=int(sys.argv[1])
rng=np.random.default_rng(0); idx=rng.choice(M,300,replace=False)
E=[];Pn=[]
for i in idx:
    b,e,p=search(Q[i].astype(np.float64)); E.append(e); Pn.append(p)
print("enters mean",np.mean(E),"p90",np.percentile(E,90),"max",max(E)," points mean",np.mean(Pn),"p90",np.percentile(Pn,90))
# diagnostics: for a few queries, leaves with box distance <= dNN, per level node counts within dNN
from collections import Counter
for i in idx[:8]:
    q=Q[i].astype(np.float64)
    b,e,p=search(q)
    cnt=[]
    for l in range(top+1):
        mn,mx=levels[l]; d=boxd2(mn,mx,q); cnt.append(int((d*(1-1e-5)<=b).sum()))
    print("dNN %.3f"%np.sqrt(b), "enters",e,"pts",p,"nodes within dNN per level",cnt)
