import numpy as np, sys
exec(open('/tmp/treesim.py').read().split("rng=np.random")[0])
# slot order: Morton of the finest-level-ish cell (h/2) of the query
hq=h/2.0
cq=np.floor((Q.astype(np.float64)-lo)/hq).astype(np.int64).clip(0,1023)
def spread64(v):
    v=v.astype(np.uint64)&np.uint64(0x1fffff)
    v=(v|(v<<np.uint64(32)))&np.uint64(0x1f00000000ffff); v=(v|(v<<np.uint64(16)))&np.uint64(0x1f0000ff0000ff)
    v=(v|(v<<np.uint64(8)))&np.uint64(0x100f00f00f00f00f); v=(v|(v<<np.uint64(4)))&np.uint64(0x10c30c30c30c30c3)
    v=(v|(v<<np.uint64(2)))&np.uint64(0x1249249249249249); return v
mq=spread64(cq[:,0])|(spread64(cq[:,1])<<np.uint64(1))|(spread64(cq[:,2])<<np.uint64(2))
slot=np.argsort(mq,kind='stable')
W=int(sys.argv[1]) if len(sys.argv)>1 else 64
def packet(qs):
    best=np.full(len(qs),np.inf); enters=0; pts=0; leaves=0
    def enter(l,r):
        nonlocal enters; enters+=1
        ch=np.arange(4*r,4*r+4); mn,mx=levels[l-1]; out=[]
        for c in range(4):
            if ch[c]>=mn.shape[0]: continue
            g=np.maximum(np.maximum(mn[ch[c]]-qs,qs-mx[ch[c]]),0); d=(g*g).sum(1)
            if (d*(1-1e-5)<=best).any(): out.append((c,d.min()))
        out.sort(key=lambda x:x[1]); return [c for c,_ in out]
    stack=[(top,0,enter(top,0))]
    while stack:
        l,r,mask=stack[-1]
        if not mask: stack.pop(); continue
        c=mask.pop(0); ch=4*r+c
        if l==1:
            mn,mx=levels[0]; g=np.maximum(np.maximum(mn[ch]-qs,qs-mx[ch]),0); d=(g*g).sum(1)
            if not (d*(1-1e-5)<=best).any(): continue
            a,b=ls[ch],le[ch]; pts+=b-a; leaves+=1
            dd=((Ps[a:b].astype(np.float64)[None,:,:]-qs[:,None,:])**2).sum(-1).min(1); best=np.minimum(best,dd); continue
        mn,mx=levels[l-1]; g=np.maximum(np.maximum(mn[ch]-qs,qs-mx[ch]),0); d=(g*g).sum(1)
        if not (d*(1-1e-5)<=best).any(): continue
        stack.append((l-1,ch,enter(l-1,ch)))
    return enters,leaves,pts
rng=np.random.default_rng(1); E=[];L=[];Pn=[]
for w in rng.choice(M//W,60,replace=False):
    qs=Q[slot[w*W:(w+1)*W]].astype(np.float64)
    e,lv,p=packet(qs); E.append(e); L.append(lv); Pn.append(p)
print("W",W,"wave enters mean",np.mean(E),"p90",np.percentile(E,90),"leaves",np.mean(L),"points",np.mean(Pn),"p90",np.percentile(Pn,90))
