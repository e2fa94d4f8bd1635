"""Bank-conflict cost of the multi-bit twist-table layouts (TwistLds in
csrc/pbs_multibit.hip).  A monomial read of lane l fetches entry r = t mod M of t = d (1 - 4 f) mod
2N, f the lane's frequency slot; ds_read_b64 serves 32-lane groups, bank pair = position mod 32.
Cost = mean over every d and slot of the largest number of distinct entries on one bank.
Usage: python twist_swizzle_search.py SEED ITERATIONS [shiftmask]  (random linear maps of bits 5-9;
with "shiftmask" also every r ^ ((r >> k) & m), about 15 CPU-minutes)."""
import numpy as np, itertools, sys
M=1024
lane=np.arange(64)
d=np.arange(M)[:,None,None]            # d mod 1024
s=np.arange(16)[None,:,None]
f=(lane&15)+64*(lane>>4)               # freq_lane
f=f[None,None,:]+16*(s>>2)+256*(s&3)
t=(d*(1-4*f))%4096
r=t%M                                   # table entry
def cost(posfun):
    p=posfun(r)                         # [d, s, 64]
    tot=0.0; worst=0
    for g in range(2):
        a=r[:,:,32*g:32*g+32]; pp=p[:,:,32*g:32*g+32]
        bank=pp%32
        # distinct addresses per bank: count unique (bank, addr) pairs per bank
        key=bank*4096+a
        ks=np.sort(key,axis=2)
        uniq=np.concatenate([np.ones(ks.shape[:2]+(1,),bool), ks[:,:,1:]!=ks[:,:,:-1]],axis=2)
        ub=np.where(uniq, ks//4096, -1)
        # max multiplicity over banks
        cnt=np.zeros(ks.shape[:2]+(33,),int)
        for b in range(32):
            cnt[:,:,b]=(ub==b).sum(axis=2)
        m=cnt.max(axis=2)
        tot+=m.mean(); worst=max(worst,m.max())
    return tot/2, worst
def mk(A):
    A=np.array(A)
    def pf(rr):
        b=(rr>>5)&31
        fb=np.zeros_like(b)
        for i in range(5):
            for j in range(5):
                if A[i][j]: fb ^= ((b>>j)&1)<<i
        return rr ^ fb
    return pf
ident=[[1 if i==j else 0 for j in range(5)] for i in range(5)]
print("plain", cost(lambda rr: rr))
print("current (r ^ (r>>5)&31)", cost(mk(ident)))
rng=np.random.default_rng(int(sys.argv[1]) if len(sys.argv)>1 else 0)
best=(9,None)
for it in range(int(sys.argv[2]) if len(sys.argv)>2 else 300):
    A=rng.integers(0,2,(5,5))
    c=cost(mk(A))
    if c[0]<best[0]: best=(c[0],A.tolist(),c); print(it, c, A.tolist(), flush=True)
print("best", best)

# Round 4, the shipped family: position r ^ ((r >> k) & m), the same two instructions as the
# round-3 swizzle (k = 5, m = 31) for every k and 10-bit m.  Best: k = 4, m = 23 -> 2.09, worst 4.
if len(sys.argv) > 3 and sys.argv[3] == "shiftmask":
    res = sorted((cost(lambda rr, k=k, m=m: rr ^ ((rr >> k) & m)), k, m) for k in range(1, 11) for m in range(1, 1024))
    for c, k, m in res[:10]:
        print("k", k, "m", m, c)
