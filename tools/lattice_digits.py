"""Distribution of the half-size scalars' signed radix-16 digits (the
Straus loop's position count and top digit), by exact big-integer Euclid on
(8L, k) with the odd-d balancing step of stellard_amd/csrc/stl_lattice.h
(lattice_half) over random k.  Used to size the top-position experiment in
DESIGN_EXPERIMENTS.md section 1.  Plain Python, no GPU.

    python3 tools/lattice_digits.py
"""
import random
L=2**252+27742317777372353535851937790883648493
N=8*L
def half(k):
    rl,rs,tl,ts=N,k,0,1   # signed t
    while rs>=2**128:
        q=rl//rs
        rl,rs=rs,rl-q*rs
        tl,ts=ts,tl-q*ts
    if ts&1: return rs,ts
    j=max(0,int((rl-abs(tl))/(rs+abs(ts))+0.5))
    return rl-j*rs, tl-j*ts
def digits(v):
    v=abs(v); out=[]
    while v:
        d=v&15; v>>=4
        if d>=8: d-=16; v+=1
        out.append(d)
    return out
random.seed(1)
from collections import Counter
need=Counter(); top=Counter(); q0=0; n=20000
for _ in range(n):
    k=random.randrange(L)
    c,d=half(k)
    dc,dd=digits(c),digits(d)
    nd=max(len(dc),len(dd)); need[nd]+=1
    def dig(ds,i): return ds[i] if i<len(ds) else 0
    t=(dig(dc,32),dig(dd,32)); top[t]+=1
    ok=all(-2<=x<=1 for x in t)
    q0+=ok
print(sorted(need.items())); print(top.most_common(8)); print("per-lane q==0 at pos32:",q0/n, "wave(64):",(q0/n)**64)
