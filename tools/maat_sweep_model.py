#!/usr/bin/env python3
"""CPU model of a sweep-style MaaT epoch: levels of a serial
prefix decided exactly (L_i / U_i of maat.hip's formula against the running
max read cts / min write cts of the committed rows), then a filter that aborts
every later txn whose bounds from the commits so far are already empty; the
survivors form the next level.  Prints the level sizes and checks the
decisions against the oracle.  PL="1024,3072,8192,..." sets the prefixes."""
import numpy as np, sys, time
import os
ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0,ROOT); sys.path.insert(0,os.path.join(ROOT,'tests'))
import deneva_amd as d, _oracle as orc
from deneva_amd import RD, WR
n=1<<20
b=d.gen_ycsb(n_txn=n, zipf_theta=0.9)
off=np.asarray(b.offsets).astype(np.int64); keys=np.asarray(b.keys); at=np.asarray(b.acctype)
# exact sequential (empty row ts)
INF=1<<62
t0=time.time()
ks=[keys[off[i]:off[i+1]].tolist() for i in range(n)]
ws=[(at[off[i]:off[i+1]]!=RD).tolist() for i in range(n)]
print('prep',time.time()-t0)
def decide(i, maxr, minw):
    L=1; U=INF
    for k,w in zip(ks[i],ws[i]):
        if w:
            r=maxr.get(k)
            if r is not None and r+1>L: L=r+1
        m=minw.get(k)
        if m is not None and m-1<U: U=m-1
    return L,U
def commit(i,L,maxr,minw):
    for k,w in zip(ks[i],ws[i]):
        if w:
            m=minw.get(k)
            if m is None or L<m: minw[k]=L
        else:
            r=maxr.get(k)
            if r is None or L>r: maxr[k]=L
# sweep
lst=list(range(n)); maxr={}; minw={}
import os
P=[int(x) for x in os.environ.get("PL","1024").split(",")]
lvl=0; res={}
while lst:
    p=P[min(lvl,len(P)-1)]
    pre=lst[:p]; rest=lst[p:]
    newr={}; neww={}
    for i in pre:
        L,U=decide(i,maxr,minw)
        if L<U: commit(i,L,maxr,minw); res[i]=L
        else: res[i]=-1
    # filter: bound check only (exact abort if L>=U with commits so far: still an abort later since L grows, U shrinks)
    surv=[]
    for i in rest:
        L,U=decide(i,maxr,minw)
        if L>=U: res[i]=-1
        else: surv.append(i)
    print('level',lvl,'serial',len(pre),'list',len(lst),'survivors',len(surv), time.time()-t0, flush=True)
    lst=surv; lvl+=1
ecomm=sum(1 for v in res.values() if v>=0); print('commits',ecomm)
rc,cts,_=orc.maat(b)
mine=np.array([0 if res[i]>=0 else 1 for i in range(n)])
print('match rc', np.array_equal((np.asarray(rc)!=0).astype(int), mine))
