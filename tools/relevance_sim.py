#!/usr/bin/env python3
"""Host simulation (float64) of relevance-box clipping for the specialised kernel:
events and sweep steps per ray with and without clipping each primitive to the meet of its
ancestors' boxes, for camera rays and scattered rays of a scene's compiled program.

    python tools/relevance_sim.py csg32_nested
"""
import os, math, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["WOLOLO_ALLOW_NO_DEVICE"]="1"
from csgrenderer_amd import wololo as wl, scenes
name=sys.argv[1]
r=wl.Renderer('x',max_nodes=8192); scenes.build(name,r); r.compile()
recs,n,npr=r.program()
INF=np.inf
def members(pc):
    out=[]
    for m in range(recs[pc].u0):
        L=recs[pc+1+m]; out.append((L.op,L.u1,list(L.f)))
    return out
nodes=[];st=[];pc=0;prim_m={}
def pbox(mem):
    lo=np.full(3,-INF);hi=np.full(3,INF)
    for op,u1,f in mem:
        if op==16:
            c=np.array(f[:3]);rr=math.sqrt(f[3]);lo=np.maximum(lo,c-rr);hi=np.minimum(hi,c+rr)
        elif op==17 and u1:
            a=u1-1
            if f[a]>0: hi[a]=min(hi[a],f[3])
            else: lo[a]=max(lo[a],-f[3])
    return lo,hi
while pc<n:
    R=recs[pc]
    if R.op==1:
        mem=members(pc);prim_m[R.u1]=mem;lo,hi=pbox(mem)
        nodes.append(dict(op='p',o=R.u1,lo=lo,hi=hi));st.append(len(nodes)-1);pc+=1+R.u0;continue
    if R.op==6: pc+=1;continue
    b=st.pop();a=st.pop();op={2:'u',3:'i',4:'d',5:'r'}[R.op]
    A,B=nodes[a],nodes[b]
    if op=='u': lo,hi=np.minimum(A['lo'],B['lo']),np.maximum(A['hi'],B['hi'])
    elif op=='i': lo,hi=np.maximum(A['lo'],B['lo']),np.minimum(A['hi'],B['hi'])
    elif op=='d': lo,hi=A['lo'],A['hi']
    else: lo,hi=B['lo'],B['hi']
    nodes.append(dict(op=op,a=a,b=b,lo=lo,hi=hi));st.append(len(nodes)-1);pc+=1
root=st[0]
# R_Q: intersection of boxes of all ancestors incl self
Rbox={}
def walk(k,lo,hi):
    nd=nodes[k];lo=np.maximum(lo,nd['lo']);hi=np.minimum(hi,nd['hi'])
    if nd['op']=='p': Rbox[nd['o']]=(lo,hi);return
    walk(nd['a'],lo,hi);walk(nd['b'],lo,hi)
walk(root,np.full(3,-INF),np.full(3,INF))
def ev(k,bits):
    nd=nodes[k]
    if nd['op']=='p': return bits[nd['o']]
    A=ev(nd['a'],bits);B=ev(nd['b'],bits)
    return {'u':A|B,'i':A&B,'d':A&~B,'r':B&~A}[nd['op']]
def prim_ivl(mem,o,d):
    a=np.full(len(o),-INF);b=np.full(len(o),INF)
    for op,u1,f in mem:
        if op==16:
            c=np.array(f[:3]);oc=o-c;bb=(oc*d).sum(1);cc=(oc*oc).sum(1)-f[3];disc=bb*bb-cc
            ok=disc>=0;s=np.sqrt(np.where(ok,disc,0));la=np.where(ok,-bb-s,INF);lb=np.where(ok,-bb+s,-INF)
        else:
            nrm=np.array(f[:3]);den=d@nrm;dist=f[3]-o@nrm
            with np.errstate(divide='ignore',invalid='ignore'): t=dist/den
            la=np.where(den<0,t,np.where(den>0,-INF,np.where(dist>=0,-INF,INF)))
            lb=np.where(den>0,t,np.where(den<0,INF,np.where(dist>=0,INF,-INF)))
        a=np.maximum(a,la);b=np.minimum(b,lb)
    return a,b
def span(lo,hi,o,d):
    with np.errstate(divide='ignore',invalid='ignore'):
        inv=1.0/d;t0=(lo-o)*inv;t1=(hi-o)*inv
        tn=np.max(np.nan_to_num(np.minimum(t0,t1),nan=-INF),axis=1);tf=np.min(np.nan_to_num(np.maximum(t0,t1),nan=INF),axis=1)
    return tn,tf
rng=np.random.default_rng(2)
import json
CAM=json.loads(os.environ.get("CAM","[[0,2.4,6],[0,1.4,0],38]"))
lf=np.array(CAM[0],float);la_=np.array(CAM[1],float);w=(lf-la_)/np.linalg.norm(lf-la_);u=np.cross([0,1,0],w);u/=np.linalg.norm(u);v=np.cross(w,u)
hh=math.tan(math.radians(CAM[2])/2);ww=hh*16/9
N=20000
s=rng.random(N);t=rng.random(N)
d=(-w)[None,:]+((2*s-1)*ww)[:,None]*u[None,:]+((1-2*t)*hh)[:,None]*v[None,:];d/=np.linalg.norm(d,axis=1)[:,None]
o=np.tile(lf,(N,1))
db=rng.normal(size=(N,3));db/=np.linalg.norm(db,axis=1)[:,None]
sets={'camera':(o,d),'bounce':(rng.normal(size=(N,3))*0.7+np.array([0,1.6,0]),db)}
tmin=1e-3
for lab,(O,D) in sets.items():
    for clip in (False,True):
        iv={}
        for p,mem in prim_m.items():
            a,b=prim_ivl(mem,O,D)
            if clip:
                tn,tf=span(*Rbox[p],O,D);a=np.maximum(a,tn);b=np.minimum(b,tf)
            iv[p]=(a,b)
        nev=np.zeros(N);steps=np.zeros(N)
        for i in range(N):
            evs=[];bits={}
            for p,(a,b) in iv.items():
                A,B=a[i],b[i]
                bits[p]=bool(A<=tmin<B)
                if A<=B:
                    if A>tmin: evs.append((A,p))
                    if B>tmin and B<INF: evs.append((B,p))
            evs.sort();nev[i]=len(evs)
            r0=ev(root,bits);k=0
            for tt,p in evs:
                k+=1;bits[p]=not bits[p]
                if ev(root,bits)!=r0: break
            steps[i]=k
        print(name,lab,'clip' if clip else 'noclip','events %.2f'%nev.mean(),'sweep steps %.2f'%steps.mean(), 'p90 events %d'%np.percentile(nev,90), 'max', nev.max())
