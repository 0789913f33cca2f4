#!/usr/bin/env python3
"""Host estimate (float64) of the primitives a wave needs per 8x8 camera tile and per wave of
scattered rays, by the primitives' own boxes and by their relevance boxes.

    CAM="[[0,2.4,6],[0,1.4,0],38]" python tools/relevance_waves.py csg32_nested
"""
import os, math, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["WOLOLO_ALLOW_NO_DEVICE"]="1"
from csgrenderer_amd import wololo as wl, scenes
name = sys.argv[1] if len(sys.argv)>1 else "csg32_nested"
r = wl.Renderer('x', max_nodes=8192)
scenes.build(name, r); r.compile()
recs, n, npr = r.program()
OPS={2:'u',3:'i',4:'d',5:'r'}
st=[]; prims={}
pc=0
INF=np.inf
def pbox(pc):
    lo=np.full(3,-INF); hi=np.full(3,INF)
    cnt=recs[pc].u0
    for m in range(cnt):
        L=recs[pc+1+m]
        if L.op==16:
            c=np.array(L.f[:3]); rr=math.sqrt(L.f[3])
            lo=np.maximum(lo,c-rr); hi=np.minimum(hi,c+rr)
        elif L.op==17 and L.u1:
            a=L.u1-1; s=L.f[a]; h=L.f[3]
            if s>0: hi[a]=min(hi[a],h/s)
            else: lo[a]=max(lo[a],h/s)
    return lo,hi
nodes=[]
while pc<n:
    R=recs[pc]
    if R.op==1:
        lo,hi=pbox(pc); nodes.append(('p',R.u1,lo,hi,None,None)); st.append(len(nodes)-1); pc+=1+R.u0; continue
    if R.op==6: pc+=1; continue
    b=st.pop(); a=st.pop()
    op=OPS[R.op]
    la,ha=nodes[a][2],nodes[a][3]; lb,hb=nodes[b][2],nodes[b][3]
    if op=='u': lo,hi=np.minimum(la,lb),np.maximum(ha,hb)
    elif op=='i': lo,hi=np.maximum(la,lb),np.minimum(ha,hb)
    elif op=='d': lo,hi=la,ha
    else: lo,hi=lb,hb
    nodes.append((op,None,lo,hi,a,b)); st.append(len(nodes)-1); pc+=1
root=st[0]
con={root:(np.full(3,-INF),np.full(3,INF))}
order=[root]
rel={}
while order:
    k=order.pop(); c=con[k]; nd=nodes[k]
    if nd[0]=='p': rel[nd[1]]=c; continue
    op,_,lo,hi,a,b=nd
    A=nodes[a]; B=nodes[b]
    meet=lambda x,y:(np.maximum(x[0],y[0]),np.minimum(x[1],y[1]))
    if op=='u': con[a]=c; con[b]=c
    elif op=='i': con[a]=meet(c,(B[2],B[3])); con[b]=meet(c,(A[2],A[3]))
    elif op=='d': con[a]=c; con[b]=meet(c,(A[2],A[3]))
    else: con[b]=c; con[a]=meet(c,(B[2],B[3]))
    order+= [a,b]
def vol(lo,hi):
    d=np.clip(hi-lo,0,None); 
    if not np.all(np.isfinite(d)): return float('inf')
    return float(np.prod(d))
tot_own=tot_rel=0
for nd in nodes:
    if nd[0]!='p': continue
    o=nd[1]; lo,hi=nd[2],nd[3]; cl,ch=rel[o]
    ml,mh=np.maximum(lo,cl),np.minimum(hi,ch)
    print(o, 'own %.3f'%vol(lo,hi), 'meet %.3f'%vol(ml,mh))
# rays: camera rays + random directions from points on the scene
rng=np.random.default_rng(1)
def slab(o,d,lo,hi):
    with np.errstate(divide='ignore',invalid='ignore'):
        inv=1.0/d
        t0=(lo-o)*inv; t1=(hi-o)*inv
        tn=np.nanmax(np.minimum(t0,t1),axis=1); tf=np.nanmin(np.maximum(t0,t1),axis=1)
    return (tn<=tf)&(tf>1e-3)
N=200000
# camera
import json; CAM=json.loads(os.environ.get("CAM","[[0,2.4,6],[0,1.4,0],38]")); lf=np.array(CAM[0],float); la=np.array(CAM[1],float); w=(lf-la)/np.linalg.norm(lf-la); u=np.cross([0,1,0],w); u/=np.linalg.norm(u); v=np.cross(w,u)
hh=math.tan(math.radians(CAM[2])/2); ww=hh*16/9
s=rng.random(N); t=rng.random(N)
d=(-w)[None,:]+((2*s-1)*ww)[:,None]*u[None,:]+((1-2*t)*hh)[:,None]*v[None,:]
o=np.tile(lf,(N,1))
for label,(O,D) in {'camera':(o,d),'bounce':(rng.normal(size=(N,3))*0.8+np.array([0,1.6,0]),rng.normal(size=(N,3)))}.items():
    own=np.zeros(N); rl=np.zeros(N)
    for nd in nodes:
        if nd[0]!='p': continue
        lo,hi=nd[2],nd[3]; cl,ch=rel[nd[1]]
        own+=slab(O,D,lo,hi); rl+=slab(O,D,np.maximum(lo,cl),np.minimum(hi,ch))
    print(label,'own-box prims/ray %.2f'%own.mean(),'relevance-meet prims/ray %.2f'%rl.mean())
# wave-level: 8x8 pixel tiles of camera rays at 1920x1080
W,H=1920,1080
ys,xs=np.mgrid[0:H:1,0:W:1]
sel=(rng.random((H,W))<1.0)
tiles_x=W//8; tiles_y=H//8
# sample 3000 tiles
tid=rng.choice(tiles_x*tiles_y,3000,replace=False)
O=[];D=[]
for t in tid:
    ty,tx=divmod(t,tiles_x)
    px=(tx*8+np.arange(8))[None,:].repeat(8,0).ravel(); py=(ty*8+np.arange(8))[:,None].repeat(8,1).ravel()
    s=(px+0.5)/W; tt=(py+0.5)/H
    dd=(-w)[None,:]+((2*s-1)*ww)[:,None]*u[None,:]+((1-2*tt)*hh)[:,None]*v[None,:]
    D.append(dd)
D=np.concatenate(D); O=np.tile(lf,(len(D),1))
for lab,fn in [('own',lambda nd:(nd[2],nd[3])),('rel',lambda nd:(np.maximum(nd[2],rel[nd[1]][0]),np.minimum(nd[3],rel[nd[1]][1])))]:
    cnt=np.zeros(len(tid))
    for nd in nodes:
        if nd[0]!='p': continue
        lo,hi=fn(nd)
        h=slab(O,D,lo,hi).reshape(len(tid),64).any(axis=1)
        cnt+=h
    print('camera waves', lab, 'prims needed per wave %.2f'%cnt.mean())
# bounce waves: random points on scene, random dirs (incoherent)
Ob=rng.normal(size=(64*3000,3))*0.8+np.array([0,1.6,0]); Db=rng.normal(size=(64*3000,3))
for lab,fn in [('own',lambda nd:(nd[2],nd[3])),('rel',lambda nd:(np.maximum(nd[2],rel[nd[1]][0]),np.minimum(nd[3],rel[nd[1]][1])))]:
    cnt=np.zeros(3000)
    for nd in nodes:
        if nd[0]!='p': continue
        lo,hi=fn(nd)
        cnt+=slab(Ob,Db,lo,hi).reshape(3000,64).any(axis=1)
    print('bounce waves', lab, 'prims needed per wave %.2f'%cnt.mean())
