#!/usr/bin/env python3
"""CPU emulation of the binary BVH traversal of bounce rays (hrt_debug_bvh_build's nodes), to separate
what the node margins cost from what the hierarchy itself needs.

Bounce rays come from a small float64 path tracer over the scene's triangles (camera rays through the
preset's ray centres, Lambertian bounces about the hit normal, up to 9 segments).  Each ray walks the
preorder / escape-link tree with the kernel's node test (back-face cone, box grown by the margin at the
node's own R, t interval [-abs, t(1 + rel) + abs]) under three margin rules: the product's scalar
a + b R ('sc'), per-axis in-plane margins ('ax': the inflated triangle stays in its plane), and none
('zero', a lower bound).  t is the ray's final closest hit (INF=1: no pruning by t at all).

    python3 tools/margin_emul.py cave 300 [INF]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from helpers import SceneCase
import test_bvh
INF=int(sys.argv[3]) if len(sys.argv)>3 else 0
scene=sys.argv[1] if len(sys.argv)>1 else 'cave'; NR=int(sys.argv[2]) if len(sys.argv)>2 else 400
case=SceneCase(scene,(64,64),1,1)
b=test_bvh.build(case.tris,case.meshes,leaf=3 if scene=='cave' else 2)
P=b['prims'].astype(np.float64); N=b['nodes']
A=P[:,0:3]; E1=P[:,4:7]; E2=P[:,8:11]; NR_=P[:,12:15]
B=A+E1; C=A+E2
nn=np.linalg.norm(NR_,axis=1); nh=NR_/nn[:,None]
eps=2.0**-24; tau=float(os.environ.get("TAU", "4.5e-3"))
rho=np.linalg.norm(NR_-np.cross(E1,E2),axis=1)/nn+1e-12
g=np.maximum(np.linalg.norm(E1,axis=1),np.linalg.norm(E2,axis=1))/nn
lo=np.minimum(np.minimum(A,B),C); hi=np.maximum(np.maximum(A,B),C); ext=(hi-lo).max(1)
D=np.maximum(np.maximum(np.abs(2*A-B-C),np.abs(2*B-A-C)),np.abs(2*C-A-B))  # per-axis in-plane displacement
inv_tpi=1.02/(tau-rho-4e-7)
ca=(6*eps+(1.01*rho+3.2*eps)*inv_tpi); cb=18.4*eps*g*inv_tpi
a_sc=2.02*ext*ca; b_sc=2.02*ext*cb
a_ax=1.01*D*ca[:,None]*1.0001; b_ax=1.01*D*cb[:,None]*1.0001
rho_max=rho.max(); inv_tp=1.02/(tau-rho_max-4e-7)
abs_coef=2.1*(4.2*eps+rho_max)*inv_tp*(1+1e-6); rel_t=(2.1*(3.2*eps+rho_max)*inv_tp+4*eps)*(1+1e-6)
nnode=len(N); info=N[:,14].view(np.uint32); esc=N[:,15].view(np.uint32)
# prim range per node
first=np.zeros(nnode,np.int64); last=np.zeros(nnode,np.int64)
for k in range(nnode-1,-1,-1):
    cnt=info[k]>>27
    if cnt: first[k]=info[k]&0x07FFFFFF; last[k]=first[k]+cnt
    else:
        l=k+1; r=info[k]; first[k]=first[l]; last[k]=last[r]
na_sc=np.array([a_sc[first[k]:last[k]].max() for k in range(nnode)]); nb_sc=np.array([b_sc[first[k]:last[k]].max() for k in range(nnode)])
na_ax=np.array([a_ax[first[k]:last[k]].max(0) for k in range(nnode)]); nb_ax=np.array([b_ax[first[k]:last[k]].max(0) for k in range(nnode)])
print('node margins: host a/b vs emul', np.median(N[:,3]/np.maximum(na_sc,1e-30)), np.median(N[:,7]/np.maximum(nb_sc,1e-30)))
lo_n=N[:,0:3].astype(np.float64); hi_n=N[:,4:7].astype(np.float64)
ax=N[:,8:11].astype(np.float64); cph=N[:,11].astype(np.float64); sph=N[:,12].astype(np.float64)
rng=np.random.default_rng(7)
area=0.5*nn; pr=area/area.sum()
R0lo=lo_n[0]; R0hi=hi_n[0]
def closest(o,d):
    ao=o-A; dn=NR_@d; det=-dn
    with np.errstate(all='ignore'):
        t=(ao*NR_).sum(1)/det; dao=np.cross(ao,d); u=(E2*dao).sum(1)/det; v=-(E1*dao).sum(1)/det
    ok=(dn<0)&(t>0.001)&(u>=0)&(v>=0)&(1-u-v>=0)
    return t[ok].min() if ok.any() else np.inf
W,H=case.size
pc=case.push(1); M=np.array(pc.cam_alignment_mat,np.float64); cam=np.array(pc.cam_pos[:3],np.float64)
rays=np.asarray(case.rays['sample_centre'],np.float64)[:,:3]
def hit_full(o,d):
    ao=o-A; dn=NR_@d; det=-dn
    with np.errstate(all='ignore'):
        t=(ao*NR_).sum(1)/det; dao=np.cross(ao,d); u=(E2*dao).sum(1)/det; v=-(E1*dao).sum(1)/det
    ok=(dn<0)&(t>0.001)&(u>=0)&(v>=0)&(1-u-v>=0)
    if not ok.any(): return np.inf,-1
    t=np.where(ok,t,np.inf); j=int(np.argmin(t)); return t[j],j
bounce=[]
tries=0
while len(bounce)<NR and tries<20000:
    tries+=1
    c=rays[rng.integers(len(rays))]; w=np.array([M[0]*c[0]+M[4]*c[1]+M[8]*c[2],M[1]*c[0]+M[5]*c[1]+M[9]*c[2],M[2]*c[0]+M[6]*c[1]+M[10]*c[2]])
    o=cam.copy(); d=w/np.linalg.norm(w)
    for k in range(9):
        t,j=hit_full(o,d)
        if j<0: break
        o=o+d*t; s_=rng.normal(size=3); s_/=np.linalg.norm(s_); d=nh[j]+s_; d/=np.linalg.norm(d)
        bounce.append((o.copy(),d.copy()))
print('bounce rays collected',len(bounce))
stats={m:[0,0] for m in ('sc','ax','zero')}
hits=0
for r in range(NR):
    o,d=bounce[r]
    tb=closest(o,d); hits+=np.isfinite(tb)
    Rs=np.sqrt(np.maximum(np.abs(o-R0lo),np.abs(R0hi-o))@np.maximum(np.abs(o-R0lo),np.abs(R0hi-o)))*1.0001
    abs_t=abs_coef*Rs; t_hi=((tb if np.isfinite(tb) else 3.4e38) if not INF else 3.4e38)*(1+rel_t)+abs_t
    with np.errstate(divide='ignore'): inv=1.0/d
    for mode in stats:
        k=0; vis=0; pt=0
        while k<nnode:
            vis+=1
            x=ax[k]@d; xa=max(abs(x)-2e-6,0); s_up=np.sqrt(max(1-xa*xa,0))+1e-6
            visit= not (x*cph[k]-s_up*sph[k]-1e-6>1e-5)
            if visit:
                f=np.maximum(o-lo_n[k],hi_n[k]-o); Rm=min(np.sqrt(f@f)*1.0001,Rs)
                if mode=='sc': mg=np.full(3,na_sc[k]+nb_sc[k]*Rm)
                elif mode=='ax': mg=na_ax[k]+nb_ax[k]*Rm
                else: mg=np.zeros(3)
                with np.errstate(invalid='ignore'):
                    t0=(lo_n[k]-mg-o)*inv; t1=(hi_n[k]+mg-o)*inv
                tn=max(-abs_t,np.nanmax(np.minimum(t0,t1))); tf=min(t_hi,np.nanmin(np.maximum(t0,t1)))
                visit= not (tn-abs(tn)*1e-6 > tf+abs(tf)*1e-6)
            cnt=info[k]>>27
            if visit and cnt: pt+=cnt
            k = k+1 if (visit and not cnt) else esc[k]
        stats[mode][0]+=vis; stats[mode][1]+=pt
print(scene,'rays',NR,'hit frac',hits/NR)
for m,(v,p) in stats.items(): print(f'  {m:5s} node tests/ray {v/NR:.1f}  prim tests/ray {p/NR:.1f}')
