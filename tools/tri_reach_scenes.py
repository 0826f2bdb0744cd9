"""The reach of the rounded triangle test (triangle.zig:48-70) on the reference
scenes' own triangles: the grazing-triangle rays of tests/grazing_tris.py traced
by the oracle through the surface LIST (every triangle tested), and for every
accepted triangle hit the exact plane crossing X's distance outside the
triangle (the largest violated edge distance), as K in
    distance = K u |ao| |e1| |e2| / det        (u = 2^-24)
Prints, per scene, the rays, the accepted hits whose X lies outside its
triangle, and the largest K (DESIGN.md §3 "Triangles: grazing rays and the
guard"; tools/tri_reach.py measures the same K on random triangles).

usage: python tools/tri_reach_scenes.py
"""
import sys, os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, zraytrace_amd as z
from oracle import oracle_py as O
from test_gpu_parity import prim_array
import grazing_tris as G
U = 2.0 ** -24
for si in [3,2,0]:
    s=z.load_scene(si); pr=prim_array(s.view.contents)
    mins,maxs,left,right,_=O.bvh_build(s.view)
    span=G.scene_span(pr)
    Kmax=0; cnt=0; tot=0
    for seed in range(5):
        o,d=G.grazing_triangle_rays(pr,mins,maxs,left,right,n=40000,seed=100+seed,span=span)
        t,p=O.trace(s.view,False,o,d)   # list: every triangle tested
        tri=(p>=0)&(pr["kind"][np.maximum(p,0)]==1)
        idx=np.nonzero(tri)[0]; P=p[idx]
        a=pr["a"][P].astype(np.float32); b=pr["b"][P].astype(np.float32); c=pr["c"][P].astype(np.float32)
        e1=(b-a).astype(np.float64); e2=(c-a).astype(np.float64)
        nn=np.cross(e1,e2); oo=o[idx].astype(np.float64); dd=d[idx].astype(np.float64); dd/=np.linalg.norm(dd,axis=1)[:,None]
        A=a.astype(np.float64)
        ts=((A-oo)*nn).sum(1)/(dd*nn).sum(1); X=oo+ts[:,None]*dd
        # exact barycentric of X: distance outside the triangle (in plane)
        M=np.stack([e1,e2],2)  # 3x2
        rhs=X-A
        uv=np.linalg.lstsq if False else None
        G11=(e1*e1).sum(1);G12=(e1*e2).sum(1);G22=(e2*e2).sum(1); r1=(rhs*e1).sum(1); r2=(rhs*e2).sum(1)
        den=G11*G22-G12*G12; uu=(G22*r1-G12*r2)/den; vv=(G11*r2-G12*r1)/den
        out=np.maximum.reduce([-uu*np.linalg.norm(e1,axis=1), -vv*np.linalg.norm(e2,axis=1), (uu+vv-1)*np.minimum(np.linalg.norm(e1,axis=1),np.linalg.norm(e2,axis=1))])
        det=-(dd*nn).sum(1)
        P12=np.linalg.norm(e1,axis=1)*np.linalg.norm(e2,axis=1)
        aon=np.linalg.norm(oo-A,axis=1)
        K=np.where(out>0, out*det/(U*aon*P12), 0)
        Kmax=max(Kmax,K.max()); cnt+=(out>0).sum(); tot+=len(o)
    print(si,'rays',tot,'accepted outside',cnt,'Kmax %.3f'%Kmax, flush=True)
