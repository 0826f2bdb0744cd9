"""Reach of the rounded triangle test (triangle.zig:48-70, f32 as the kernel and
the oracle compute it): how far outside a triangle the exact ray-plane point may
lie while the rounded barycentrics still accept the hit, against the incidence.

For each |cos theta| in 0.1 .. 1e-4: 10 x 200 000 random triangles (sizes 0.01-1,
random shapes), rays aimed at points pushed 1e-9 .. 1e-4 |ao| outside an edge
(in the triangle's plane), from 0.3 - 100 units away.  Prints the largest
accepted gap as K in  gap = K u |ao| / (sin phi |cos theta|)  (u = 2^-24, phi the
triangle's angle at a).  DESIGN.md §3 "Triangles: what the margins cover".

usage: python tools/tri_reach.py
"""
import numpy as np
f=np.float32
rng=np.random.default_rng(7)
def unit(d):
    l=np.sqrt(((d[:,0]*d[:,0]+d[:,1]*d[:,1])+d[:,2]*d[:,2]).astype(f)).astype(f)
    return (d/l[:,None]).astype(f)
def cross(u,v):
    return np.stack([(u[:,1]*v[:,2]-u[:,2]*v[:,1]),(u[:,2]*v[:,0]-u[:,0]*v[:,2]),(u[:,0]*v[:,1]-u[:,1]*v[:,0])],1).astype(f)
def dot(u,v): return ((u[:,0]*v[:,0]+u[:,1]*v[:,1])+u[:,2]*v[:,2]).astype(f)
N=200000
res={}
for cosv in [1e-1,1e-2,1e-3,1e-4]:
  worst=0
  for rep in range(10):
    # random triangles of size ~s at random positions
    s=10**rng.uniform(-2,0,N)
    A=rng.uniform(-1,1,(N,3)); B=A+s[:,None]*rng.normal(size=(N,3)); C=A+s[:,None]*rng.normal(size=(N,3))
    a=A.astype(f); b=B.astype(f); c=C.astype(f)
    e1=(b-a).astype(f); e2=(c-a).astype(f); n=cross(e1,e2)
    n64=np.cross(e1.astype(np.float64),e2.astype(np.float64)); nn=n64/np.linalg.norm(n64,axis=1)[:,None]
    sinphi=np.linalg.norm(n64,axis=1)/(np.linalg.norm(e1,axis=1)*np.linalg.norm(e2,axis=1))
    # target: a point on edge ab pushed out in-plane by g
    t_=rng.uniform(0,1,N); P=a.astype(np.float64)+t_[:,None]*e1.astype(np.float64)
    eo=np.cross(nn,e1.astype(np.float64)); eo/=np.linalg.norm(eo,axis=1)[:,None]
    sgn=np.sign((eo*(c.astype(np.float64)-a)).sum(1)); eo*=-sgn[:,None]
    dist=10**rng.uniform(-0.5,2,N)
    g=dist*10**rng.uniform(-9,-4,N)
    P=P+g[:,None]*eo
    w=rng.normal(size=(N,3)); w-=(w*nn).sum(1)[:,None]*nn; w/=np.linalg.norm(w,axis=1)[:,None]
    cs=cosv*rng.uniform(1,2,N)
    d=-(cs[:,None]*nn)+np.sqrt(1-cs**2)[:,None]*w
    o=(P-d*dist[:,None]).astype(f); d=unit(d.astype(f))
    ao=(o-a).astype(f)
    det=(-dot(d,n)).astype(f); inv=(f(1)/det).astype(f)
    dao=cross(ao,d)
    u=(dot(e2,dao)*inv).astype(f); v=(-dot(e1,dao)*inv).astype(f); t=(dot(ao,n)*inv).astype(f)
    acc=(det>=f(1e-6))&(t>f(0.001))&(u>=0)&(v>=0)&((u+v)<=1)
    aon=np.linalg.norm(ao.astype(np.float64),axis=1)
    k=(g/aon)*sinphi*cs/6e-8
    if acc.any(): worst=max(worst,k[acc].max())
  res[cosv]=worst
  print(f"cos ~{cosv}: max accepted gap/|ao| * sinphi*cos/u = {worst:.3g}", flush=True)
