#!/usr/bin/env python3
"""How much of the pass's fp32 screen could a per-batch bound skip? (CPU study,
round 5; the screen is 31 % of wave time at 2^20, profiles/r05/wave_times.)

For 1,500 random 64-point chunks of the 2^20 bench cloud (ordered by a Morton
key, an approximation of the device's Hilbert sort) and every hull that is the
nearest one for some lane of the chunk (those hulls are screened in full), each
8-face batch gets the bound  UB = a.q + r|q| - min_f d'_f  (a the batch's mean
normal, r its chord radius, q = p - c); the batch is skippable for the wave when
UB < the lane's final maximum for every lane (optimistic: the real loop knows
only the maximum so far). Batches of the hull's face order vs batches of faces
sorted along an octahedral Morton curve of their normals. Uses the CPU oracle
for the nearest hulls (test infrastructure only).

    python tools/screen_skip_study.py   ->  profiles/r05/screen_skip_study.txt
"""
import sys, numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'point-cloud-signed-distance_amd')); sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import flash
from flash import Models, synthetic
import oracle
m=Models.arm_grid()
qt,qe=synthetic.perturbed_configuration(m,1234)
poses=flash.hull_poses(m,qe)
pts=synthetic.depth_cloud(m,qt,1<<20,seed=1234+17,order="shuffled")
# Hilbert-ish order: sort by morton of quantized coords (approximation of the device sort)
lo=pts.min(0); hi=pts.max(0); q=((pts-lo)/(hi-lo+1e-12)*1023).astype(np.int64)
def spread(x):
    x=(x|(x<<16))&0x030000FF; x=(x|(x<<8))&0x0300F00F; x=(x|(x<<4))&0x030C30C3; x=(x|(x<<2))&0x09249249; return x
key=spread(q[:,0])|(spread(q[:,1])<<1)|(spread(q[:,2])<<2)
pts=pts[np.argsort(key,kind='stable')]
om=oracle.OracleModel.from_manipulator(m)
rng=np.random.default_rng(0)
chunks=rng.choice(len(pts)//64, 1500, replace=False)
sel=np.concatenate([np.arange(c*64,c*64+64) for c in chunks])
d,k,g=om.skin(poses, pts[sel])
P=np.asarray(poses).reshape(len(m.surfaces),12) if np.asarray(poses).ndim==1 else np.asarray(poses)
res={'orig':[0,0],'sorted':[0,0]}
def hull_world(si):
    s=m.surfaces[si]; R=P[si,:9].reshape(3,3); t=P[si,9:]
    pl=np.asarray(s.hull.planes); n=pl[:,:3]@R.T; dd=pl[:,3]+n@t
    v=np.asarray(s.hull.vertices)@R.T+t
    return n,dd,v
def order_sorted(n):
    # greedy: sort normals by octahedral-map morton
    o=n/np.abs(n).sum(1,keepdims=True)
    u=np.where(o[:,2]>=0,o[:,0],(1-np.abs(o[:,1]))*np.sign(o[:,0]+1e-30))
    w=np.where(o[:,2]>=0,o[:,1],(1-np.abs(o[:,0]))*np.sign(o[:,1]+1e-30))
    qu=((u+1)*511).astype(np.int64); qw=((w+1)*511).astype(np.int64)
    kk=spread(qu)|(spread(qw)<<1)
    return np.argsort(kk,kind='stable')
for ci in range(len(chunks)):
    idx=slice(ci*64,ci*64+64)
    P64=pts[sel][idx]; ks=np.unique(k[idx])
    for si in ks:
        n,dd,v=hull_world(si)
        c=v.mean(0)
        qv=P64-c; nq=np.linalg.norm(qv,axis=1)
        h=qv@n.T-(dd-n@c)  # [64, nf]
        b1=h.max(1)
        for name,perm in (('orig',np.arange(len(n))),('sorted',order_sorted(n))):
            nb=(len(n)+7)//8
            for b in range(nb):
                f=perm[8*b:8*b+8]
                a=n[f].sum(0); a/=np.linalg.norm(a)
                r=np.linalg.norm(n[f]-a,axis=1).max()
                dmin=(dd[f]-n[f]@c).min()
                ub=qv@a+r*nq-dmin
                res[name][1]+=1
                if np.all(ub < b1-1e-6): res[name][0]+=1
for kk, v in res.items():
    print(f'{kk:7s} batches skippable {v[0] / v[1]:.3f} of {v[1]} (wave level, final maximum)')
