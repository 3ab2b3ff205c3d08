#!/usr/bin/env python3
"""How often would the fp32 screen's batch certificate (sdf_kernels.hip
screen_plane_max: b2 < b1 - 2E) fail at a wider margin? (CPU study)

For 800 random 64-point chunks of the bench cloud (M64, Hilbert-like Morton
order) and every candidate hull, the exact batch maxima give b1 / b2; a wave
falls back to the full fp64 scan when any lane that needs the hull fails the
certificate. Margins: the fp32 E times 1, 8, 64, 512 and 8192 (fp16's unit
roundoff is 2^13 times fp32's). The per-lane best is approximated by the
plane-max lower bound, so the rejection share is indicative.

    python tools/screen_margin_study.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from screen_cone_study import morton3
import flash
from flash import Models, synthetic
m = Models.arm_grid()
qt, qe = synthetic.perturbed_configuration(m, 1234)
poses = flash.hull_poses(m, qe)
pts = synthetic.depth_cloud(m, qt, 1 << 18, seed=1234 + 17, order="shuffled")
pts = pts[morton3(pts)]
H=[]
for k, s in enumerate(m.surfaces):
    R = poses[k, :9].reshape(3, 3); t = poses[k, 9:]
    P = s.hull.planes; n = P[:, :3] @ R.T; d = P[:, 3] + n @ t
    V = s.hull.vertices @ R.T + t; c = V.mean(0); r = np.linalg.norm(V - c, axis=1).max()
    H.append((n, d, c, r))
C = np.stack([h[2] for h in H]); Rr = np.array([h[3] for h in H])
rng = np.random.default_rng(5); nch = len(pts)//64
chunks = rng.choice(nch, 800, replace=False)
res = {}
for fac in (1, 8, 64, 512, 8192):
    res[fac] = [0, 0, 0, 0, 0]  # evals, wave-fail, lane-fail(active), active lanes, rejected-waves
# exact best per point: approximate as min over hulls of max_f h (inside) or true dist; use max h lower bound proxy
for ci in chunks:
    p = pts[64*ci:64*ci+64]
    dc = np.linalg.norm(p[:, None, :] - C[None], axis=2); ub = dc.min(1); lb = dc - Rr[None]
    # per-hull sdf proxy: max plane value (lower bound of d) -> best proxy = min over hulls of max(maxh, lb)
    mh = np.stack([(p @ h[0].T - h[1]).max(1) for h in H], 1)
    best = np.minimum(ub, np.maximum(mh, lb).min(1))
    cand = np.nonzero((lb <= ub[:, None]).any(0))[0]
    for k in cand:
        n, d, c, r = H[k]
        need = lb[:, k] <= best + 1e-5
        if not need.any(): continue
        q = p - c
        h = p @ n.T - d
        F = h.shape[1]; nb = -(-F // 8)
        hp = np.concatenate([h, np.repeat(h[:, -1:], nb*8 - F, 1)], 1)
        bm = hp.reshape(64, nb, 8).max(2)
        b1 = bm.max(1); ib = bm.argmax(1)
        bm2 = bm.copy(); bm2[np.arange(64), ib] = -np.inf; b2 = bm2.max(1)
        E32 = 32 * 5.9604645e-8 * (np.abs(q).sum(1) + r)
        for fac in res:
            E2 = E32 * fac
            thr = best + E2
            rej = not np.any(need & ~(b1 > thr))
            rr = res[fac]; rr[0] += 1
            if rej: rr[4] += 1; continue
            safe = b2 < b1 - E2
            rr[3] += need.sum(); rr[2] += (need & ~safe).sum(); rr[1] += np.any(need & ~safe)
for fac, rr in res.items():
    print(fac, dict(evals=rr[0], rejected=rr[4]/rr[0], wave_fail_of_nonrej=rr[1]/max(rr[0]-rr[4],1), lane_fail=rr[2]/max(rr[3],1)))
