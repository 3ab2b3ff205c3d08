"""CPU study of why the heaviest pass waves stay heavy.

On the bench's M64 cloud (bench.py defaults: arm_grid, seed 0, 2^20 points) it
computes, for every point, the exact distance to every hull whose box/sphere
lower bound does not already exclude it (numpy_hull_sdf, independent of the
kernel), and then counts the hulls an exact best-first search must evaluate:
hull k is needed for point p when LB_k(p) < d*(p) (or k attains d*). It reports
the union of needed hulls per chunk (what one wave evaluates) for
  * Morton-ordered 64-point chunks (the kernel's Hilbert chunks' stand-in),
  * chunks grouped by winning hull first (regrouping),
  * 32/16/8-point sub-chunks and single points,
under the kernel's lower bounds (oriented box ∪ sphere, here a PCA box) and
under hypothetical per-hull distance grids with 5 / 10 mm half-diagonal cells
(LB = d − 2·hd).  Runs ~3 minutes on 8 cores; prints a text report.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))
sys.path.insert(0, ROOT)
from flash import Models, synthetic  # noqa: E402
from oracle.oracle import numpy_hull_sdf  # noqa: E402


def spread(x):
    x = x & 0x3FF
    x = (x | (x << 16)) & 0x30000FF
    x = (x | (x << 8)) & 0x300F00F
    x = (x | (x << 4)) & 0x30C30C3
    return (x | (x << 2)) & 0x9249249


def main():
    manip = Models.arm_grid()
    q_true, q_eval = synthetic.perturbed_configuration(manip, 0)
    pts = synthetic.depth_cloud(manip, q_true, 1 << 20, seed=17)
    hulls = synthetic.world_hulls(manip, q_eval)
    K = len(hulls)
    planes = []
    for v, f in hulls:
        a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
        n = np.cross(b - a, c - a)
        n /= np.linalg.norm(n, axis=1)[:, None]
        n *= np.sign(((a - v.mean(0)) * n).sum(1))[:, None]
        planes.append(np.concatenate([n, (n * a).sum(1)[:, None]], 1))
    lo, hi = pts.min(0), pts.max(0)
    qk = np.floor((pts - lo) / (hi - lo + 1e-9) * 1023).astype(np.uint64)
    key = spread(qk[:, 0]) | (spread(qk[:, 1]) << np.uint64(1)) | (spread(qk[:, 2]) << np.uint64(2))
    o = np.argsort(key, kind="stable")
    pts, key = pts[o], key[o]
    N = len(pts)
    box_lb = np.empty((N, K), np.float64)
    ubc = np.full(N, np.inf)
    for k, (v, _) in enumerate(hulls):
        c = v.mean(0)
        vt = np.linalg.svd(v - c)[2]
        loc = (v - c) @ vt.T
        pl = (pts - c) @ vt.T
        e = np.maximum(loc.min(0) - pl, 0) + np.maximum(pl - loc.max(0), 0)
        dc = np.linalg.norm(pts - c, axis=1)
        box_lb[:, k] = np.maximum(np.linalg.norm(e, axis=1), dc - np.sqrt(((v - c) ** 2).sum(1).max()))
        ubc = np.minimum(ubc, dc)  # the vertex centroid lies inside the hull: d_k <= |p - c_k|
    D = np.full((N, K), np.inf)
    t = time.time()
    for k, ((v, f), pl) in enumerate(zip(hulls, planes)):
        idx = np.nonzero(box_lb[:, k] <= ubc + 1e-9)[0]
        for s in range(0, len(idx), 20000):
            ii = idx[s:s + 20000]
            D[ii, k] = numpy_hull_sdf(v, f, pl, pts[ii])
    dstar = D.min(1)
    kstar = D.argmin(1)
    print(f"exact distances: {np.isfinite(D).sum()} point-hull pairs in {time.time() - t:.0f} s")
    grouped = np.lexsort((key, kstar))
    for name, lb in (("box", box_lb), ("grid 5 mm", np.maximum(box_lb, D - 0.01)),
                     ("grid 10 mm", np.maximum(box_lb, D - 0.02))):
        need = (lb < dstar[:, None] - 1e-12) | (D <= dstar[:, None])
        per = need.sum(1)
        print(f"[{name}] hulls needed per point: mean {per.mean():.2f}, max {per.max()}, "
              f"points needing >= 6: {(per >= 6).sum()}")
        for order_name, perm in (("Morton", None), ("winner-grouped", grouped)):
            nd = need if perm is None else need[perm]
            for sub in (64, 32, 16, 8):
                u = nd.reshape(-1, sub, K).any(1).sum(1)
                top = np.sort(u)[::-1][:8].tolist()
                print(f"  {order_name:15s} {sub:2d}-point chunks: union mean {u.mean():.2f} max {u.max()} "
                      f"top {top} p99.9 {np.percentile(u, 99.9):.0f}")


if __name__ == "__main__":
    main()
