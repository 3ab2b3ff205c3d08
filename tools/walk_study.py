#!/usr/bin/env python3
"""Where do the heavy chunks' descent walks come from? (CPU study)

The per-hull SDF's closest-feature search walks from the max-plane face's
closest point to the certified closest feature (kernel cert_step / oracle
skin_impl.h). A wave pays, per hull it evaluates, the LONGEST walk among its
lanes that need the hull. This study takes a cloud (M64, generator G, chunks of
64 points in Morton order as an approximation of the device's Hilbert order),
the hulls each point needs (lower bound |p - c_k| - r_k <= d*(p): what culling
cannot exclude), and reports the per-(chunk, hull) maximal walk lengths, per
chunk their sum, and how many chunks carry long walks.

    python tools/walk_study.py [--points 131072]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "point-cloud-signed-distance_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)


def morton(pts):
    lo, hi = pts.min(0), pts.max(0)
    q = np.clip(((pts - lo) / (hi - lo + 1e-12) * 1023).astype(np.int64), 0, 1023)
    key = np.zeros(len(pts), np.int64)
    for b in range(10):
        for a in range(3):
            key |= ((q[:, a] >> b) & 1) << (3 * b + a)
    return np.argsort(key, kind="stable")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=1 << 17)
    ap.add_argument("--lib", default=os.path.join(ROOT, "scratch", "libwalk.so"))
    a = ap.parse_args()
    import flash
    import oracle
    from flash import Models, synthetic
    m = Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m, 1234)
    pts = synthetic.depth_cloud(m, qt, a.points, seed=1234 + 17, order="shuffled")
    pts = np.ascontiguousarray(pts[morton(pts)])
    poses = flash.hull_poses(m, qe)
    om = oracle.OracleModel.from_manipulator(m)
    d, k, _ = om.skin(poses, pts, culled=True)
    st, keep = om.pose(poses)
    V = keep[2][:, :3].astype(np.float64)
    cen = np.stack([V[om.vert_off[h]:om.vert_off[h + 1]].mean(0) for h in range(om.K)])
    rad = np.array([np.linalg.norm(V[om.vert_off[h]:om.vert_off[h + 1]] - cen[h], axis=1).max() for h in range(om.K)])
    dist = np.linalg.norm(pts[:, None, :] - cen[None], axis=-1)
    need = (dist - rad[None]) <= d[:, None] + 1e-9
    pi, hk = np.nonzero(need)
    lib = ctypes.CDLL(a.lib)
    lib.walk_study.argtypes = [ctypes.POINTER(oracle.Posed)] + [ctypes.c_void_p] * 3 + [ctypes.c_int64] + \
        [ctypes.c_void_p] * 3
    n = len(pi)
    pi32, hk32 = pi.astype(np.int32), hk.astype(np.int32)
    dd = np.empty(n)
    steps = np.empty(n, np.int32)
    scan = np.empty(n, np.int32)
    lib.walk_study(ctypes.byref(st), pts.ctypes.data, pi32.ctypes.data, hk32.ctypes.data, n, dd.ctypes.data,
                   steps.ctypes.data, scan.ctypes.data)
    chunk = pi // 64
    nc = (len(pts) + 63) // 64
    print(f"points {len(pts)}, needed (point, hull) pairs {n} ({n / len(pts):.2f} per point)")
    print("walk steps over pairs that walk:", np.bincount(steps[steps >= 0]).tolist(), " exhaustive:", int(scan.sum()))
    # per (chunk, hull): max steps over the lanes needing it (-1 -> 0: no walk)
    key = chunk * om.K + hk
    mx = np.zeros(nc * om.K, np.int32)
    np.maximum.at(mx, key, np.maximum(steps, 0))
    ev = np.zeros(nc * om.K, bool)
    ev[key] = True
    mx = mx.reshape(nc, om.K)
    ev = ev.reshape(nc, om.K)
    evals = ev.sum(1)
    wsum = mx.sum(1)
    print("hull evaluations per chunk: mean %.2f p99 %d max %d" % (evals.mean(), np.quantile(evals, 0.99), evals.max()))
    print("sum of max walk steps per chunk: mean %.2f p99 %d max %d" % (wsum.mean(), np.quantile(wsum, 0.99),
                                                                     wsum.max()))
    top = np.argsort(-(evals * 4 + wsum))[:10]
    for c in top:
        print(f"  chunk {c}: {evals[c]} hull evaluations, per-hull max walks {mx[c][ev[c]].tolist()}")
    print("per-(chunk, hull) max walk distribution:", np.bincount(mx[ev]).tolist())


if __name__ == "__main__":
    main()
