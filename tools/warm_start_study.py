"""CPU study: how much of a pass a certified warm start could skip.

track! runs ~30 passes per frame over ONE cloud with slowly moving poses (the
bench alternates q and q + 1e-3). A pass at pose B may reuse the previous pass
at pose A: with k*_A(p) and a proven lower bound e2(p) <= min_{k != k*_A}
d_k(p; A), and δ_k the largest displacement of hull k's vertices from A to B
(a rigid motion moves every point of a convex hull by at most the largest
vertex displacement, and the signed distance is 1-Lipschitz under it),
    d_k(p; B) >= e2(p) - δ_k  for every k != k*_A,
so when d_{k*_A}(p; B) < e2(p) - max_k δ_k the point's winner at B is k*_A and
ONE evaluation is exact. This study measures, on the bench cloud (M64, 2^20
points, seed 1234, shuffled then Morton-ordered 64-point chunks), the share of
points and of whole chunks that resolve, with e2 the exact second-best distance
(an upper bound on what the kernel's proven bounds give) and with e2 from the
box/sphere bounds only, and the hull unions the unresolved lanes still need.
Exact distances by numpy_hull_sdf (independent of the kernel). ~3-5 min, 8 cores.
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
from tools.free_space_study import spread  # noqa: E402


def planes_of(hulls):
    out = []
    for v, f in hulls:
        a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
        n = np.cross(b - a, c - a)
        n /= np.linalg.norm(n, axis=1)[:, None]
        n *= np.sign(((a - v.mean(0)) * n).sum(1))[:, None]
        out.append(np.concatenate([n, (n * a).sum(1)[:, None]], 1))
    return out


def distances(hulls, pts):
    """[N, K] exact distances where the box/sphere bound may not exclude the hull, else that bound (-> LB)."""
    N, K = len(pts), len(hulls)
    lb = np.empty((N, K))
    ubc = np.full(N, np.inf)
    for k, (v, _) in enumerate(hulls):
        c = v.mean(0)
        vt = np.linalg.svd(v - c)[2]
        loc = (v - c) @ vt.T
        pl = (pts - c) @ vt.T
        e = np.maximum(loc.min(0) - pl, 0) + np.maximum(pl - loc.max(0), 0)
        dc = np.linalg.norm(pts - c, axis=1)
        lb[:, k] = np.maximum(np.linalg.norm(e, axis=1), dc - np.sqrt(((v - c) ** 2).sum(1).max()))
        ubc = np.minimum(ubc, dc)
    D = lb.copy()
    exact = np.zeros((N, K), bool)
    for k, ((v, f), pl) in enumerate(zip(hulls, planes_of(hulls))):
        # every hull that could be the winner or the runner-up within 5 cm
        idx = np.nonzero(lb[:, k] <= ubc + 0.05)[0]
        for s in range(0, len(idx), 20000):
            ii = idx[s:s + 20000]
            D[ii, k] = numpy_hull_sdf(v, f, pl, pts[ii])
            exact[ii, k] = True
    return D, lb, exact


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    manip = Models.arm_grid()
    q_true, q_eval = synthetic.perturbed_configuration(manip, 1234)
    pts = synthetic.depth_cloud(manip, q_true, n, seed=1234 + 17, order="shuffled")
    lo, hi = pts.min(0), pts.max(0)
    qk = np.floor((pts - lo) / (hi - lo + 1e-9) * 1023).astype(np.uint64)
    key = spread(qk[:, 0]) | (spread(qk[:, 1]) << np.uint64(1)) | (spread(qk[:, 2]) << np.uint64(2))
    pts = pts[np.argsort(key, kind="stable")]
    A = synthetic.world_hulls(manip, q_eval)
    print(f"{n} points, {len(A)} hulls")
    t = time.time()
    DA, lbA, exA = distances(A, pts)
    print(f"pose A distances {time.time() - t:.0f} s")
    kA = DA.argmin(1)
    dA = DA[np.arange(len(pts)), kA]
    for step in (1e-3, 3e-3, 1e-2):
        B = synthetic.world_hulls(manip, q_eval + step)
        delta = np.array([np.linalg.norm(vb - va, axis=1).max() for (va, _), (vb, _) in zip(A, B)])
        t = time.time()
        DB, _, _ = distances(B, pts)
        kB = DB.argmin(1)
        dkB = DB[np.arange(len(pts)), kA]  # k*_A's exact distance at B
        # (the study's box/sphere bound is >= 0, not a bound inside a hull: capped by the exact value there)
        lbv = np.minimum(lbA, DA)
        # what a pass proves: exact (or better) values for the hulls it evaluates — those whose
        # box/sphere bound lies below the winner's distance — the box/sphere bound for the rest
        kern = np.where(lbv > dA[:, None], lbv, DA)
        for e2name, src in (("exact runner-up", DA), ("pass-provable", kern), ("box/sphere only", lbv)):
            M = src.copy()
            M[np.arange(len(pts)), kA] = np.inf
            for dname, dl in (("max_k delta", np.full(len(delta), delta.max())), ("per-hull delta", delta)):
                bound = (M - dl[None, :]).min(1)  # min_{k != k*_A} (e2_k - δ_k)
                ok = dkB + 1e-9 * (1 + np.abs(dkB)) < bound
                assert np.all(kB[ok] == kA[ok]), "a resolved point changed winner"
                ch = ok.reshape(-1, 64)
                full = ch.all(1)
                # what the unresolved lanes of each chunk still need at B (exact best-first under box bounds)
                need = (DB < dkB[:, None]) & ~ok[:, None]
                u = need.reshape(-1, 64, len(A)).any(1).sum(1)
                print(f"step {step:g} rad (max δ {delta.max() * 1e3:.2f} mm) e2 = {e2name:15s} {dname:14s}: "
                      f"points resolved {ok.mean():.3f}, chunks fully resolved {full.mean():.3f}, "
                      f"unresolved-lane hull union per chunk mean {u.mean():.2f} max {u.max()}", flush=True)
        print(f"  (pose B {time.time() - t:.0f} s; winners changed A->B: {(kA != kB).mean():.4f})")


if __name__ == "__main__":
    main()
