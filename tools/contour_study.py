#!/usr/bin/env python3
"""Which conventions reproduce the reference's contour-mesh counts
(tests/golden/contour_pins.json)? CPU study, output in profiles/r04/contour_study.txt.

1. Grid conventions x level tests (tests/contour_mesh.py variants) for the
   three pinned calls, scene SDF from the C oracle (== the GPU path).
2. RBF formulations (kernels x polynomial tails x normalizations of
   tools/rbf_formulation_search.py) for the squishable zero set (294 / 584)
   and for the C5 scene (4,494 / 8,912), hulls from the oracle.
3. (needs /root/reference) An emulation of EnhancedGJK @404de6a9's gjk!
   (src/Flash.jl:238-249) for the IRB140 call: NeighborMesh hill-climbing
   support over the STL's vertex adjacency (src/models.jl:152), a 4-point
   simplex with the closest-point weights, atol 1e-6, max 100 iterations,
   one CollisionCache per surface warm-started across the grid sweep in
   GeometryTypes' loop order (z fastest) or x fastest; the support by brute
   force as the control. The package is un-vendored: this is a restatement
   of its published design, not of its code.

    python tools/contour_study.py [--no-gjk]
"""
import itertools
import math
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "point-cloud-signed-distance_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)

import contour_mesh as cm  # noqa: E402

MESHES = "/root/reference/examples/data/IRB140/urdf/meshes/"
LINKS = ["base_link", "link1", "link2", "link3", "link4", "link5", "link6"]


def oracle_parts(m, x):
    import flash
    import oracle
    from flash import rbf as host_rbf
    nq = m.mechanism.num_positions
    q = m.mechanism.normalize(x[:nq])
    om = oracle.OracleModel.from_manipulator(m)
    poses = flash.core.surface_poses(m, q)
    rows = host_rbf.rows(host_rbf.solve(m, q, x[nq:])) if m.has_rbf() else None
    return lambda pts: om.skin(poses, pts, rbf_rows=rows)[0]


def section_grids(out):
    out.append("## 1. grid conventions x level test (oracle SDF); reference in brackets")
    for name in ("irb140", "irb_and_squishable", "squishable"):
        m, x, lb, ub, iso, res = cm.pinned_case(name)
        res_ = cm.count_variants(oracle_parts(m, x), lb, ub, iso, res)
        out.append(f"{name} [{cm.EXPECTED[name]}]")
        for (v, mode), (V, F, shape) in res_.items():
            mark = "  <== reference" if (V, F) == cm.EXPECTED[name] else ""
            out.append(f"  {v:9s} {mode:6s} grid {shape}: {V} / {F}   chi {V - F // 2}{mark}")


def section_rbf(out):
    import rbf_formulation_search as rs
    from flash import rbf as host_rbf
    from flash.core import ConvexGeometry, Manipulator
    out.append("## 2. RBF formulations (kernel, tail, normalization)")
    for name in ("squishable", "irb_and_squishable"):
        m, x, lb, ub, iso, res = cm.pinned_case(name)
        nq = m.mechanism.num_positions
        C = host_rbf.solve(m, m.mechanism.normalize(x[:nq]), x[nq:])[0].centres
        v = np.concatenate([np.zeros(len(C) - 1), [-1.0]])
        axes = cm.grid_axes(lb, ub, res)
        P = cm.grid_points(axes)
        hulls = [s for s in m.surfaces if isinstance(s, ConvexGeometry)]
        dh = oracle_parts(Manipulator(m.mechanism, hulls), x[:nq])(P) if hulls else np.full(len(P), np.inf)
        out.append(f"{name} [{cm.EXPECTED[name]}]")
        for kn, (phi, dphi) in rs.KERNELS.items():
            for poly in ("affine", "const", "none"):
                w, a, b = rs.fit(C, v, phi, poly)[:3]
                f, g = rs.field(C, w, a, b, dphi, phi, P)
                G = np.linalg.norm(g, axis=1)
                norms = rs.NORMS.items() if hulls else [("sign of f", lambda f, G: f)]
                for nn, fn in norms:
                    V, F = cm.mesh_counts(cm.to_volume(np.minimum(dh, fn(f, G)), axes) < iso)
                    mark = "  <== reference" if (V, F) == cm.EXPECTED[name] else ""
                    out.append(f"  {kn:10s} {poly:7s} {nn:24s} {V} / {F}{mark}")


# ---- EnhancedGJK emulation ------------------------------------------------------------
def stl_mesh(name):
    b = open(MESHES + name + "_chull.stl", "rb").read()
    n = struct.unpack("<I", b[80:84])[0]
    tri = np.frombuffer(b[84:84 + 50 * n], dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
    verts, idx, faces = [], {}, []
    for t in tri["v"].astype(np.float64):
        f = []
        for p in t:
            key = tuple(p)
            if key not in idx:
                idx[key] = len(verts)
                verts.append(tuple(float(c) for c in p))
            f.append(idx[key])
        faces.append(f)
    nb = [set() for _ in verts]
    for f in faces:
        for i, j in itertools.permutations(range(3), 2):
            if f[i] != f[j]:
                nb[f[i]].add(f[j])
    return verts, [sorted(s) for s in nb]


def closest_weights(S):
    """Barycentric weights of the point of conv(S) nearest the origin (every
    sub-simplex enumerated; positive weights required)."""
    best = None
    for k in range(1, len(S) + 1):
        for sub in itertools.combinations(range(len(S)), k):
            P = np.array([S[i] for i in sub])
            if k == 1:
                lam = np.array([1.0])
            else:
                A = (P[1:] - P[0]).T
                G = A.T @ A
                if abs(np.linalg.det(G)) < 1e-30:
                    continue
                mu = np.linalg.solve(G, -A.T @ P[0])
                lam = np.concatenate([[1 - mu.sum()], mu])
                if lam.min() <= 0:
                    continue
            y = lam @ P
            if best is None or y @ y < best[0]:
                w = np.zeros(len(S))
                w[list(sub)] = lam
                best = (y @ y, w)
    return best[1]


def gjk_surface(verts, nbrs, R, t, brute, atol=1e-6, max_iter=100):
    V = np.asarray(verts)
    W = V @ R.T + t
    cache = [0, 0, 0, 0]  # any_inside: the mesh's first vertex

    def climb(start, d):
        s = V @ d
        cur = start
        while True:
            nxt = max(nbrs[cur], key=lambda i: s[i])
            if s[nxt] > s[cur]:
                cur = nxt
            else:
                return cur

    def f(p):
        S = [W[i] - p for i in cache]
        it = 1
        while True:
            w = closest_weights(S)
            j = int(np.argmin(w))
            if w[j] > 0:
                return -1.0  # in collision
            best = w @ np.array(S)
            d = -best
            dA = R.T @ d
            if brute:
                v = int(np.argmax(V @ dA))
            else:
                v = climb(max(cache, key=lambda i: V[i] @ dA), dA)
            imp = W[v] - p
            if imp @ d <= best @ d + atol or it >= max_iter:
                return math.sqrt(best @ best)
            cache[j] = v
            S[j] = imp
            it += 1
    return f


def section_gjk(out):
    import flash
    from flash import Models
    out.append("## 3. EnhancedGJK emulation, IRB140 call [(2226, 4460)]")
    m = Models.irb140()
    poses = flash.core.surface_poses(m, m.mechanism.zero_configuration())
    lb, ub, iso, res = cm.REGIONS["irb140"]
    axes = cm.grid_axes(lb, ub, res)
    nx, ny, nz = (len(a) for a in axes)
    meshes = [stl_mesh(n) for n in LINKS]
    for order, brute in (("z fastest", False), ("x fastest", False), ("z fastest", True)):
        surfs = [gjk_surface(v, nb, p[:9].reshape(3, 3), p[9:], brute) for (v, nb), p in zip(meshes, poses)]
        sweep = itertools.product(range(nx), range(ny), range(nz)) if order == "z fastest" else \
            ((x, y, z) for z in range(nz) for y in range(ny) for x in range(nx))
        vol = np.empty((nx, ny, nz))
        for x, y, z in sweep:
            p = np.array([axes[0][x], axes[1][y], axes[2][z]])
            vol[x, y, z] = min(s(p) for s in surfs)
        V, F = cm.mesh_counts(vol - iso < 0.0)
        out.append(f"  support {'brute force' if brute else 'hill climbing'}, sweep {order}: {V} / {F}   chi {V - F // 2}")


def main():
    out = ["# contour-mesh count study (tools/contour_study.py)"]
    section_grids(out)
    section_rbf(out)
    if "--no-gjk" not in sys.argv and os.path.isdir(MESHES):
        section_gjk(out)
    print("\n".join(out))


if __name__ == "__main__":
    main()
