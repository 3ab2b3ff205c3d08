#!/usr/bin/env python3
"""Host-code AddressSanitizer run (CPU only; tools/asan_host.sh builds the
instrumented libraries and runs this under LD_PRELOAD=libasan).

Exercises every host C/C++ path the tests reach, through ASan builds:
  * csrc/hull.cpp (fsdf_convex_hull): the IRB140 meshes, random clouds, and
    degenerate inputs (duplicates, coplanar and collinear sets, < 4 points);
  * csrc/kinematics.cpp (fsdf_tree_transforms, fsdf_config_gradient): FK and
    the chain rule of every model at random q;
  * csrc/rbf_host.cpp (fsdf_rbf_solve, fsdf_rbf_adjoint): the weight solve and
    its adjoint of every RBF scene, and a singular system;
  * oracle/flash_oracle.c: skin (brute force and culled), cost/accumulators,
    the RBF skin and the raycaster on samples of each BASELINE scene.
GPU entry points are not loaded (the instrumented host library has none)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "point-cloud-signed-distance_amd"), os.path.join(ROOT, "oracle")]


def main():
    from flash import _lib as L
    host = ctypes.CDLL(os.environ["ASAN_HOST_LIB"])
    for name in ("fsdf_convex_hull", "fsdf_tree_transforms", "fsdf_config_gradient", "fsdf_rbf_solve",
                 "fsdf_rbf_adjoint"):
        res, args = L._PROTOS[name]
        getattr(host, name).restype = res
        getattr(host, name).argtypes = args
    L._lib = host  # the host package's native calls go to the instrumented build
    import oracle
    oracle.LIB = os.environ["ASAN_ORACLE_LIB"]
    import flash
    from flash import Models, synthetic
    rng = np.random.default_rng(3)
    n_hulls = 0
    for n in (4, 5, 8, 20, 100, 1000):
        for _ in range(5):
            L.convex_hull(rng.normal(size=(n, 3)))
            n_hulls += 1
    cube = np.array([[x, y, z] for x in (0, 1) for y in (0, 1) for z in (0, 1)], float)
    for pts in (np.concatenate([cube] * 3), np.concatenate([cube, rng.uniform(0, 1, (50, 3))])):
        L.convex_hull(pts)
        n_hulls += 1
    for bad in (np.zeros((3, 3)), rng.normal(size=(30, 2)) @ np.array([[1, 0, 0], [0, 1, 0]], float),
                np.outer(np.arange(10.0), [1, 2, 3])):
        try:
            L.convex_hull(bad)
        except L.FlashNativeError:
            pass
        n_hulls += 1
    scenes = [Models.irb140(), Models.arm_grid(), Models.table(), Models.beanbag(), Models.two_link_arm(False)]
    m5 = Models.irb_and_squishable()[0]
    scenes.append(m5)
    n_eval = 0
    for m in scenes:
        om = oracle.OracleModel.from_manipulator(m)
        for seed in range(3):
            x = m.mechanism.zero_configuration() + rng.normal(scale=0.2, size=m.mechanism.num_positions)
            q = m.mechanism.normalize(x)
            from flash.core import surface_poses
            poses = surface_poses(m, q)
            rows = None
            if m.has_rbf():
                from flash import rbf as host_rbf
                rows = host_rbf.rows(host_rbf.solve(m, q, np.zeros(flash.num_states(m) - m.mechanism.num_positions)))
            pts = rng.normal(scale=0.6, size=(3000, 3)) + np.array([0.2, 0.0, 0.5])
            om.skin(poses, pts, rbf_rows=rows)
            om.skin(poses, pts, rbf_rows=rows, culled=True)
            if not m.has_rbf():
                om.cost_accum(poses, pts)
            # chain rule: random surface wrenches (+ the RBF adjoint's body wrenches)
            sb = [s.body if hasattr(s, "hull") else -1 for s in m.surfaces]
            m.mechanism.config_gradient(x, rng.normal(size=(m.mechanism.num_bodies, 6)), sb,
                                        rng.normal(size=(len(sb), 6)))
            if m.has_rbf():
                from flash import rbf as host_rbf
                for r in host_rbf.solve(m, q, np.zeros(flash.num_states(m) - m.mechanism.num_positions)):
                    n, mm = r.n, r.n + 4
                    C = np.ascontiguousarray(r.centres)
                    sf = m.surfaces[r.surface]
                    v = np.r_[np.zeros(len(sf.surface_points)), -np.ones(len(sf.skeleton_points))]
                    u, lu, piv = np.empty(mm), np.empty(mm * mm), np.empty(mm, np.int32)
                    assert host.fsdf_rbf_solve(n, C.ctypes.data, v.ctypes.data, u.ctypes.data, lu.ctypes.data,
                                               piv.ctypes.data) == 0
                    block, G, work = rng.normal(size=4 * n + 4), np.empty(3 * n), np.empty(mm)
                    assert host.fsdf_rbf_adjoint(n, C.ctypes.data, u.ctypes.data, lu.ctypes.data, piv.ctypes.data,
                                                 block.ctypes.data, G.ctypes.data, work.ctypes.data) == 0
                z, z4 = np.zeros((4, 3)), np.zeros(4)  # coincident centres: singular
                u, lu, piv = np.empty(8), np.empty(64), np.empty(8, np.int32)
                assert host.fsdf_rbf_solve(4, z.ctypes.data, z4.ctypes.data, u.ctypes.data, lu.ctypes.data,
                                           piv.ctypes.data) != 0
            rays = rng.normal(size=(200, 3))
            rays /= np.linalg.norm(rays, axis=1, keepdims=True)
            om.raycast(poses, np.array([0.0, 0.0, 3.0]), rays, rbf_rows=rows)
            n_eval += 1
    print(f"asan host run clean: {n_hulls} hulls, {len(scenes)} models x 3 configurations "
          f"(FK, chain rule, RBF solve / adjoint, oracle skin / culled / accumulators / raycast)")


if __name__ == "__main__":
    main()
