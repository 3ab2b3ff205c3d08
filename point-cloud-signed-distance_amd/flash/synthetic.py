"""Seeded synthetic depth clouds (SURVEY.md §8d generator G).

G(model, q, N, seed):
  85 %  uniform-by-area samples on the world-frame hull faces + N(0, σ=5 mm) noise
  10 %  uniform in the model's world bounding box expanded by 0.25 m
   5 %  strictly inside a hull (random convex combination of 4 hull vertices)
The reference makes its clouds by raycasting the SDF (src/depthsensors.jl:88-118)
and reads real ones in sensor (raster) order (src/depthdata.jl:19-30); the
default `order="raster"` emits points in a top-down scan order, `"shuffled"`
is the adversarial order for wave coherence.
"""
from __future__ import annotations

import numpy as np

from .core import Manipulator, hull_poses


def world_hulls(manip: Manipulator, q):
    poses = hull_poses(manip, manip.mechanism.normalize(q))
    out = []
    for s, p in zip(manip.convex_surfaces(), poses):
        R, t = p[:9].reshape(3, 3), p[9:]
        out.append((s.hull.vertices @ R.T + t, s.hull.faces))
    return out


def depth_cloud(manip: Manipulator, q, n: int, seed: int = 0, order: str = "raster", sigma: float = 0.005,
                pad: float = 0.25, frac_surface: float = 0.85, frac_box: float = 0.10) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    hulls = world_hulls(manip, q)
    n_surf = int(round(frac_surface * n))
    n_box = int(round(frac_box * n))
    n_in = n - n_surf - n_box
    # surface samples, area-weighted over every triangle of every hull
    tris = np.concatenate([v[f] for v, f in hulls])  # [T,3,3]
    area = 0.5 * np.linalg.norm(np.cross(tris[:, 1] - tris[:, 0], tris[:, 2] - tris[:, 0]), axis=1)
    ti = rng.choice(len(tris), size=n_surf, p=area / area.sum())
    u, v = rng.random(n_surf), rng.random(n_surf)
    flip = u + v > 1
    u[flip], v[flip] = 1 - u[flip], 1 - v[flip]
    t = tris[ti]
    surf = t[:, 0] + u[:, None] * (t[:, 1] - t[:, 0]) + v[:, None] * (t[:, 2] - t[:, 0])
    surf += rng.normal(0.0, sigma, size=surf.shape)
    allv = np.concatenate([v for v, _ in hulls])
    lo, hi = allv.min(0) - pad, allv.max(0) + pad
    box = lo + rng.random((n_box, 3)) * (hi - lo)
    hk = rng.integers(0, len(hulls), size=n_in)
    inside = np.empty((n_in, 3))
    for k in range(len(hulls)):
        sel = np.nonzero(hk == k)[0]
        if len(sel) == 0:
            continue
        verts = hulls[k][0]
        idx = rng.integers(0, len(verts), size=(len(sel), 4))
        w = rng.dirichlet(np.ones(4), size=len(sel))
        inside[sel] = np.einsum("nj,njc->nc", w, verts[idx])
    pts = np.concatenate([surf, box, inside])
    if order == "shuffled":
        pts = pts[rng.permutation(len(pts))]
    elif order == "raster":
        cell = 0.005
        row = np.floor((pts[:, 1] - lo[1]) / cell).astype(np.int64)
        col = np.floor((pts[:, 0] - lo[0]) / cell).astype(np.int64)
        pts = pts[np.lexsort((pts[:, 2], col, row))]
    elif order != "generated":
        raise ValueError(order)
    return np.ascontiguousarray(pts)


def perturbed_configuration(manip: Manipulator, seed: int, sigma: float = 0.05):
    """(q_true, q_eval): q_true ~ U(joint limits) (seed), q_eval = q_true + N(0, σ) (seed+1)."""
    from .models import joint_limits
    lo, hi = joint_limits(manip)
    rng = np.random.Generator(np.random.PCG64(seed))
    q = manip.mechanism.zero_configuration()
    rev = np.isfinite(lo) & np.isfinite(hi)
    q[rev] = lo[rev] + rng.random(rev.sum()) * (hi[rev] - lo[rev])
    rng2 = np.random.Generator(np.random.PCG64(seed + 1))
    q_eval = q.copy()
    q_eval[rev] += rng2.normal(0.0, sigma, size=rev.sum())
    return q, q_eval


def skin_cloud(manip: Manipulator, x, n: int, seed: int = 0, near: float = 0.85, sigma: float = 0.005,
               pad: float = 0.3) -> np.ndarray:
    """Synthetic cloud for scenes with RBF skins (BASELINE configs 3 and 5):
    uniform samples of the centres' box padded by `pad`; the first `near`
    fraction is projected onto the scene's zero set (five Newton steps
    p <- p - d*(p) grad d*(p) through the device skin) and jittered by
    N(0, sigma). x is the full state vector (q then deformations)."""
    from . import core
    from . import rbf as host_rbf
    st = core.ManipulatorState(manip)
    nq = manip.mechanism.num_positions
    st.q[:] = x[:nq]
    st.deformation_data[:] = x[nq:]
    f = core.skin(st)
    r = np.random.Generator(np.random.PCG64(seed))
    solves = host_rbf.solve(manip, manip.mechanism.normalize(np.asarray(x[:nq], np.float64)), np.asarray(x[nq:]))
    C = np.concatenate([s.centres for s in solves])
    lo, hi = C.min(0) - pad, C.max(0) + pad
    pts = lo + r.random((n, 3)) * (hi - lo)
    k = int(near * n)
    for _ in range(5):
        d, _, g = f.evaluate(pts[:k])
        pts[:k] -= d[:, None] * g
    pts[:k] += r.normal(scale=sigma, size=(k, 3))
    return pts


def c5_cloud(manip: Manipulator, x, n: int, real_xyz: np.ndarray, seed: int = 0, sigma: float = 0.002,
             frac_real: float = 0.5) -> np.ndarray:
    """BASELINE config 5's cloud: the reference's recorded
    Kinect cloud of the squishable (examples/data/squishable_unsquished_xyzrgb.txt,
    25,571 points, read by examples/squishable.ipynb cell 4 / src/depthdata.jl:19-30)
    tiled to `frac_real`·n points — copy j > 0 jittered by N(0, sigma) — plus
    generator G (depth_cloud) on the scene's hulls at the configuration x[:nq]
    for the rest, shuffled together. `real_xyz` is the [N,3] position array
    (tests/golden/squishable_unsquished.npz)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    real = np.asarray(real_xyz, np.float64)
    n_real = int(round(frac_real * n))
    reps = -(-n_real // len(real))
    tiled = np.tile(real, (reps, 1))[:n_real].copy()
    tiled[len(real):] += rng.normal(0.0, sigma, size=(n_real - min(n_real, len(real)), 3))
    nq = manip.mechanism.num_positions
    arm = depth_cloud(manip, np.asarray(x[:nq], np.float64), n - n_real, seed=seed + 1, order="generated")
    pts = np.concatenate([tiled, arm])
    return np.ascontiguousarray(pts[rng.permutation(len(pts))])
