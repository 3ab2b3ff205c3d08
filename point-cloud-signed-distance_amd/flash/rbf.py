"""RBF interpolating skins: the host work around the GPU pass.

Flash.skin for an InterpolatingGeometry (src/Flash.jl:207-213) builds
SpatialFields.InterpolatingSurface(points, values, XCubed(), true) from the
world-frame surface points (value 0, each displaced by its deformation δ_i in
its body frame, src/Flash.jl:158-168) and skeleton points (value -1). Per pass
the host
  1. places the centres (forward kinematics + δ) and solves the (n+4)² system
     [A P; Pᵀ 0][w; a; b] = [v; 0], A_ik = |c_i - c_k|^3, P_i = [1, c_iᵀ];
  2. ships rows (c_i, w_i) and (a, b) to the device (fsdf_set_rbf_params);
and after the pass turns the RBF adjoint block of the accumulator
(λ = Σ 2s ∂s/∂(w,a,b), E_i = Σ 2s ∂s/∂c_i) into ∂c/∂c_j through the solve
(μ = M⁻ᵀλ), then into body wrenches (∂c/∂q) and ∂c/∂δ. The field value on the
device is s = f/|∇f| (matches the KAT test/runtests.jl:17; diverges from the
examples/manipulator.ipynb costs by 4.44x / 2.0x — DESIGN.md §2).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .core import InterpolatingGeometry, Manipulator


@dataclass
class RbfSolve:
    surface: int                  # index in Manipulator.surfaces
    centres: np.ndarray           # [n,3] world
    bodies: np.ndarray            # [n] body of each centre
    deform_rows: np.ndarray       # [n] row of deformation_data/3, -1 if none
    M: np.ndarray                 # [(n+4),(n+4)]
    u: np.ndarray                 # [n+4] = w, a, b

    @property
    def n(self) -> int:
        return len(self.centres)


def rbf_surfaces(manip: Manipulator):
    return [i for i, s in enumerate(manip.surfaces) if isinstance(s, InterpolatingGeometry)]


def solve(manip: Manipulator, q: np.ndarray, deformation_data: np.ndarray) -> list[RbfSolve]:
    """Centres and coefficients of every RBF surface at (q, δ); q normalized by the caller."""
    T = manip.mechanism.body_transforms(q)
    out = []
    row0 = 0
    for i, s in enumerate(manip.surfaces):
        nd = s.num_deformations()
        if not isinstance(s, InterpolatingGeometry):
            row0 += nd
            continue
        cs, bodies, drows = [], [], []
        for j, (b, p) in enumerate(s.surface_points):
            loc = p + deformation_data[3 * (row0 + j): 3 * (row0 + j) + 3] if nd else p
            cs.append(T[b].R @ loc + T[b].t)
            bodies.append(b)
            drows.append(row0 + j if nd else -1)
        for b, p in s.skeleton_points:
            cs.append(T[b].R @ p + T[b].t)
            bodies.append(b)
            drows.append(-1)
        C = np.array(cs)
        n = len(C)
        v = np.concatenate([np.zeros(len(s.surface_points)), -np.ones(len(s.skeleton_points))])
        D = np.linalg.norm(C[:, None] - C[None], axis=-1)
        P = np.hstack([np.ones((n, 1)), C])
        M = np.block([[D ** 3, P], [P.T, np.zeros((4, 4))]])
        u = np.linalg.solve(M, np.concatenate([v, np.zeros(4)]))
        out.append(RbfSolve(i, C, np.array(bodies), np.array(drows), M, u))
        row0 += nd
    return out


def rows(solves: list[RbfSolve]) -> np.ndarray:
    """Device rows: per surface n rows (c, w) then (a, b)."""
    parts = []
    for r in solves:
        n = r.n
        parts.append(np.hstack([r.centres, r.u[:n, None]]))
        parts.append(r.u[n:][None])
    return np.ascontiguousarray(np.concatenate(parts))


def chain(manip: Manipulator, q: np.ndarray, solves: list[RbfSolve], block: np.ndarray, n_deform: int):
    """RBF accumulator block -> (body wrenches [nb,6] in the δc = -(ω·M + v·F)
    convention, ∂c/∂δ [3·n_deform]); q normalized as for `solve`."""
    T = manip.mechanism.body_transforms(q)
    nb = manip.mechanism.num_bodies
    wrench = np.zeros((nb, 6))
    gdef = np.zeros(3 * n_deform)
    off = 0
    for r in solves:
        n = r.n
        acc = block[off: off + 4 * n + 4]
        off += 4 * n + 4
        lam, E = acc[: n + 4], acc[n + 4:].reshape(n, 3)
        mu = np.linalg.solve(r.M.T, lam)
        w, b = r.u[:n], r.u[n + 1:]
        mw, mb = mu[:n], mu[n + 1:]
        d = r.centres[:, None, :] - r.centres[None]          # c_j - c_i
        gphi = 3 * np.linalg.norm(d, axis=-1)[..., None] * d  # ∇φ(c_j - c_i)
        term = (w[:, None] * np.einsum("i,jid->jd", mw, gphi) + mw[:, None] * np.einsum("i,jid->jd", w, gphi)
                + mw[:, None] * b[None] + w[:, None] * mb[None])
        G = E - term                                           # ∂c/∂c_j (world)
        np.add.at(wrench[:, :3], r.bodies, -G)
        np.add.at(wrench[:, 3:], r.bodies, -np.cross(r.centres, G))
        for j in range(n):
            if r.deform_rows[j] >= 0:                          # c_j = R_B (p_j + δ_j) + t_B
                row = r.deform_rows[j]
                gdef[3 * row: 3 * row + 3] = T[r.bodies[j]].R.T @ G[j]
    return wrench, gdef
