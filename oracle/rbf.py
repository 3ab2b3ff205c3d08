"""RBF implicit skins — numpy restatement (TEST INFRASTRUCTURE ONLY).

Restates SpatialFields.InterpolatingSurface(points, values, XCubed(), true) as
used by Flash.skin for InterpolatingGeometry (src/Flash.jl:207-213):
  centres c_i = surface points (value 0) then skeleton points (value -1),
  f(x) = Σ_i w_i |x - c_i|^3 + a + b·x           (XCubed + affine polynomial)
  [A P; Pᵀ 0] [w; a; b] = [v; 0],  A_ik = |c_i - c_k|^3,  P_i = [1, c_iᵀ]
  s(x) = f(x) / |∇f(x)|                           (the field, made distance-like)
SpatialFields @06046c27 is un-vendored. This formulation satisfies the
reference's only numeric test (test/runtests.jl:17): beanbag, default state,
s(100, 0, 0) ≈ 99 (rtol 2e-2) — it gives 98.893 (the r³+affine field without
normalization gives 162.3). It does NOT reproduce the two
costs examples/manipulator.ipynb prints (:5512, :14179): 4.44× and 2.0× of
them; a bounded search over 55 formulations found none fitting all three
(tools/rbf_formulation_search.py, tests/test_notebook_pins.py). RBF parity is
therefore partial: pinned by one KAT, contradicted by two notebook outputs.

Also the cost gradient through the weight solve (adjoint): for cost
c = Σ_p s(p)^2 over the points whose nearest surface is this skin,
  λ = Σ_p 2 s ∂s/∂u   (u = [w; a; b]),   μ = M⁻ᵀ λ,
  dc/dc_j = Σ_p 2 s ∂s/∂c_j |_u  −  μᵀ (∂M/∂c_j) u.
"""
from __future__ import annotations

import numpy as np


def fit(centres, values):
    C = np.asarray(centres, np.float64)
    n = len(C)
    D = np.linalg.norm(C[:, None] - C[None], axis=-1)
    P = np.hstack([np.ones((n, 1)), C])
    M = np.block([[D ** 3, P], [P.T, np.zeros((4, 4))]])
    u = np.linalg.solve(M, np.concatenate([np.asarray(values, np.float64), np.zeros(4)]))
    return u, M


def field(centres, u, x):
    """f, ∇f, Hessian(f) at points x [m,3]."""
    C = np.asarray(centres, np.float64)
    n = len(C)
    x = np.asarray(x, np.float64).reshape(-1, 3)
    w, a, b = u[:n], u[n], u[n + 1:]
    d = x[:, None, :] - C[None]                       # [m,n,3]
    r = np.linalg.norm(d, axis=-1)                    # [m,n]
    f = (w[None] * r ** 3).sum(1) + a + x @ b
    g = (3 * (w * r)[..., None] * d).sum(1) + b
    with np.errstate(invalid="ignore", divide="ignore"):
        ddr = np.where(r[..., None, None] > 0, d[..., :, None] * d[..., None, :] / r[..., None, None], 0.0)
    H = 3 * (w[None, :, None, None] * (r[..., None, None] * np.eye(3) + ddr)).sum(1)
    return f, g, H


def skin(centres, u, x):
    """s = f/|∇f| and ∇s = ∇f/|∇f| − f H ∇f / |∇f|³."""
    f, g, H = field(centres, u, x)
    G = np.linalg.norm(g, axis=1)
    s = f / G
    grad = g / G[:, None] - (f / G ** 3)[:, None] * np.einsum("mij,mj->mi", H, g)
    return s, grad


def cost_gradient(centres, values, x):
    """(c, dc/dc_j [n,3]) for c = Σ_p s(p)^2 over points x (all assigned to this skin)."""
    C = np.asarray(centres, np.float64)
    n = len(C)
    u, M = fit(C, values)
    w, b = u[:n], u[n + 1:]
    x = np.asarray(x, np.float64).reshape(-1, 3)
    f, g, H = field(C, u, x)
    G = np.linalg.norm(g, axis=1)
    s = f / G
    dsdf = 1.0 / G                                    # [m]
    dsdg = -(f / G ** 3)[:, None] * g                 # [m,3]
    d = x[:, None, :] - C[None]
    r = np.linalg.norm(d, axis=-1)
    phi = r ** 3
    dphi = 3 * r[..., None] * d                       # ∇_x φ_i  [m,n,3]
    with np.errstate(invalid="ignore", divide="ignore"):
        ddr = np.where(r[..., None, None] > 0, d[..., :, None] * d[..., None, :] / r[..., None, None], 0.0)
    Hphi = 3 * (r[..., None, None] * np.eye(3) + ddr)  # [m,n,3,3]
    two_s = 2 * s
    lam_w = (two_s[:, None] * (dsdf[:, None] * phi + np.einsum("mj,mnj->mn", dsdg, dphi))).sum(0)
    lam_a = (two_s * dsdf).sum()
    lam_b = (two_s[:, None] * (dsdf[:, None] * x + dsdg)).sum(0)
    lam = np.concatenate([lam_w, [lam_a], lam_b])
    expl = (two_s[:, None, None] * (-w[None, :, None]) * (dsdf[:, None, None] * dphi
            + np.einsum("mj,mnjk->mnk", dsdg, Hphi))).sum(0)   # [n,3]
    mu = np.linalg.solve(M.T, lam)
    mw, mb = mu[:n], mu[n + 1:]
    dcc = C[:, None, :] - C[None]                     # c_j - c_i
    rc = np.linalg.norm(dcc, axis=-1)
    gphi = 3 * rc[..., None] * dcc                    # ∇φ(c_j - c_i)  [n(j),n(i),3]
    term = (w[:, None] * np.einsum("i,jid->jd", mw, gphi)
            + mw[:, None] * np.einsum("i,jid->jd", w, gphi)
            + mw[:, None] * b[None] + w[:, None] * mb[None])
    return float((s ** 2).sum()), expl - term


def surface_centres(manip, q, deformation_data, surface):
    """World centres of an InterpolatingGeometry at configuration q (surface
    points + δ in their body frame, then skeleton points; src/Flash.jl:152-196)."""
    T = manip.mechanism.body_transforms(manip.mechanism.normalize(q))
    cs = []
    k = manip.surfaces.index(surface)
    off = 3 * sum(s.num_deformations() for s in manip.surfaces[:k])
    deform = surface.num_deformations() > 0
    for i, (body, p) in enumerate(surface.surface_points):
        loc = p + (deformation_data[off + 3 * i: off + 3 * i + 3] if deform else 0.0)
        cs.append(T[body].apply(loc[None])[0])
    for body, p in surface.skeleton_points:
        cs.append(T[body].apply(p[None])[0])
    vals = [0.0] * len(surface.surface_points) + [-1.0] * len(surface.skeleton_points)
    return np.array(cs), np.array(vals)
