"""CPU: the native RBF weight solve and adjoint (fsdf_rbf_solve /
fsdf_rbf_adjoint, csrc/rbf_host.cpp) against their numpy twins (flash/rbf.py
solve / chain) on the reference's RBF scenes: beanbag (C3), squishable,
two_link_arm and irb_and_squishable (C5). No device is used."""
import ctypes

import numpy as np
import pytest


def _scenes():
    from flash import Models
    return {"beanbag": Models.beanbag(), "squishable": Models.squishable(), "two_link_arm": Models.two_link_arm(),
            "irb_and_squishable": Models.irb_and_squishable()[0]}


def _native_solve(lib, C, v):
    n = len(C)
    m = n + 4
    u, lu, piv = np.empty(m), np.empty(m * m), np.empty(m, np.int32)
    C = np.ascontiguousarray(C, np.float64)
    v = np.ascontiguousarray(v, np.float64)
    assert lib.fsdf_rbf_solve(n, C.ctypes.data, v.ctypes.data, u.ctypes.data, lu.ctypes.data, piv.ctypes.data) == 0
    return u, lu, piv


@pytest.mark.parametrize("name", ["beanbag", "squishable", "two_link_arm", "irb_and_squishable"])
def test_native_rbf_solve_and_adjoint(name):
    from flash import _lib, rbf
    lib = _lib.load()
    m = _scenes()[name]
    mech = m.mechanism
    rng = np.random.default_rng(7)
    q = mech.normalize(mech.zero_configuration() + 0.05 * rng.normal(size=mech.num_positions))
    nd = m.num_deformations()
    delta = 0.01 * rng.normal(size=3 * nd)
    solves = rbf.solve(m, q, delta)
    assert solves
    blocks = []
    for r in solves:
        n = r.n
        s = m.surfaces[r.surface]
        v = np.concatenate([np.zeros(len(s.surface_points)), -np.ones(len(s.skeleton_points))])
        u, lu, piv = _native_solve(lib, r.centres, v)
        assert np.allclose(u, r.u, rtol=1e-10, atol=1e-10 * np.abs(r.u).max())
        # adjoint: a random accumulator block through both chains
        block = rng.normal(size=4 * n + 4)
        blocks.append(block)
        G = np.empty(3 * n)
        work = np.empty(n + 4)
        rows_c = np.ascontiguousarray(r.centres)
        assert lib.fsdf_rbf_adjoint(n, rows_c.ctypes.data, u.ctypes.data, lu.ctypes.data, piv.ctypes.data,
                                    block.ctypes.data, G.ctypes.data, work.ctypes.data) == 0
        G = G.reshape(n, 3)
        # numpy chain of this surface alone -> wrenches / ∂c/∂δ; rebuild them from G
        w_np, gd_np = rbf.chain(m, q, [r], block, nd)
        T = mech.body_transforms(q)
        w_nat = np.zeros_like(w_np)
        gd_nat = np.zeros_like(gd_np)
        np.add.at(w_nat[:, :3], r.bodies, -G)
        np.add.at(w_nat[:, 3:], r.bodies, -np.cross(r.centres, G))
        for j in range(n):
            if r.deform_rows[j] >= 0:
                gd_nat[3 * r.deform_rows[j]: 3 * r.deform_rows[j] + 3] = T[r.bodies[j]].R.T @ G[j]
        scale = max(np.abs(w_np).max(), 1e-300)
        assert np.allclose(w_nat, w_np, rtol=1e-9, atol=1e-9 * scale)
        if nd:
            assert np.allclose(gd_nat, gd_np, rtol=1e-9, atol=1e-9 * max(np.abs(gd_np).max(), 1e-300))


def test_native_rbf_solve_degenerate():
    """Coincident centres make the system singular: FSDF_ERR_DEGENERATE, no NaNs returned as success."""
    from flash import _lib
    lib = _lib.load()
    C = np.zeros((5, 3))
    v = np.zeros(5)
    m = 9
    u, lu, piv = np.empty(m), np.empty(m * m), np.empty(m, np.int32)
    st = lib.fsdf_rbf_solve(5, C.ctypes.data, v.ctypes.data, u.ctypes.data, lu.ctypes.data, piv.ctypes.data)
    assert _lib.STATUS_NAMES[st] == "FSDF_ERR_DEGENERATE"
    st = lib.fsdf_rbf_solve(0, C.ctypes.data, v.ctypes.data, u.ctypes.data, lu.ctypes.data, piv.ctypes.data)
    assert _lib.STATUS_NAMES[st] == "FSDF_ERR_ARG"
