"""RBF interpolating skins (src/Flash.jl:207-213): the C oracle vs the numpy
restatement, the reference's KAT (test/runtests.jl:17), and the adjoint
cost gradient through the weight solve vs finite differences."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, rng


def _model(name):
    from flash import Models
    if name == "scene":
        return Models.irb_and_squishable()
    m = {"beanbag": Models.beanbag, "squishable": Models.squishable, "two_link_arm": Models.two_link_arm}[name]()
    import flash
    x0 = np.zeros(flash.num_states(m))
    x0[:m.mechanism.num_positions] = m.mechanism.zero_configuration()
    return m, x0


def _state(m, x):
    nq = m.mechanism.num_positions
    return m.mechanism.normalize(x[:nq]), np.asarray(x[nq:], np.float64)


def _oracle_inputs(m, x):
    import flash
    from flash import rbf as host_rbf
    q, dd = _state(m, x)
    solves = host_rbf.solve(m, q, dd)
    return flash.core.surface_poses(m, q), host_rbf.rows(solves), solves


def test_beanbag_kat(oracle_mod):
    """@test isapprox(skin(SVector(100.0, 0, 0)), 99.0, rtol=2e-2) (test/runtests.jl:17)."""
    m, x0 = _model("beanbag")
    poses, rows, _ = _oracle_inputs(m, x0)
    om = oracle_mod.OracleModel.from_manipulator(m)
    d, k, _ = om.skin(poses, np.array([[100.0, 0, 0]]), rbf_rows=rows)
    assert d[0] == pytest.approx(99.0, rel=2e-2)
    assert d[0] == pytest.approx(98.893, abs=1e-3)
    # interpolation: surface points at 0, the skeleton (origin) at -1 before normalization
    import rbf
    C = rows[:-1, :3]
    f, _, _ = rbf.field(C, np.concatenate([rows[:-1, 3], rows[-1]]), C)
    assert np.allclose(f, [0, 0, 0, 0, 0, 0, -1], atol=1e-12)


@pytest.mark.parametrize("name", ["beanbag", "squishable", "two_link_arm"])
def test_c_oracle_matches_numpy_rbf(name, oracle_mod):
    import rbf
    m, x0 = _model(name)
    x = x0.copy()
    r = rng(3)
    nq = m.mechanism.num_positions
    x[nq:] = 0.05 * r.normal(size=len(x) - nq)
    poses, rows, solves = _oracle_inputs(m, x)
    pts = solves[0].centres.mean(0) + r.normal(scale=0.6, size=(2000, 3))
    om = oracle_mod.OracleModel.from_manipulator(m)
    d, k, g = om.skin(poses, pts, rbf_rows=rows)
    s, gs = rbf.skin(solves[0].centres, solves[0].u, pts)
    assert np.abs(d - s).max() < 1e-9 * max(1, np.abs(s).max())
    assert np.abs(g - gs).max() < 1e-7
    assert (k == 0).all()


@pytest.mark.parametrize("name", ["beanbag", "squishable", "scene"])
def test_rbf_chain_rule_matches_finite_differences(name, oracle_mod):
    """Analytic ∂c/∂x (RBF adjoint + weight-solve backsolve + hull wrenches +
    quaternion projection + regularizer) == central FD of the oracle cost."""
    import flash
    from flash.gradientdescent import gradient_from_accum
    m, x0 = _model(name)
    r = rng(7)
    x = x0.copy()
    nq = m.mechanism.num_positions
    x[:nq] += 0.05 * r.normal(size=nq)
    x[nq:] = 0.03 * r.normal(size=len(x) - nq)
    poses, rows, solves = _oracle_inputs(m, x)
    centre = np.concatenate([s.centres for s in solves]).mean(0)
    pts = centre + r.normal(scale=0.3, size=(300, 3))
    om = oracle_mod.OracleModel.from_manipulator(m)

    def cost(xx):
        p_, rw, _ = _oracle_inputs(m, xx)
        return om.cost_accum(p_, pts, rbf_rows=rw)[0] + 10 * np.dot(xx[nq:], xx[nq:])

    acc = om.cost_accum(poses, pts, rbf_rows=rows)
    g = gradient_from_accum(m, x, acc, solves, 10)
    h = 1e-6
    idx = r.choice(len(x), size=min(len(x), 14), replace=False)
    for i in idx:
        xp, xm = x.copy(), x.copy()
        xp[i] += h
        xm[i] -= h
        fd = (cost(xp) - cost(xm)) / (2 * h)
        assert g[i] == pytest.approx(fd, rel=2e-5, abs=2e-6), (i, g[i], fd)


def test_scene_structure():
    import flash
    m, x0 = _model("scene")
    assert flash.num_states(m) == 63 and len(m.surfaces) == 9
    kinds = [type(s).__name__ for s in m.surfaces]
    assert kinds[:7] == ["ConvexGeometry"] * 7 and kinds[7] == "DeformableInterpolatingSkin" and kinds[8] == "ConvexGeometry"


@pytest.mark.parametrize("name", ["c3_beanbag", "c5_scene"])
def test_oracle_reproduces_rbf_golden(name, oracle_mod):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    m, _ = _model("beanbag" if name == "c3_beanbag" else "scene")
    poses, rows, _ = _oracle_inputs(m, z["x"])
    assert np.array_equal(poses, z["poses"]) and np.array_equal(rows, z["rbf_rows"])
    om = oracle_mod.OracleModel.from_manipulator(m)
    d, k, g = om.skin(poses, z["points"], rbf_rows=rows)
    assert np.array_equal(k, z["kstar"]) and np.array_equal(d, z["d"]) and np.array_equal(g, z["grad"])
    assert np.allclose(om.cost_accum(poses, z["points"], rbf_rows=rows), z["accum"], rtol=1e-13, atol=1e-13)
