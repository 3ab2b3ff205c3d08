"""Pin the CPU oracle: independent numpy formulation, closed forms, the
first-index tie rule, finite differences and the committed golden vectors."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, rng


def _poses(manip, q):
    import flash
    return flash.hull_poses(manip, manip.mechanism.normalize(q))


def test_oracle_matches_independent_numpy_irb140(irb, oracle_mod):
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(irb, 5)
    pts = synthetic.depth_cloud(irb, qt, 6000, seed=6, order="shuffled")
    om = oracle_mod.OracleModel.from_manipulator(irb)
    poses = _poses(irb, qe)
    d, k, g = om.skin(poses, pts, threads=1)
    per = np.stack([oracle_mod.numpy_hull_sdf(*om.world_hull(poses, kk), pts) for kk in range(om.K)], 1)
    assert np.abs(d - per.min(1)).max() < 1e-12
    # k* attains the minimum; first index among (numerical) ties
    assert np.abs(per[np.arange(len(pts)), k] - d).max() < 1e-12
    assert (d < 0).any() and (d > 0).any()


def test_oracle_matches_independent_numpy_m64_subset(m64, oracle_mod):
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 7)
    pts = synthetic.depth_cloud(m64, qt, 1500, seed=8, order="shuffled")
    om = oracle_mod.OracleModel.from_manipulator(m64)
    poses = _poses(m64, qe)
    d, k, _ = om.skin(poses, pts)
    per = np.stack([oracle_mod.numpy_hull_sdf(*om.world_hull(poses, kk), pts) for kk in range(om.K)], 1)
    assert np.abs(d - per.min(1)).max() < 1e-12


def test_box_closed_form(oracle_mod):
    """The table box (examples/irb_and_squishable.ipynb cell 3) is an exact box SDF."""
    from flash import Models
    from flash.geometry import quat_to_matrix
    tab = Models.table()
    r = rng(3)
    qq = r.normal(size=4)
    qq /= np.linalg.norm(qq)
    R, t = quat_to_matrix(qq), np.array([0.4, -0.2, 0.6])
    poses = np.concatenate([R.ravel(), t])[None]
    pts = t + r.uniform(-0.5, 0.5, size=(4000, 3))
    om = oracle_mod.OracleModel.from_manipulator(tab)
    d, k, g = om.skin(poses, pts, threads=1)
    loc = (pts - t) @ R  # box frame
    qd = np.abs(loc) - np.array([0.25, 0.25, 0.05])
    exact = np.linalg.norm(np.maximum(qd, 0), axis=1) + np.minimum(qd.max(1), 0)
    assert np.abs(d - exact).max() < 1e-14
    assert (k == 0).all()
    assert np.allclose(np.linalg.norm(g, axis=1), 1.0)


def test_first_index_wins_ties(irb, oracle_mod):
    """Julia's left-fold `minimum` keeps the earlier surface (src/Flash.jl:267)."""
    s = irb.surfaces[2]
    h = (s.hull.vertices, s.hull.faces, s.hull.planes)
    om = oracle_mod.OracleModel([h, h, h])
    pose = np.concatenate([np.eye(3).ravel(), np.zeros(3)])
    poses = np.stack([pose] * 3)
    pts = s.hull.vertices.mean(0) + rng(4).normal(scale=0.2, size=(500, 3))
    _, k, _ = om.skin(poses, pts)
    assert (k == 0).all()


def test_point_gradient_finite_differences(irb, oracle_mod):
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(irb, 9)
    pts = synthetic.depth_cloud(irb, qt, 3000, seed=10, order="shuffled")
    om = oracle_mod.OracleModel.from_manipulator(irb)
    poses = _poses(irb, qe)
    d, _, g = om.skin(poses, pts)
    h = 1e-7
    for ax in range(3):
        e = np.zeros(3)
        e[ax] = h
        fd = (om.skin(poses, pts + e)[0] - om.skin(poses, pts - e)[0]) / (2 * h)
        err = np.abs(fd - g[:, ax])
        assert np.median(err) < 1e-8 and np.percentile(err, 99) < 1e-6
    assert np.allclose(np.linalg.norm(g, axis=1), 1.0, atol=1e-12)


@pytest.mark.parametrize("name", ["c1_irb140", "m64_2k", "table_quat"])
def test_oracle_reproduces_golden(name, oracle_mod):
    from flash import Models
    manip = {"c1_irb140": Models.irb140, "m64_2k": Models.arm_grid, "table_quat": Models.table}[name]()
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    import flash
    # the host kinematics reproduce the stored poses (native FK vs the numpy FK
    # the vectors were generated with: same factors, last-bit summation order)
    assert np.allclose(flash.hull_poses(manip, manip.mechanism.normalize(z["q"])), z["poses"], rtol=0, atol=1e-14)
    poses = z["poses"]
    om = oracle_mod.OracleModel.from_manipulator(manip)
    d, k, g = om.skin(poses, z["points"])
    assert np.array_equal(k, z["kstar"])
    assert np.array_equal(d, z["d"])
    assert np.array_equal(g, z["grad"])
    acc = om.cost_accum(poses, z["points"])
    assert np.allclose(acc, z["accum"], rtol=1e-13, atol=1e-13)
    assert acc[0] == pytest.approx(np.dot(d, d), rel=1e-12)


def _cone_hull(n=48, radius=0.08, height=0.12):
    """n-gon base (its triangulation is coplanar) + apex of valence n > 32."""
    from flash import _lib
    a = 2 * np.pi * np.arange(n) / n
    pts = np.vstack([np.stack([radius * np.cos(a), radius * np.sin(a), np.zeros(n)], 1), [[0.0, 0.0, height]]])
    return _lib.convex_hull(pts)


def _cone_cloud(r, n):
    """points over the apex (its normal cone: the walk's fan test exceeds 32
    faces), above and below the coplanar base facets, and around."""
    apex = np.array([0.0, 0.0, 0.12])
    up = apex + np.abs(r.normal(size=(n // 3, 3))) * [0.01, 0.01, 0.05] * r.choice([-1, 1], size=(n // 3, 3)) * [1, 1, 0] \
        + [0, 0, 0.02]
    base = np.stack([r.uniform(-0.07, 0.07, n // 3), r.uniform(-0.07, 0.07, n // 3), r.normal(scale=0.01, size=n // 3)], 1)
    rest = r.normal(size=(n - 2 * (n // 3), 3)) * 0.1
    return np.vstack([up, base, rest])


def test_oracle_matches_numpy_on_high_valence_cone(oracle_mod):
    """The descent walk's fallbacks (fan > 32 faces -> exhaustive scan) and the
    coplanar base still give the exact distance (independent numpy, 1e-12)."""
    v, f, p = _cone_hull()
    assert len(f) >= 90
    om = oracle_mod.OracleModel([(v, f, p)])
    pose = np.array([[1.0, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0]])
    pts = _cone_cloud(rng(31), 3000)
    d, k, g = om.skin(pose, pts)
    ref = oracle_mod.numpy_hull_sdf(*om.world_hull(pose, 0), pts)
    assert np.abs(d - ref).max() < 1e-12
    assert np.allclose(np.linalg.norm(g, axis=1), 1.0, atol=1e-12)


def test_oracle_matches_independent_numpy_m64_large(m64, oracle_mod):
    """40,000 shuffled M64 points (all 64 hulls in play): the C restatement ==
    the independent numpy polytope SDF (its own pruning, no shared code) to
    1e-12, and k* is a minimiser."""
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 21)
    pts = synthetic.depth_cloud(m64, qt, 40000, seed=22, order="shuffled")
    om = oracle_mod.OracleModel.from_manipulator(m64)
    poses = _poses(m64, qe)
    d, k, _ = om.skin(poses, pts)
    nd, mins = oracle_mod.numpy_scene_sdf(om, poses, pts)
    assert np.abs(d - nd).max() < 1e-12
    assert mins[np.arange(len(pts)), k].all()
    assert len(np.unique(k)) >= 48  # the arms' link hulls all win somewhere


@pytest.mark.parametrize("scene", ["m64", "c5"])
def test_oracle_culled_equals_brute_force(m64, oracle_mod, scene):
    """The culled CPU leg (bench cpu_baseline) returns the brute-force minimum
    bit for bit (ties to the smaller k), hull-only and with an RBF skin."""
    from flash import synthetic
    if scene == "m64":
        qt, qe = synthetic.perturbed_configuration(m64, 23)
        pts = synthetic.depth_cloud(m64, qt, 30000, seed=24, order="shuffled")
        om = oracle_mod.OracleModel.from_manipulator(m64)
        poses, rows = _poses(m64, qe), None
    else:
        from flash import Models
        z = np.load(os.path.join(GOLDEN, "c5_scene.npz"))
        om = oracle_mod.OracleModel.from_manipulator(Models.irb_and_squishable()[0])
        pts, poses, rows = z["points"], z["poses"], z["rbf_rows"]
    a = om.skin(poses, pts, rbf_rows=rows)
    b = om.skin(poses, pts, rbf_rows=rows, culled=True)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("name", ["c1_irb140", "m64_2k", "table_quat", "c3_beanbag", "c5_scene"])
def test_oracle_fp32_instantiation(name, oracle_mod):
    """The fp32 restatement (skin_impl.h with R = float, what fp32 contexts are
    checked against bit for bit on the GPU): its world rows are the fp64 rows
    rounded once to fp32, and its per-point results stay within fp32 resolution
    of the fp64 goldens (|Δd*| < 2e-5, |Δ∇d*| small where k* agrees, k* equal
    except at near-ties)."""
    from flash import Models
    manip = {"c1_irb140": Models.irb140, "m64_2k": Models.arm_grid, "table_quat": Models.table,
             "c3_beanbag": Models.beanbag, "c5_scene": lambda: Models.irb_and_squishable()[0]}[name]()
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    om = oracle_mod.OracleModel.from_manipulator(manip)
    rows = z["rbf_rows"] if "rbf_rows" in z.files else None
    if om.K:
        st64, (pw, fx, vw, hs, _) = om.pose(z["poses"], rows)
        st32, (pw32, fx32, vw32, hs32, _) = om.pose(z["poses"], rows, precision=32)
        assert pw32.dtype == np.float32 and np.array_equal(pw32, pw.astype(np.float32))
        assert np.array_equal(vw32, vw.astype(np.float32))
        assert np.allclose(fx32, fx, rtol=0, atol=1e-5 * max(1.0, np.abs(fx).max()))
    d, k, g = om.skin(z["poses"], z["points"], rbf_rows=rows, precision=32)
    same = k == z["kstar"]
    assert same.mean() > 0.995
    assert np.abs(d - z["d"]).max() < 2e-5 * max(1.0, np.abs(z["d"]).max())
    assert np.median(np.abs(g - z["grad"])[same]) < 1e-4
    # determinism and the fp32 grid: every value is an fp32 number
    assert np.array_equal(d.astype(np.float32).astype(np.float64), d)
    d2, k2, g2 = om.skin(z["poses"], z["points"], rbf_rows=rows, precision=32, threads=1)
    assert np.array_equal(d2, d) and np.array_equal(k2, k) and np.array_equal(g2, g)
