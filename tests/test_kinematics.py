"""Forward kinematics, model factories and the analytic DOF chain rule."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, REFERENCE, rng


def test_irb140_matches_independent_fk(oracle_mod):
    import flash
    from flash import Models
    from flash.models import _irb140_fixture
    import kinematics
    fx = _irb140_fixture()
    for ati in (False, True):
        m = Models.irb140(ati=ati)
        for seed in range(4):
            q = rng(seed).uniform(-2, 2, size=6)
            P = flash.hull_poses(m, q)
            H = kinematics.irb140_hull_poses(fx, q, ati=ati)
            assert len(P) == len(H)
            for p, h in zip(P, H):
                assert np.abs(p[:9].reshape(3, 3) - h[:3, :3]).max() < 1e-14
                assert np.abs(p[9:] - h[:3, 3]).max() < 1e-14


def test_irb140_assembles_at_zero():
    """at q = 0 the hulls stack from z = 0 to 0.809 m and
    link_6 sits at x in [0.47, 0.515]."""
    import flash
    from flash import Models
    m = Models.irb140()
    P = flash.hull_poses(m, np.zeros(6))
    w = [s.hull.vertices @ p[:9].reshape(3, 3).T + p[9:] for s, p in zip(m.surfaces, P)]
    allv = np.concatenate(w)
    assert allv[:, 2].min() == pytest.approx(0.0, abs=2e-3)
    assert allv[:, 2].max() == pytest.approx(0.809, abs=2e-3)
    assert w[6][:, 0].min() == pytest.approx(0.47, abs=2e-3)
    assert w[6][:, 0].max() == pytest.approx(0.515, abs=2e-3)
    assert repr(m) == "Manipulator with 8 links and 7 surfaces"  # examples/irb140.ipynb:261


def test_model_state_counts():
    """num_states of the reference models (src/Flash.jl:90; trace
    examples/irb_and_squishable.ipynb:480 gives 63 for the merged scene)."""
    import flash
    from flash import Models
    from flash.mechanism import QuaternionFloating
    assert flash.num_states(Models.two_link_arm()) == 2
    assert flash.num_states(Models.beanbag()) == 25
    assert flash.num_states(Models.squishable()) == 43
    assert flash.num_states(Models.irb140()) == 6
    m64 = Models.arm_grid()
    assert flash.num_states(m64) == 48 and len(m64.surfaces) == 64
    scene = Models.irb140()
    scene.mechanism.change_joint_type(1, QuaternionFloating("base"))
    Models.merge(scene, Models.squishable())
    Models.merge(scene, Models.table())
    assert flash.num_states(scene) == 63
    assert len(scene.surfaces) == 9  # examples/irb_and_squishable.ipynb:258
    assert len(Models.two_link_arm().surfaces[0].surface_points) == 40
    assert len(Models.two_link_arm().surfaces[0].skeleton_points) == 6


def test_squishable_points_on_scaled_ellipse():
    """src/models.jl:114-127: each point lies on the ellipse of radii 1.25·r."""
    from flash import Models
    s = Models.squishable().surfaces[0]
    radii = np.array([0.22, 0.20, 0.15]) * 1.25
    for _, p in s.surface_points:
        nz = np.nonzero(p)[0]
        assert len(nz) == 2
        assert (p[nz] ** 2 / radii[nz] ** 2).sum() == pytest.approx(1.0, rel=1e-12)


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference checkout absent (GPU box)")
def test_load_urdf_equals_fixture_model():
    import flash
    from flash import Models
    u = Models.load_urdf(os.path.join(REFERENCE, "examples/data/IRB140/urdf/irb_140_convhull.urdf"))
    f = Models.irb140()
    q = rng(1).uniform(-1, 1, 6)
    assert np.array_equal(flash.hull_poses(u, q), flash.hull_poses(f, q))
    for a, b in zip(u.surfaces, f.surfaces):
        assert np.array_equal(a.hull.vertices, b.hull.vertices)
        assert np.array_equal(a.hull.planes, b.hull.planes)


def _body_wrench(manip, accum):
    w = np.zeros((manip.mechanism.num_bodies, 6))
    for k, s in enumerate(manip.convex_surfaces()):
        w[s.body] += accum[1 + 6 * k: 7 + 6 * k]
    return w


@pytest.mark.parametrize("name", ["c1_irb140", "table_quat"])
def test_chain_rule_matches_finite_differences(name):
    """∂c/∂q from the per-hull wrenches == central FD of the oracle cost (golden),
    incl. the quaternion normalization projection (src/gradientdescent.jl:30)."""
    from flash import Models
    manip = {"c1_irb140": Models.irb140, "table_quat": Models.table}[name]()
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    g = manip.mechanism.config_gradient(z["q"], _body_wrench(manip, z["accum"]))
    scale = np.abs(z["dcdq_fd"]).max()
    assert np.abs(g - z["dcdq_fd"]).max() < 1e-6 * scale


def test_chain_rule_m64_subset(m64, oracle_mod):
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 3)
    pts = synthetic.depth_cloud(m64, qt, 400, seed=4)
    om = oracle_mod.OracleModel.from_manipulator(m64)
    acc = om.cost_accum(flash.hull_poses(m64, qe), pts)
    g = m64.mechanism.config_gradient(qe, _body_wrench(m64, acc))
    h = 1e-6
    for i in rng(0).choice(48, 8, replace=False):
        qp, qm = qe.copy(), qe.copy()
        qp[i] += h
        qm[i] -= h
        fd = (om.cost_accum(flash.hull_poses(m64, qp), pts)[0] - om.cost_accum(flash.hull_poses(m64, qm), pts)[0]) / (2 * h)
        assert g[i] == pytest.approx(fd, rel=1e-5, abs=1e-7)


def test_fixture_json_is_data_only():
    from flash.models import DATA_DIR
    d = json.load(open(os.path.join(DATA_DIR, "irb140.json")))
    assert set(d) == {"source", "urdf", "ati", "meshes"}
    assert len(d["urdf"]["joints"]) == 6


def test_native_forward_kinematics_matches_numpy():
    """fsdf_tree_transforms (csrc/kinematics.cpp) == the numpy level-batched FK
    to the last bits (revolute chains, fixed joints, a quaternion-floating
    base), and it rejects a tree that is not in topological order."""
    from flash import Models, _lib
    r = np.random.default_rng(41)
    for m in (Models.arm_grid(), Models.table(), Models.irb140(), Models.irb_and_squishable()[0], Models.two_link_arm()):
        mech = m.mechanism
        for _ in range(5):
            q = mech.normalize(mech.zero_configuration() + r.normal(size=mech.num_positions))
            for a, b in zip(mech.body_transform_arrays(q), mech.body_transform_arrays_numpy(q)):
                assert np.allclose(a, b, rtol=0, atol=1e-14)
    P = Models.irb140().mechanism._kinematic_plan()
    bad = P["native"][0].copy()
    bad[2] = 3  # parent after child
    out = [np.empty(len(bad) * k) for k in (9, 3, 9, 3)]
    q = np.zeros(16)
    st = _lib.load().fsdf_tree_transforms(len(bad), bad.ctypes.data, *P["native_ptrs"][1:], q.ctypes.data,
                                          *[o.ctypes.data for o in out])
    assert st == 1  # FSDF_ERR_ARG


def test_native_chain_rule_matches_numpy():
    """fsdf_config_gradient (csrc/kinematics.cpp) == the numpy chain rule
    (mechanism.config_gradient_numpy) on every model, revolute and
    quaternion-floating joints, from per-body wrenches, per-surface wrenches
    (with surfaces that carry none) and both together."""
    from flash import Models
    r = np.random.default_rng(41)
    models = [Models.irb140(), Models.arm_grid(), Models.table(), Models.beanbag(), Models.two_link_arm(False),
              Models.irb_and_squishable()[0]]
    for m in models:
        mech = m.mechanism
        nb, S = mech.num_bodies, len(m.surfaces)
        for _ in range(3):
            q = mech.zero_configuration() + r.normal(scale=0.3, size=mech.num_positions)
            bw = r.normal(size=(nb, 6))
            sb = r.integers(-1, nb, size=S).astype(np.int32)
            sw = r.normal(size=(S, 6))
            ref_b = mech.config_gradient_numpy(q, bw)
            assert np.allclose(mech.config_gradient(q, bw), ref_b, rtol=1e-12, atol=1e-12)
            sb_w = np.zeros((nb, 6))
            for k in range(S):
                if sb[k] >= 0:
                    sb_w[sb[k]] += sw[k]
            ref_s = mech.config_gradient_numpy(q, sb_w)
            assert np.allclose(mech.config_gradient(q, None, sb, sw), ref_s, rtol=1e-12, atol=1e-12)
            assert np.allclose(mech.config_gradient(q, bw, sb, sw), mech.config_gradient_numpy(q, bw + sb_w),
                               rtol=1e-12, atol=1e-12)


def test_native_chain_rule_rejects_bad_input():
    import pytest
    from flash import Models, FlashNativeError
    m = Models.irb140()
    q = m.mechanism.zero_configuration()
    with pytest.raises(FlashNativeError):
        m.mechanism.config_gradient(q, None, np.array([99], np.int32), np.zeros((1, 6)))
