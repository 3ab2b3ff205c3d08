"""GPU: fsdf_value_and_gradient — the whole CostFunctor iteration of a rigid
scene in one native call (host FK, surface poses, one pass, chain rule) —
against the composed host path (Python poses, fsdf_eval, the numpy chain
rule), on revolute (IRB140, M64) and quaternion-floating (the table, an
un-normalized quaternion) mechanisms. The native poses are summed in another
order than numpy's, so the pass sees poses equal to ~1 ulp: cost within
1e-12, gradient within 1e-9 relative."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["irb140", "arm_grid", "table"])
def test_fused_matches_composed(name):
    import flash
    from flash import Models, synthetic, _lib
    from flash.core import surface_poses
    from flash.gradientdescent import CostFunctor
    m = getattr(Models, name)()
    mech = m.mechanism
    if name == "table":
        x = mech.zero_configuration()
        x[:4] = [0.9, 0.2, -0.3, 0.1]  # un-normalized quaternion
        x[4:7] = [0.05, -0.02, 0.01]
        qt = mech.normalize(x)
        pts = qt[4:7] + np.random.default_rng(3).uniform(-0.4, 0.4, size=(20000, 3))
    else:
        qt, x = synthetic.perturbed_configuration(m, 17)
        pts = synthetic.depth_cloud(m, qt, 60000, seed=18)
    cf = CostFunctor(m, pts)
    assert cf._native
    c1, g1 = cf.value_and_gradient(x)
    # composed host path on the same context
    poses = surface_poses(m, mech.normalize(x))
    c0, acc, _ = cf.ctx.eval(poses)
    surf = m.surfaces
    bw = np.zeros((mech.num_bodies, 6))
    for k, s in enumerate(surf):
        bw[s.body] += acc[1 + 6 * k:7 + 6 * k]
    g0 = mech.config_gradient_numpy(np.asarray(x, np.float64), bw)
    assert c1 == pytest.approx(c0, rel=1e-12)
    assert np.allclose(g1, g0, rtol=1e-9, atol=1e-9 * np.abs(g0).max())
    # repeated calls are deterministic and follow x
    c2, g2 = cf.value_and_gradient(x)
    assert c2 == c1 and np.array_equal(g2, g1)
    c3, _ = cf.value_and_gradient(np.asarray(x) + 1e-3)
    assert c3 != c1


def test_fused_refuses_rbf_scene():
    """RBF scenes keep the host weight solve: the context refuses the fused call."""
    import flash
    from flash import Models, FlashNativeError
    from flash.gradientdescent import CostFunctor
    m = Models.beanbag()
    cf = CostFunctor(m, np.random.default_rng(1).normal(size=(100, 3)))
    assert not cf._native
    c, g = cf.value_and_gradient(np.zeros(flash.num_states(m)) + np.r_[1.0, np.zeros(flash.num_states(m) - 1)])
    assert np.isfinite(c) and np.isfinite(g).all()
    ctx = cf.ctx
    mech = m.mechanism
    ctx.set_mechanism(mech, [0] * len(m.surfaces), [np.eye(3)] * len(m.surfaces), [np.zeros(3)] * len(m.surfaces))
    with pytest.raises(FlashNativeError):
        ctx.value_and_gradient(mech.zero_configuration())
