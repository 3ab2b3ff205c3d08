"""GPU: fsdf_value_and_gradient — the whole CostFunctor iteration in one
native call (host FK, surface poses, RBF weight solve, one pass, chain rule) —
against the composed host path (Python poses, fsdf_eval, the numpy chain
rule), on revolute (IRB140, M64) and quaternion-floating (the table, an
un-normalized quaternion) mechanisms. The native poses are summed in another
order than numpy's, so the pass sees poses equal to ~1 ulp: cost within
1e-12, gradient within 1e-9 relative."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,n", [("irb140", 60000), ("arm_grid", 60000), ("table", 20000),
                                    ("irb140", 150000), ("arm_grid", 150000)])
def test_fused_matches_composed(name, n):
    """(150,000 points: inside the planned pass's window — its per-chunk rows and
    two-level reduction write the accumulator straight into pinned host memory)"""
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
        pts = qt[4:7] + np.random.default_rng(3).uniform(-0.4, 0.4, size=(n, 3))
    else:
        qt, x = synthetic.perturbed_configuration(m, 17)
        pts = synthetic.depth_cloud(m, qt, n, seed=18)
    cf = CostFunctor(m, pts)
    assert cf._native
    c1, g1 = cf.value_and_gradient(x)
    assert cf.ctx.pass_kernel_name().startswith("planned_pass_kernel") == (n > 98304)
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


def _rbf_scene(name):
    from flash import Models
    return Models.beanbag() if name == "c3_beanbag" else Models.irb_and_squishable()[0]


@pytest.mark.parametrize("name", ["c3_beanbag", "c5_scene"])
def test_fused_rbf_matches_golden_and_composed(name):
    """RBF scenes (BASELINE configs 3, 5): the native iteration (centres from FK
    + δ, LU weight solve, rows, pass, RBF adjoint, chain rule, regularizer)
    against the oracle's golden dc/dx and against the composed host path
    (numpy solve/chain on the same context). The two weight solves (LAPACK vs
    the native LU) agree to ~1e-13, so the passes see rows equal to a few ulp."""
    import os
    from conftest import GOLDEN
    from flash.gradientdescent import CostFunctor
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    m = _rbf_scene(name)
    nq = m.mechanism.num_positions
    cf = CostFunctor(m, z["points"])
    assert cf._native
    x = np.asarray(z["x"], np.float64)
    c1, g1 = cf.value_and_gradient(x)
    reg = 10.0 * float(np.dot(x[nq:], x[nq:]))
    assert c1 == pytest.approx(float(z["accum"][0]) + reg, rel=1e-9)
    assert np.allclose(g1, z["dcdx"], rtol=1e-7, atol=1e-7 * np.abs(z["dcdx"]).max())
    # deformations away from the golden state, vs the composed host path
    x2 = x.copy()
    x2[nq:] += 0.01 * np.random.default_rng(5).normal(size=len(x) - nq)
    for xx in (x, x2):
        c1, g1 = cf.value_and_gradient(xx)
        cf._native = False
        c0, g0 = cf.value_and_gradient(xx)
        cf._native = True
        assert c1 == pytest.approx(c0, rel=1e-10)
        assert np.allclose(g1, g0, rtol=1e-8, atol=1e-8 * np.abs(g0).max())
    c2, g2 = cf.value_and_gradient(x2)
    assert c2 == c1 and np.array_equal(g2, g1)


def test_fused_rbf_needs_declared_centres():
    """An RBF scene without fsdf_set_rbf_centres is refused (FSDF_ERR_STATE)."""
    from flash import Models, FlashNativeError, _lib
    m = Models.beanbag()
    c = _lib.Context(device=0)
    c.set_surfaces([("rbf", len(s.surface_points) + len(s.skeleton_points)) for s in m.surfaces])
    c.set_points(np.random.default_rng(1).normal(size=(100, 3)))
    mech = m.mechanism
    c.set_mechanism(mech, [-1] * len(m.surfaces), [np.eye(3)] * len(m.surfaces), [np.zeros(3)] * len(m.surfaces))
    with pytest.raises(FlashNativeError):
        c.value_and_gradient(mech.zero_configuration())
    c.close()


def test_state_split_and_validation():
    """fsdf_eval_state_device + fsdf_state_gradient (the sharded path's halves)
    equal fsdf_value_and_gradient, also pipelined (two passes in flight, the
    chain rule of the first after the second was enqueued: its host FK / RBF
    solve is redone, bit for bit); deformation rows beyond
    fsdf_set_deformations are refused."""
    import os
    import torch
    from conftest import GOLDEN
    from flash import FlashNativeError
    from flash.gradientdescent import CostFunctor
    z = np.load(os.path.join(GOLDEN, "c5_scene.npz"))
    from flash import Models
    m = Models.irb_and_squishable()[0]
    cf = CostFunctor(m, z["points"])
    x = np.asarray(z["x"], np.float64)
    c1, g1 = cf.value_and_gradient(x)
    ctx = cf.ctx
    acc = torch.zeros(ctx.accum_len, dtype=torch.float64, device="cuda:0")
    ctx.set_stream(torch.cuda.current_stream(0).cuda_stream)
    ctx.eval_state_device(x, acc.data_ptr())
    c2, g2 = ctx.state_gradient(x, acc.cpu().numpy())
    ctx.set_stream(None)
    assert c2 == c1 and np.array_equal(g2, g1)
    x2 = x + 1e-3
    c4, g4 = cf.value_and_gradient(x2)
    acc2 = torch.zeros_like(acc)
    ctx.set_stream(torch.cuda.current_stream(0).cuda_stream)
    ctx.eval_state_device(x, acc.data_ptr())
    ctx.eval_state_device(x2, acc2.data_ptr())
    c5, g5 = ctx.state_gradient(x, acc.cpu().numpy())
    c6, g6 = ctx.state_gradient(x2, acc2.cpu().numpy())
    ctx.set_stream(None)
    assert c5 == c1 and np.array_equal(g5, g1)
    assert c6 == c4 and np.array_equal(g6, g4)
    with pytest.raises(FlashNativeError):  # not the x of either of the context's last two passes
        ctx.state_gradient(x + 0.5, acc.cpu().numpy())
    ctx.set_deformations(1, 10.0)  # the squishable's 13 deformable points need 13 rows
    with pytest.raises(FlashNativeError):
        ctx.value_and_gradient(x[:m.mechanism.num_positions + 3])
    ctx._mechanism_of = None  # the functor re-registers before its next call
    c3, g3 = cf.value_and_gradient(x)
    assert c3 == c1 and np.array_equal(g3, g1)


def test_fused_rbf_fp32_context():
    """An fp32 context (BASELINE configs 3/5 run f32): the native iteration
    uploads the rows through the f32 conversion and matches the composed host
    path on the same context (same f32 pass, f64 chain rule)."""
    import os
    from conftest import GOLDEN
    from flash import Models
    from flash.gradientdescent import CostFunctor
    z = np.load(os.path.join(GOLDEN, "c5_scene.npz"))
    m = Models.irb_and_squishable()[0]
    cf = CostFunctor(m, z["points"], precision=32)
    assert cf._native
    x = np.asarray(z["x"], np.float64)
    c1, g1 = cf.value_and_gradient(x)
    cf._native = False
    c0, g0 = cf.value_and_gradient(x)
    cf._native = True
    assert c1 == pytest.approx(c0, rel=1e-6)
    assert np.allclose(g1, g0, rtol=1e-5, atol=1e-5 * np.abs(g0).max())
    # and close to the f64 golden gradient (f32 pass)
    assert np.allclose(g1, z["dcdx"], rtol=2e-2, atol=2e-2 * np.abs(z["dcdx"]).max())


def test_set_surfaces_drops_the_mechanism():
    """fsdf_set_surfaces after fsdf_set_mechanism: the mechanism's surface
    bodies, frames and pose scratch refer to the old surface list, so the
    library drops the mechanism and native iterations fail with
    FSDF_ERR_STATE until it is registered again (it used to index
    the old per-surface vectors past their end). Python-side, the context
    forgets its registration, so CostFunctor re-registers by itself."""
    from flash import Models, synthetic, _lib
    from flash.gradientdescent import CostFunctor
    m = Models.irb140()
    big = Models.arm_grid()
    qt, x = synthetic.perturbed_configuration(m, 5)
    pts = synthetic.depth_cloud(m, qt, 4096, seed=6)
    cf = CostFunctor(m, pts)
    cf.value_and_gradient(x)
    ctx = cf.ctx
    # a larger surface list on the same context (more surfaces than the mechanism knows)
    ctx.set_surfaces([("hull", (s.hull.vertices, s.hull.faces, s.hull.planes)) for s in big.surfaces])
    assert ctx._mechanism_of is None
    with pytest.raises(_lib.FlashNativeError) as e:
        ctx.value_and_gradient(x)
    assert "mechanism" in str(e.value)
    with pytest.raises(ValueError):
        ctx.value_and_gradient(np.zeros(3))  # short x is refused before the C call


@pytest.mark.parametrize("name", ["arm_grid", "c5_scene"])
def test_sharded_functor_inflight_same_bits(name):
    """ShardedCostFunctor(inflight=2): every other launch on a second context
    over the shard, on a stream of its own, so value_and_gradient_many's
    consecutive passes run together — the same bits as one pass at a time
    (one rank, no collective; rigid M64 at a planned-window size and the RBF
    C5 scene)."""
    from flash import Models, synthetic
    from flash.distributed import ShardedCostFunctor
    if name == "c5_scene":
        m = _rbf_scene(name)
        import os
        from conftest import GOLDEN
        z = np.load(os.path.join(GOLDEN, name + ".npz"))
        pts, x0 = z["points"], np.asarray(z["x"], np.float64)
    else:
        m = getattr(Models, name)()
        qt, x0 = synthetic.perturbed_configuration(m, 31)
        pts = synthetic.depth_cloud(m, qt, 150000, seed=32)
    xs = [x0 + 1e-3 * i for i in range(6)]
    one = ShardedCostFunctor(m, pts)
    want = [one.value_and_gradient(x) for x in xs]
    two = ShardedCostFunctor(m, pts, inflight=2)
    assert len(two.ctxs) == 2
    got = two.value_and_gradient_many(xs)
    for (c0, g0), (c1, g1) in zip(want, got):
        assert c1 == c0 and np.array_equal(g1, g0)
