"""GPU: the device solver loop of fsdf_descend (csrc/solver.hip) and the
library's own regroup on the track! path.

estimate_state's iteration (src/tracking.jl:8-27: c/N, NaiveSolver rate /
max_step / iteration_limit, src/tracking.jl:12-15) runs for rigid scenes with
every step on the device — FK, chain rule, the clipped step — from the pass's
accumulator, and must give the host loop's x, value and iteration count bit
for bit (the same per-body arithmetic, kin_impl.h). The regroup the track!
path now applies by itself (fsdf_set_regroup AUTO) changes sums in rounding
only: x within 1e-9 relative, the same iteration count."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _floating_irb_table():
    """IRB140 on a QuaternionFloating base plus the floating table box
    (examples/irb_and_squishable.ipynb cells 3-4 without the RBF skin): a
    rigid scene with quaternion joints."""
    import flash
    from flash import Models
    from flash.mechanism import QuaternionFloating
    m = Models.irb140()
    m.mechanism.change_joint_type(1, QuaternionFloating("base_link_floating"))
    Models.merge(m, Models.table())
    x0 = np.array(m.mechanism.zero_configuration(), np.float64)
    for name, t in (("base_link", (0.0, 0.0, 0.75)), ("table_body", (0.4, 0.0, 0.6))):
        r = m.mechanism.q_range(m.mechanism.body_index(name))
        x0[r.start + 4: r.start + 7] = t
    assert flash.num_states(m) == len(x0) == 20
    return m, x0


def _scene(name, n):
    import flash
    from flash import Models, synthetic
    if name == "floating":
        m, x_true = _floating_irb_table()
        rng = np.random.default_rng(5)
        x_true[7:13] = rng.uniform(-0.4, 0.4, 6)
        pts = synthetic.depth_cloud(m, x_true, n, seed=6, frac_box=0.1, frac_surface=0.9, sigma=0.002)
        x0 = x_true.copy()
        x0[7:13] += 0.04
        x0[4:7] += 0.01
        x0[13:17] = [0.999, 0.02, -0.01, 0.03]  # table orientation off identity, not normalized
        return m, pts, x0
    m = Models.irb140() if name == "irb140" else Models.arm_grid()
    q_true, q_eval = synthetic.perturbed_configuration(m, 41)
    pts = synthetic.depth_cloud(m, q_true, n, seed=42)
    return m, pts, np.asarray(q_eval, np.float64)


@pytest.mark.parametrize("name,n", [("irb140", 6000), ("m64", 1 << 16), ("floating", 20000), ("m64", 300000)])
def test_device_loop_bit_identical_to_host_loop(name, n):
    """Device solver loop == host loop over fsdf_value_and_gradient: x, f and
    the iteration count bit for bit, with preconditioning divisors, under a
    convergence tolerance that stops early and one that never does."""
    from flash.gradientdescent import CostFunctor
    m, pts, x0 = _scene(name, n)
    cf = CostFunctor(m, pts)
    ctx = cf.ctx
    nx = len(x0)
    div = np.linspace(1.0, 1.5, nx)
    for tol, limit, rate, div_ in ((0.0, 7, 0.5, None), (1e-3, 40, 2.0, div), (1e30, 5, 1.0, None)):
        res = []
        for dev_loop in (False, "require"):  # (require: fails rather than fall back to the host loop)
            ctx.set_solver(dev_loop)
            res.append(cf.descend(x0, limit, rate, 0.05, tol, div_, float(len(pts))))
        (xa, fa, ia), (xb, fb, ib) = res
        assert ia == ib, (ia, ib)
        assert fa == fb, (fa, fb)
        assert np.array_equal(xa, xb), np.abs(xa - xb).max()
        if tol == 0.0:
            assert ib == limit
        if tol == 1e30:  # converged at the first evaluation: x untouched, f = c/N there
            assert ib == 1 and np.array_equal(xb, x0)
            c, _ = cf.value_and_gradient(x0)
            assert fb == c / len(pts)
    ctx.set_solver(True)  # (the default)


def test_device_loop_refuses_bad_configuration():
    """A zero quaternion fails FK on the device as on the host (FSDF_ERR_ARG),
    and the context stays usable."""
    from flash._lib import FlashNativeError
    from flash.gradientdescent import CostFunctor
    m, pts, x0 = _scene("floating", 4000)
    cf = CostFunctor(m, pts)
    bad = x0.copy()
    bad[13:17] = 0.0
    for dev_loop in (False, "require"):
        cf.ctx.set_solver(dev_loop)
        with pytest.raises(FlashNativeError):
            cf.descend(bad, 3, 1.0, 0.05, 0.0, None, float(len(pts)))
    x, f, its = cf.descend(x0, 2, 1.0, 0.05, 0.0, None, float(len(pts)))
    assert its == 2 and np.isfinite(f)


@pytest.mark.parametrize("name", ["irb140", "m64"])
def test_auto_regroup_descend_matches_unregrouped(name):
    """A 2^20-point frame runs one wave per chunk, so fsdf_descend regroups the
    cloud after its first pass by itself (fsdf_set_regroup AUTO, the default):
    the resident order changes, and the frame ends at the unregrouped frame's x
    within 1e-9 relative with the same iteration count (sums differ in rounding
    only). Estimate_state's default solver (rate 0.1, max_step 0.5, 30
    iterations, src/tracking.jl:12-15; tolerance 1e-3) on c/N."""
    from flash import _lib
    m, pts, x0 = _scene(name, 1 << 20)
    surf = m.surfaces
    ctx = m.engine(0, 64)
    ctx.set_mechanism(m.mechanism, [s.body for s in surf], [s.frame.R for s in surf], [s.frame.t for s in surf])
    ctx.set_solver("require")
    out = {}
    for auto in (False, True):
        ctx.set_regroup(auto)
        ctx.set_points(pts)
        perm0 = ctx.permutation()
        x, f, its = ctx.descend(x0, 30, 0.1, 0.5, 1e-3, None, float(len(pts)))
        perm1 = ctx.permutation()
        out[auto] = (x, f, its, not np.array_equal(perm0, perm1))
        assert np.array_equal(np.sort(perm1), np.arange(len(pts)))
    (xa, fa, ia, ra), (xb, fb, ib, rb) = out[False], out[True]
    assert not ra and rb, "the auto regroup did not run (or ran with regroup off)"
    assert ia == ib
    scale = np.maximum(np.abs(xa), 1.0)
    assert np.all(np.abs(xa - xb) <= 1e-9 * scale), np.abs(xa - xb).max()
    assert abs(fa - fb) <= 1e-9 * abs(fa)
    ctx.set_regroup(True)
    # the explicit rule: a context that already regrouped this cloud refuses a second auto regroup
    assert ctx.regroup_auto() is False


def test_regrouped_range_refuses_chunk_costs():
    """fsdf_chunk_costs of a ranged cloud after a regroup: FSDF_ERR_STATE (its
    chunks are no longer the whole cloud's Hilbert chunks), until the next
    set_points."""
    import flash
    from flash import Models, synthetic
    from flash._lib import FlashNativeError
    m = Models.irb140()
    q_true, q_eval = synthetic.perturbed_configuration(m, 3)
    pts = synthetic.depth_cloud(m, q_true, 200000, seed=4)
    ctx = m.engine(0, 64)
    ctx.set_points_range(pts, 0, 100032)
    poses = flash.hull_poses(m, q_eval)
    ctx.eval(poses)
    ctx.chunk_costs()
    ctx.regroup_points()
    with pytest.raises(FlashNativeError):
        ctx.chunk_costs()
    ctx.set_points_range(pts, 0, 100032)
    ctx.eval(poses)
    ctx.chunk_costs()


def test_device_loop_required_refuses_rbf_scene():
    """fsdf_set_solver(2): an RBF scene cannot iterate on the device: refused
    (FSDF_ERR_STATE) instead of silently running the host loop."""
    from flash import Models
    from flash._lib import FlashNativeError
    from flash.gradientdescent import CostFunctor
    m, x0 = Models.irb_and_squishable()
    rng = np.random.default_rng(3)
    pts = np.array([-0.1, -0.3, 0.55]) + rng.random((3000, 3)) * np.array([1.0, 1.0, 0.8])
    cf = CostFunctor(m, pts)
    cf.ctx.set_solver("require")
    with pytest.raises(FlashNativeError):
        cf.descend(np.asarray(x0, np.float64), 2, 1.0, 0.05, 0.0, None, float(len(pts)))
    cf.ctx.set_solver(True)
    x, f, its = cf.descend(np.asarray(x0, np.float64), 2, 1.0, 0.05, 0.0, None, float(len(pts)))
    assert its == 2 and np.isfinite(f)
