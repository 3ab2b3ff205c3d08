"""GPU: the heavy-wave split (fsdf_set_split_budget). A pass-kernel wave that
has run B hull evaluations hands the hulls it still needs to the overflow
kernel; the merge kernel folds them back. The split must not change any
per-point result (d*, k*, ∇d* bit for bit against the unsplit pass and the
oracle) and changes the accumulator only in summation order (1e-12 relative);
a given budget is deterministic run to run."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ctx(m, precision=64, sort_points=True, budget=0):
    from flash import _lib
    c = _lib.Context(device=0, precision=precision, cull=True, sort_points=sort_points)
    c.set_model([(s.hull.vertices, s.hull.faces, s.hull.planes) for s in m.convex_surfaces()])
    c.set_split_budget(budget)
    return c


@pytest.fixture(scope="module")
def scene():
    import flash
    from flash import Models, synthetic
    m = Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m, 1234)
    return m, flash.hull_poses(m, qe), synthetic.depth_cloud(m, qt, 1 << 20, seed=1234 + 17, order="shuffled")


def _close(a, b, rtol=1e-12):
    return np.allclose(a, b, rtol=rtol, atol=rtol * np.abs(b).max())


@pytest.mark.parametrize("n", [1 << 20, 131072, 4099])
def test_split_matches_unsplit(scene, n):
    m, poses, pts = scene
    pts = pts[:n]
    ref = _ctx(m, budget=0)
    ref.set_points(pts)
    c0, a0, (k0, d0, g0) = ref.eval(poses, per_point=True)
    ref.close()
    for budget in (1, 2, 3):
        c = _ctx(m, budget=budget)
        c.set_points(pts)
        for _ in range(2):  # the second pass runs the cost-ordered schedule
            cost, acc, (k, d, g) = c.eval(poses, per_point=True)
            assert np.array_equal(k, k0), f"budget {budget}: k* differs at {np.nonzero(k != k0)[0][:8]}"
            assert np.array_equal(d, d0) and np.array_equal(g, g0), f"budget {budget}"
            assert _close(acc, a0), f"budget {budget}: max |Δacc| {np.abs(acc - a0).max()}"
        # deterministic for a given budget and schedule
        _, acc2, _ = c.eval(poses, per_point=True)
        _, acc3, _ = c.eval(poses, per_point=True)
        assert np.array_equal(acc2, acc3)
        c.close()


def test_split_resident_order_and_oracle(scene, oracle_mod):
    """Resident-order outputs of a split pass + the oracle on a sample."""
    m, poses, pts = scene
    c = _ctx(m, budget=1)
    c.set_points(pts)
    c.set_output_order(True)
    _, acc, (k, d, g) = c.eval(poses, per_point=True)
    perm = c.permutation()
    c.close()
    ref = _ctx(m, budget=0)
    ref.set_points(pts)
    _, acc0, (k0, d0, g0) = ref.eval(poses, per_point=True)
    ref.close()
    assert np.array_equal(k, k0[perm]) and np.array_equal(d, d0[perm]) and np.array_equal(g, g0[perm])
    assert _close(acc, acc0)
    om = oracle_mod.OracleModel.from_manipulator(m)
    idx = np.random.default_rng(5).choice(len(pts), 20000, replace=False)
    od, ok, og = om.skin(poses, pts[idx])
    assert np.array_equal(k0[idx], ok) and np.array_equal(d0[idx], od) and np.array_equal(g0[idx], og)


def test_split_capacity_overflow(scene):
    """Budget 1 on 4M points reserves more items than the 16,384-item buffer
    holds: the waves past the capacity evaluate in place; results unchanged."""
    import flash
    from flash import synthetic
    m, poses, _ = scene
    qt, _ = synthetic.perturbed_configuration(m, 1234)
    pts = synthetic.depth_cloud(m, qt, 4 << 20, seed=99, order="shuffled")
    out = []
    for budget in (0, 1):
        c = _ctx(m, budget=budget)
        c.set_points(pts)
        c.kernel_stats(True)
        cost, acc, (k, d, g) = c.eval(poses, per_point=True)
        c.kernel_stats(False)
        out.append((acc, k, d, g))
        c.close()
    (a0, k0, d0, g0), (a1, k1, d1, g1) = out
    assert np.array_equal(k0, k1) and np.array_equal(d0, d1) and np.array_equal(g0, g1)
    assert _close(a1, a0)


def test_split_f32_and_skin(scene):
    """fp32 context and fsdf_skin (unsorted query, no schedule) split too."""
    m, poses, pts = scene
    q = pts[:200000]
    res = []
    for budget in (0, 2):
        c = _ctx(m, precision=32, budget=budget)
        c.set_points(q)
        _, acc, (k, d, g) = c.eval(poses, per_point=True)
        c.close()
        c = _ctx(m, budget=budget, sort_points=False)
        sd, sk, sg = c.skin(poses, q[:50000])
        c.close()
        res.append((acc, k, d, g, sd, sk, sg))
    a, b = res
    assert _close(b[0], a[0], rtol=1e-6)  # f32 contexts still sum in f64
    for x, y in zip(a[1:], b[1:]):
        assert np.array_equal(x, y)


def test_split_budget_argument():
    from flash import Models, FlashNativeError
    c = _ctx(Models.irb140())
    with pytest.raises(FlashNativeError):
        c.set_split_budget(-1)
    c.close()
