"""GPU: the track! frame loop (examples/irb_and_squishable.ipynb cells 11-12)
on a moving IRB140 — per frame a new sensed cloud, estimate_state warm-started
from the previous frame's solution, the resident cloud swapped in place.
Solver kwargs as examples/irb140.ipynb cell 9 passes them (rate 20, a
gradient-convergence tolerance); the update rule itself is unpinned
(SimpleGradientDescent is un-vendored), so the checks are behavioural: the
tracker follows the motion, warm starts beat cold starts, and every frame's
cost falls."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sequence(m, frames=12, n=4000, seed=70):
    from flash import synthetic
    qa, _ = synthetic.perturbed_configuration(m, seed)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    qb = qa + rng.uniform(-0.08, 0.08, size=qa.shape)
    qs = [qa + (qb - qa) * t / (frames - 1) for t in range(frames)]
    clouds = [synthetic.depth_cloud(m, q, n, seed=seed + 10 + t, sigma=0.001, frac_surface=1.0, frac_box=0.0)
              for t, q in enumerate(qs)]
    return qs, clouds


def test_track_follows_motion_with_warm_start():
    import flash
    from flash import Models
    from flash.tracking import NaiveSolver, Tracker, track
    from flash.gradientdescent import CostFunctor
    m = Models.irb140()
    qs, clouds = _sequence(m)
    n = flash.num_states(m)
    x0 = qs[0] + 0.05
    state = flash.ManipulatorState(m)
    state.q[:] = x0
    seen = []
    solver = NaiveSolver(n, rate=20.0, max_step=0.1, iteration_limit=30, gradient_convergence_tolerance=1e-6)
    xs, tr = track(m, clouds, state=state, solver=solver, callback=lambda x, c: seen.append(c))
    assert xs.shape == (len(clouds), n)
    assert np.array_equal(state.q, xs[-1])  # unflatten!(state, x_star)
    # the first three joints (the notebook ignores the wrist, examples/irb140.ipynb cell 9)
    err = [np.abs(x[:3] - q[:3]).max() for x, q in zip(xs, qs)]
    hold = np.abs(x0[:3] - qs[-1][:3]).max()  # error of not tracking at all
    assert err[-1] < 0.5 * hold and np.mean(err) < 0.04, (err, hold)
    # per frame the objective falls from the first to the last iteration
    assert len(seen) == sum(tr.iterations) and tr.iteration_ms() > 0
    k = 0
    for its in tr.iterations:
        assert seen[k + its - 1] <= seen[k]
        k += its


def test_notebook_frame_solver_single_iteration():
    """gradient_descent!'s NaiveSolver(rate=0.5, max_step=0.1,
    iteration_limit=1): one pass per frame, the step bounded by max_step."""
    import flash
    from flash import Models
    from flash.tracking import Tracker, notebook_frame_solver
    m = Models.irb140()
    qs, clouds = _sequence(m, frames=3, n=2000, seed=80)
    state = flash.ManipulatorState(m)
    state.q[:] = qs[0] + 0.02
    tr = Tracker(m, state, notebook_frame_solver(m))
    prev = state.q.copy()
    for pts in clouds:
        x = tr.step(pts)
        assert np.abs(x - prev).max() <= 0.1 + 1e-15
        prev = x.copy()
    assert tr.iterations == [1, 1, 1]


def test_track_lcm_log(tmp_path):
    """examples/irb_and_squishable.ipynb cell 12 end to end: a log of
    bot_core.pointcloud_t frames on KINECT_POINTS_REDUCED (plus an unrelated
    channel), decoded, subsampled [1:200:end], tracked with the warm start
    carried — identical to tracking the same clouds directly."""
    import flash
    from flash import Models, lcmlog
    from flash.tracking import NaiveSolver, track
    m = Models.irb140()
    qs, clouds = _sequence(m, frames=4, n=40000, seed=90)
    events = []
    for t, c in enumerate(clouds):
        msg = lcmlog.PointCloudMsg(utime=1000 * t, points=c, channel_names=["r", "g", "b"],
                                   channels=np.zeros((3, len(c))))
        events += [(1000 * t, "KINECT_POINTS_REDUCED", lcmlog.encode_pointcloud(msg)), (1000 * t + 1, "OTHER", b"x")]
    path = tmp_path / "track.lcm"
    lcmlog.write_log(path, events)
    n = flash.num_states(m)

    def run(frames):
        st = flash.ManipulatorState(m)
        st.q[:] = qs[0] + 0.03
        return track(m, frames, state=st, solver=NaiveSolver(n, rate=20.0, max_step=0.1, iteration_limit=5))[0]

    xs_log, tr = lcmlog.track_log(m, str(path), state=None, solver=NaiveSolver(n, rate=20.0, max_step=0.1,
                                                                                 iteration_limit=5))
    assert xs_log.shape == (4, n) and len(tr.frame_ms) == 4
    st = flash.ManipulatorState(m)
    st.q[:] = qs[0] + 0.03
    xs_a, _ = lcmlog.track_log(m, str(path), state=st, solver=NaiveSolver(n, rate=20.0, max_step=0.1,
                                                                            iteration_limit=5))
    xs_b = run([c.astype(np.float32)[::200].astype(np.float64) for c in clouds])
    assert np.array_equal(xs_a, xs_b)


@pytest.mark.parametrize("scene", ["irb140", "irb_and_squishable"])
def test_native_descend_matches_python_loop(scene):
    """fsdf_descend (the NaiveSolver loop inside the library) against the
    Python loop over value_and_gradient (taken whenever a callback is given):
    the same x trajectory bit for bit, with preconditioning divisors, and the
    same stopping iteration under a convergence tolerance."""
    import flash
    from flash import Models, synthetic
    from flash.gradientdescent import CostFunctor, flatten
    from flash.tracking import NaiveSolver, _optimize
    if scene == "irb140":
        m = Models.irb140()
        q_true, _ = synthetic.perturbed_configuration(m, 31)
        pts = synthetic.depth_cloud(m, q_true, 6000, seed=32, frac_box=0.0, frac_surface=1.0, sigma=0.001)
        st = flash.ManipulatorState(m)
        st.q[:] = q_true + 0.03
        x0 = flatten(st)
    else:  # 7 hulls + the squishable RBF skin (deformations) + table, 63 states
        m, x0 = Models.irb_and_squishable()
        nq = m.mechanism.num_positions
        x0 = np.array(x0, np.float64)
        rng = np.random.default_rng(33)
        x0[nq:] = 0.004 * rng.normal(size=len(x0) - nq)
        pts = np.array([-0.1, -0.3, 0.55]) + rng.random((6000, 3)) * np.array([1.0, 1.0, 0.8])
    n = flash.num_states(m)
    cf = CostFunctor(m, pts)
    assert cf._native
    div = np.linspace(1.0, 2.0, n)
    for tol, limit in ((0.0, 6), (1e-3, 40)):
        sa = NaiveSolver(n, rate=5.0, max_step=0.05, iteration_limit=limit, gradient_convergence_tolerance=tol,
                         precondition_divisors=div)
        sb = NaiveSolver(n, rate=5.0, max_step=0.05, iteration_limit=limit, gradient_convergence_tolerance=tol,
                         precondition_divisors=div)
        seen = []
        xa = _optimize(cf, len(pts), x0, lambda x, c: seen.append(c), sa)  # Python loop
        xb = _optimize(cf, len(pts), x0, None, sb)                          # fsdf_descend
        assert np.array_equal(xa, xb), np.abs(xa - xb).max()
        assert sa.iterations == sb.iterations == len(seen)
        if tol == 0.0:
            assert sb.iterations == limit
    with pytest.raises(ValueError):
        cf.descend(x0[:-1], 2, 1.0, 0.1)
    x_same, f0, its = cf.descend(x0, 0, 1.0, 0.1)  # iteration_limit 0: x untouched
    assert its == 0 and np.array_equal(x_same, x0)
    x1, f1, its = cf.descend(x0, 1, 5.0, 0.05, n_points=len(pts))
    c, g = cf.value_and_gradient(x0)
    assert its == 1 and f1 == c / len(pts)
    assert np.array_equal(x1, x0 + np.clip(-5.0 * (g / len(pts)), -0.05, 0.05))


def test_prefetched_frames_same_bits():
    """track() uploads frame t+1 during frame t's iterations
    (fsdf_prefetch_points on the context's copy stream, fsdf_set_points_prefetched):
    the per-frame solutions equal a Tracker.step loop without prefetch bit for
    bit (native solver loop). The ABI refuses set_points_prefetched with nothing
    pending, a second prefetch replaces the first, and a page-locked cloud
    becomes resident exactly as fsdf_set_points makes it."""
    import torch
    import flash
    from flash import Models
    from flash._lib import FlashNativeError
    from flash.tracking import NaiveSolver, Tracker, track
    m = Models.irb140()
    qs, clouds = _sequence(m, frames=5, n=20000, seed=90)
    n = flash.num_states(m)
    out = []
    for prefetch in (True, False):
        state = flash.ManipulatorState(m)
        state.q[:] = qs[0] + 0.03
        solver = NaiveSolver(n, rate=20.0, max_step=0.1, iteration_limit=10)
        if prefetch:
            xs, _ = track(m, clouds, state=state, solver=solver)
        else:
            tr = Tracker(m, state, solver)
            xs = np.array([tr.step(c) for c in clouds])
        out.append(xs)
    assert np.array_equal(out[0], out[1])
    ctx, ref = m.engine(0, 64, slot=5), m.engine(0, 64, slot=6)
    poses = flash.hull_poses(m, qs[2])
    with pytest.raises(FlashNativeError):
        ctx.set_points_prefetched()
    pinned = torch.empty((len(clouds[3]), 3), dtype=torch.float64, pin_memory=True)
    pinned.copy_(torch.from_numpy(clouds[3]))
    ctx.prefetch_points(clouds[1])
    ctx.prefetch_points(pinned.numpy())  # replaces the pending prefetch
    ctx.set_points_prefetched()
    ref.set_points(clouds[3])
    assert ctx.n == ref.n == len(clouds[3])
    (c0, a0, (k0, d0, g0)), (c1, a1, (k1, d1, g1)) = ctx.eval(poses, True), ref.eval(poses, True)
    assert c0 == c1 and np.array_equal(a0, a1)
    assert np.array_equal(k0, k1) and np.array_equal(d0, d1) and np.array_equal(g0, g1)
    with pytest.raises(FlashNativeError):  # consumed
        ctx.set_points_prefetched()


@pytest.mark.parametrize("sort_points", [True, False])
def test_prefetch_edge_cases(sort_points):
    """fsdf_prefetch_points with an unsorted context (consumed through the
    plain device ingest), an empty cloud, and a plain set_points between a
    prefetch and its consumption (the prefetched cloud still becomes resident,
    then the next frame's buffers are swapped back and forth): every resident
    cloud evaluates exactly as fsdf_set_points makes it."""
    import flash
    from flash import Models
    m = Models.irb140()
    qs, clouds = _sequence(m, frames=4, n=30000, seed=95)
    poses = flash.hull_poses(m, qs[1])
    ctx = m.engine(0, 64, sort_points=sort_points, slot=7)
    ref = m.engine(0, 64, sort_points=sort_points, slot=8)

    def same(pts):
        ref.set_points(pts)
        assert ctx.n == ref.n == len(pts)
        (c0, a0, p0), (c1, a1, p1) = ctx.eval(poses, True), ref.eval(poses, True)
        assert c0 == c1 and np.array_equal(a0, a1)
        for u, v in zip(p0, p1):
            assert np.array_equal(u, v)

    ctx.prefetch_points(np.zeros((0, 3)))
    ctx.set_points_prefetched()
    assert ctx.n == 0
    ctx.prefetch_points(clouds[0])
    ctx.set_points(clouds[1])  # (does not consume the prefetch)
    same(clouds[1])
    ctx.set_points_prefetched()
    same(clouds[0])
    for t in (2, 3, 0):  # buffers swapped back and forth
        ctx.prefetch_points(clouds[t])
        ctx.eval(poses)  # (a pass of the current frame while the next one is copied)
        ctx.set_points_prefetched()
        same(clouds[t])


def test_prefetch_grouped_frames_match_to_rounding():
    """2^20-point M64 frames (the one-wave grid, where the library groups a
    cloud by nearest surface): with prefetch the next cloud is grouped on the
    copy stream by the seeds carried from two frames back (fsdf_prefetch_points),
    without it by the auto regroup after each frame's first pass. Per-point
    results do not depend on the grouping, the sums differ in rounding only:
    the per-frame solutions agree to 1e-9 relative."""
    import flash
    from flash import Models
    from flash.tracking import NaiveSolver, Tracker, track
    m = Models.arm_grid()
    qs, clouds = _sequence(m, frames=4, n=1 << 20, seed=97)
    n = flash.num_states(m)
    out = []
    for prefetch in (True, False):
        state = flash.ManipulatorState(m)
        state.q[:] = qs[0] + 0.02
        solver = NaiveSolver(n, rate=20.0, max_step=0.1, iteration_limit=8)
        if prefetch:
            xs, tr = track(m, clouds, state=state, solver=solver)
        else:
            tr = Tracker(m, state, solver)
            xs = np.array([tr.step(c) for c in clouds])
        out.append((xs, list(tr.iterations)))
    (xa, ia), (xb, ib) = out
    assert ia == ib
    scale = np.maximum(np.abs(xb), 1.0)
    assert np.all(np.abs(xa - xb) <= 1e-9 * scale), np.abs(xa - xb).max()
