"""GPU parity: the HIP residual pass (through the C-ABI) against the CPU oracle
and the committed golden vectors.

Bar (BASELINE.json north_star): nearest-primitive index k* bit-exact; fp64
distances/gradients within 1e-6 relative. The kernel and oracle share the
operation order, so d* and ∇d* are in fact compared bit for bit; sums (cost,
wrenches) differ only in summation order and are compared at 1e-9 relative.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, rng

pytestmark = pytest.mark.gpu

RTOL_SUM = 1e-9


@pytest.fixture(scope="module")
def ctx_factory():
    from flash import _lib
    made = []

    def make(manip, precision=64, cull=True, sort_points=False):
        c = _lib.Context(device=0, precision=precision, cull=cull, sort_points=sort_points)
        c.set_model([(s.hull.vertices, s.hull.faces, s.hull.planes) for s in manip.convex_surfaces()])
        made.append(c)
        return c
    yield make
    for c in made:
        c.close()


def _model(name):
    from flash import Models
    return {"c1_irb140": Models.irb140, "m64_2k": Models.arm_grid, "table_quat": Models.table}[name]()


def _check_against(oracle_out, d, k, g, accum=None, oracle_accum=None, exact=True):
    od, ok, og = oracle_out
    assert np.array_equal(k, ok), f"k* mismatch at {np.nonzero(k != ok)[0][:10]}"
    if exact:
        assert np.array_equal(d, od), f"max |Δd| = {np.abs(d - od).max()}"
        assert np.array_equal(g, og), f"max |Δg| = {np.abs(g - og).max()}"
    else:
        assert np.allclose(d, od, rtol=1e-6, atol=1e-12)
        assert np.allclose(g, og, rtol=1e-6, atol=1e-9)
    if accum is not None:
        assert np.allclose(accum, oracle_accum, rtol=RTOL_SUM, atol=1e-9 * max(1.0, abs(oracle_accum).max()))


@pytest.mark.parametrize("name", ["c1_irb140", "m64_2k", "table_quat"])
@pytest.mark.parametrize("cull", [True, False])
def test_golden_parity(name, cull, ctx_factory):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    ctx = ctx_factory(_model(name), cull=cull)
    ctx.set_points(z["points"])
    cost, accum, (k, d, g) = ctx.eval(z["poses"], per_point=True)
    _check_against((z["d"], z["kstar"], z["grad"]), d, k, g, accum, z["accum"])
    assert cost == accum[0]
    # the skin() entry point (arbitrary query points) agrees with the resident pass
    d2, k2, g2 = ctx.skin(z["poses"], z["points"])
    assert np.array_equal(d2, d) and np.array_equal(k2, k) and np.array_equal(g2, g)


def test_m64_parity_64k(m64, oracle_mod, ctx_factory):
    from flash import synthetic
    import flash
    qt, qe = synthetic.perturbed_configuration(m64, 101)
    for order in ("raster", "shuffled"):
        pts = synthetic.depth_cloud(m64, qt, 65536 + 37, seed=102, order=order)
        poses = flash.hull_poses(m64, qe)
        om = oracle_mod.OracleModel.from_manipulator(m64)
        ref = om.skin(poses, pts)
        ref_acc = om.cost_accum(poses, pts)
        for cull in (True, False):
            ctx = ctx_factory(m64, cull=cull)
            ctx.set_points(pts)
            _, acc, (k, d, g) = ctx.eval(poses, per_point=True)
            _check_against(ref, d, k, g, acc, ref_acc)


def test_edge_cases(irb, oracle_mod, ctx_factory):
    import flash
    ctx = ctx_factory(irb)
    poses = flash.hull_poses(irb, np.zeros(6))
    om = oracle_mod.OracleModel.from_manipulator(irb)
    # empty cloud: zero cost and wrenches
    ctx.set_points(np.zeros((0, 3)))
    cost, acc, _ = ctx.eval(poses)
    assert cost == 0.0 and not acc.any()
    # ragged sizes around wave/block boundaries, points exactly on vertices,
    # hull centroids (deep inside), far field, and duplicates
    verts = np.concatenate([s.hull.vertices @ p[:9].reshape(3, 3).T + p[9:] for s, p in zip(irb.surfaces, poses)])
    cents = np.stack([(s.hull.vertices @ p[:9].reshape(3, 3).T + p[9:]).mean(0) for s, p in zip(irb.surfaces, poses)])
    far = rng(5).normal(size=(50, 3)) * 1e3
    special = np.concatenate([verts, cents, far, verts[:10]])
    assert np.isfinite(special).all()
    for n in (1, 2, 63, 64, 65, 255, 256, 257, 1000, len(special)):
        pts = special[:n] if n <= len(special) else special
        ctx.set_points(pts)
        _, acc, (k, d, g) = ctx.eval(poses, per_point=True)
        _check_against(om.skin(poses, pts), d, k, g, acc, om.cost_accum(poses, pts))


def test_duplicate_hulls_first_index_wins(irb, ctx_factory):
    from flash import Manipulator
    s = irb.surfaces[3]
    m = Manipulator(irb.mechanism, [s, s, s])
    ctx = ctx_factory(m)
    pose = np.concatenate([np.eye(3).ravel(), np.zeros(3)])
    pts = s.hull.vertices.mean(0) + rng(6).normal(scale=0.3, size=(3000, 3))
    d, k, _ = ctx.skin(np.stack([pose] * 3), pts)
    assert (k == 0).all()


def test_deterministic_and_resident(irb, ctx_factory):
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(irb, 7)
    pts = synthetic.depth_cloud(irb, qt, 200000, seed=8)
    ctx = ctx_factory(irb)
    ctx.set_points(pts)
    poses = flash.hull_poses(irb, qe)
    a = ctx.eval(poses, per_point=True)
    b = ctx.eval(poses, per_point=True)
    assert a[0] == b[0] and np.array_equal(a[1], b[1])
    for x, y in zip(a[2], b[2]):
        assert np.array_equal(x, y)


def test_full_size_properties(m64, ctx_factory):
    """BASELINE config size (2^20 points, M64): culled == brute force bit for bit,
    cost == Σ d², and Σ_k F_k == Σ_p 2 d ∇d (size-independent identities)."""
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 201)
    pts = synthetic.depth_cloud(m64, qt, 1 << 20, seed=202)
    poses = flash.hull_poses(m64, qe)
    out = {}
    for cull in (True, False):
        ctx = ctx_factory(m64, cull=cull)
        ctx.set_points(pts)
        out[cull] = ctx.eval(poses, per_point=True)
    (c1, a1, (k1, d1, g1)), (c0, a0, (k0, d0, g0)) = out[True], out[False]
    assert np.array_equal(k1, k0) and np.array_equal(d1, d0) and np.array_equal(g1, g0)
    assert np.array_equal(a1, a0)  # same grid, same fixed-order reduction
    assert c1 == pytest.approx(np.dot(d1, d1), rel=1e-10)
    F = a1[1:].reshape(-1, 6)[:, :3].sum(0)
    assert np.allclose(F, (2 * d1[:, None] * g1).sum(0), rtol=1e-8, atol=1e-8)
    assert np.allclose(np.linalg.norm(g1, axis=1), 1.0, atol=1e-12)


def test_fp32_within_tolerance(m64, oracle_mod, ctx_factory):
    """fp32 residual pass (BASELINE configs 3/5) vs the fp64 oracle."""
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 301)
    pts = synthetic.depth_cloud(m64, qt, 50000, seed=302)
    poses = flash.hull_poses(m64, qe)
    od, ok, og = oracle_mod.OracleModel.from_manipulator(m64).skin(poses, pts)
    ctx = ctx_factory(m64, precision=32)
    ctx.set_points(pts)
    cost, acc, (k, d, g) = ctx.eval(poses, per_point=True)
    assert np.abs(d - od).max() < 2e-5
    # k* may differ only where two hulls are within fp32 resolution of each other
    mism = np.nonzero(k != ok)[0]
    assert len(mism) <= 1e-3 * len(pts)
    assert cost == pytest.approx(np.dot(od, od), rel=1e-4)


def test_cost_functor_gradient_and_tracking(irb):
    """CostFunctor value/gradient on the GPU vs central differences of the GPU
    cost; estimate_state lowers the tracking cost (src/tracking.jl:8-27)."""
    import flash
    from flash import synthetic
    from flash.gradientdescent import CostFunctor
    from flash.tracking import NaiveSolver, estimate_state
    qt, qe = synthetic.perturbed_configuration(irb, 401)
    pts = synthetic.depth_cloud(irb, qt, 20000, seed=402)
    cf = CostFunctor(irb, pts)
    c, g = cf.value_and_gradient(qe)
    h = 1e-6
    for i in range(6):
        xp, xm = qe.copy(), qe.copy()
        xp[i] += h
        xm[i] -= h
        assert g[i] == pytest.approx((cf(xp) - cf(xm)) / (2 * h), rel=1e-5, abs=1e-6)
    seen = []
    x = estimate_state(irb, pts, qe, callback=lambda x, c: seen.append(c),
                       solver=NaiveSolver(6, rate=0.5, max_step=0.05, iteration_limit=20))
    assert seen[-1] < seen[0]
    assert np.linalg.norm(x - qt) < np.linalg.norm(qe - qt) + 1e-9


def test_sort_points_preserves_caller_order(m64, oracle_mod, ctx_factory):
    """sort_points (device Hilbert order) changes only speed: per-point outputs
    come back in caller order, bit-identical to the oracle."""
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 501)
    pts = synthetic.depth_cloud(m64, qt, 30011, seed=502, order="shuffled")
    poses = flash.hull_poses(m64, qe)
    om = oracle_mod.OracleModel.from_manipulator(m64)
    ref, ref_acc = om.skin(poses, pts), om.cost_accum(poses, pts)
    for precision in (64, 32):
        ctx = ctx_factory(m64, precision=precision, sort_points=True)
        ctx.set_points(pts)
        _, acc, (k, d, g) = ctx.eval(poses, per_point=True)
        if precision == 64:
            _check_against(ref, d, k, g, acc, ref_acc)
        else:
            assert np.abs(d - ref[0]).max() < 2e-5
    # a second frame replaces the permutation
    pts2 = pts[::-1].copy()
    ctx.set_points(pts2)
    _, _, (k2, d2, _) = ctx.eval(poses, per_point=True)
    assert np.abs(d2 - ref[0][::-1]).max() < 2e-5


def test_grid_stride_beyond_max_grid(irb, ctx_factory):
    """More points than one wave-iteration per wave covers (16,384 blocks x 256):
    the pass grid-strides; culled == brute force bit for bit, the sorted run
    returns the same per-point values in caller order, cost == Σ d²."""
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(irb, 211)
    n = 16384 * 256 + 12345
    pts = synthetic.depth_cloud(irb, qt, n, seed=212, order="shuffled")
    poses = flash.hull_poses(irb, qe)
    out = {}
    for cull, srt in ((True, True), (False, False)):
        ctx = ctx_factory(irb, cull=cull, sort_points=srt)
        ctx.set_points(pts)
        out[cull] = ctx.eval(poses, per_point=True)
    (c1, a1, (k1, d1, g1)), (c0, a0, (k0, d0, g0)) = out[True], out[False]
    assert np.array_equal(k1, k0) and np.array_equal(d1, d0) and np.array_equal(g1, g0)
    assert c1 == pytest.approx(np.dot(d1, d1), rel=1e-10)
    assert np.allclose(a1, a0, rtol=1e-9, atol=1e-9 * np.abs(a0).max())


def test_cost_ordered_schedule_is_invisible(m64, oracle_mod, ctx_factory):
    """Resident-cloud passes launch their workgroups heaviest-first by the
    previous pass's durations (rebuilt on the first scheduled pass, then every
    16): across 40 passes alternating two configurations, every pass equals the
    first (unscheduled) pass of its configuration bit for bit — per-point
    outputs AND the accumulator (partial sums stay in logical-block columns) —
    and the oracle. A different grid (new cloud size) starts unscheduled."""
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 901)
    pts = synthetic.depth_cloud(m64, qt, 300007, seed=902, order="shuffled")
    poses = [flash.hull_poses(m64, qe), flash.hull_poses(m64, qe + 2e-3)]
    ctx = ctx_factory(m64, sort_points=True)
    ctx.set_points(pts)
    first = [ctx.eval(p, per_point=True) for p in poses]
    for it in range(40):
        c, acc, pp = ctx.eval(poses[it % 2], per_point=True)
        c0, acc0, pp0 = first[it % 2]
        assert c == c0 and np.array_equal(acc, acc0), it
        for x, y in zip(pp, pp0):
            assert np.array_equal(x, y), it
    om = oracle_mod.OracleModel.from_manipulator(m64)
    _check_against(om.skin(poses[1], pts), first[1][2][1], first[1][2][0], first[1][2][2], first[1][1],
                   om.cost_accum(poses[1], pts))
    # a smaller cloud: another grid, the order of the old one is not used
    ctx.set_points(pts[:100003])
    for _ in range(3):
        _, acc_s, (k_s, d_s, _) = ctx.eval(poses[0], per_point=True)
        assert np.array_equal(k_s, first[0][2][0][:100003]) and np.array_equal(d_s, first[0][2][1][:100003])


def test_resident_order_outputs(m64, oracle_mod, ctx_factory):
    """FSDF_ORDER_RESIDENT: per-point outputs in the device (Hilbert) order,
    coalesced; scattered through fsdf_get_permutation they are the caller-order
    outputs bit for bit, and the accumulator does not change. Frames of other
    sizes reuse / grow the sort scratch; device and host permutations agree."""
    import torch
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 511)
    poses = flash.hull_poses(m64, qe)
    ctx = ctx_factory(m64, sort_points=True)
    for n in (40009, 70001, 1000, 40009):
        pts = synthetic.depth_cloud(m64, qt, n, seed=512 + n, order="shuffled")
        ctx.set_points(pts)
        ctx.set_output_order(False)
        _, acc_c, (kc, dc, gc) = ctx.eval(poses, per_point=True)
        ctx.set_output_order(True)
        _, acc_r, (kr, dr, gr) = ctx.eval(poses, per_point=True)
        perm = ctx.permutation()
        assert np.array_equal(np.sort(perm), np.arange(n))
        assert np.array_equal(acc_c, acc_r)
        assert np.array_equal(kr, kc[perm]) and np.array_equal(dr, dc[perm]) and np.array_equal(gr, gc[perm])
        dp = torch.empty(n, dtype=torch.int64, device="cuda:0")
        ctx.permutation_device(dp.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(dp.cpu().numpy(), perm)
    od, ok, _ = oracle_mod.OracleModel.from_manipulator(m64).skin(poses, pts)
    assert np.array_equal(kc, ok) and np.array_equal(dc, od)
    # without sort_points the two orders coincide and the permutation is the identity
    plain = ctx_factory(m64)
    plain.set_points(pts)
    plain.set_output_order(True)
    _, _, (k0, d0, _) = plain.eval(poses, per_point=True)
    assert np.array_equal(plain.permutation(), np.arange(len(pts)))
    assert np.array_equal(k0, kc) and np.array_equal(d0, dc)


@pytest.mark.parametrize("model", ["m64", "irb"])
@pytest.mark.parametrize("tier", [4, 2])
@pytest.mark.parametrize("planned", [False, True])
def test_hull_partitioned_pass_matches_one_wave_per_chunk(m64, irb, ctx_factory, model, tier, planned):
    """Clouds up to the model's 4-way limit run the hull-partitioned pass with
    4 waves per chunk, up to its 2-way limit with 2 (pass_kernel HPART, or the
    planned pass's default shape: hull k goes to wave k % parts, lexicographic
    (d, k) merge; limits per model, fsdf_get_partition); one point more runs
    the next tier (2 waves per chunk, then one wave per chunk). Per-point
    outputs do not depend on the block structure: the shared points agree bit
    for bit, sums to rounding. The same cloud with the tiers forced off
    (fsdf_set_partition) agrees too. planned: the product default
    (fsdf_set_plan), whose first pass on a cloud runs the tier's shape."""
    from flash import synthetic
    import flash
    m = {"m64": m64, "irb": irb}[model]
    probe = ctx_factory(m)
    lim4, lim2, _ = probe.get_partition(0)
    n = lim4 if tier == 4 else lim2
    if n <= 0:
        pytest.skip(f"{model}: the {tier}-way tier is off by default")
    assert probe.get_partition(n)[2] == tier
    assert probe.get_partition(n + 1)[2] == (2 if tier == 4 and lim2 > n else 0)
    qt, qe = synthetic.perturbed_configuration(m, 303)
    poses = flash.hull_poses(m, qe)
    pts = synthetic.depth_cloud(m, qt, n + 1, seed=304, order="shuffled")
    out = {}
    for cull in (True, False):
        for mm in (n, n + 1):
            ctx = ctx_factory(m, cull=cull)
            ctx.set_plan(planned, -1, -1, 1 << 30)  # (planned at every size: the tier's first-pass shape)
            ctx.set_points(pts[:mm])
            out[cull, mm] = ctx.eval(poses, per_point=True)
            name = ctx.pass_kernel_name()
            if planned:
                assert name.startswith("planned_pass_kernel<double"), name
            else:
                assert name.endswith(f"true, true, 256, {tier}>") == (mm == n), name
    forced = ctx_factory(m)
    forced.set_plan(planned, -1, -1, 1 << 30)
    forced.set_partition(0, 0)
    forced.set_points(pts[:n])
    _, _, (kf, df, gf) = forced.eval(poses, per_point=True)
    if not planned:
        assert forced.pass_kernel_name().endswith("true, false, 256, 4>")  # ALIAS, not HPART
    for cull in (True, False):
        (c1, a1, (k1, d1, g1)), (c0, a0, (k0, d0, g0)) = out[cull, n], out[cull, n + 1]
        assert np.array_equal(k1, k0[:n]) and np.array_equal(d1, d0[:n]) and np.array_equal(g1, g0[:n])
        assert np.array_equal(k1, kf) and np.array_equal(d1, df) and np.array_equal(g1, gf)
        assert c1 == pytest.approx(np.dot(d1, d1), rel=1e-10)
    # culled and brute force share the partitioned block structure (planned:
    # per-chunk rows summed in chunk order): identical sums
    assert np.array_equal(out[True, n][1], out[False, n][1])


@pytest.mark.parametrize("sort_points", [True, False])
def test_planned_pass_bits_independent_of_plan(m64, oracle_mod, ctx_factory, sort_points):
    """The planned pass (fsdf_set_plan; per-chunk partial rows summed in chunk
    order) gives the same bits whatever the plan: four plan compositions — all
    chunks one wave, the default shares, a quarter split 4 ways and half 2 ways,
    every chunk 4 ways — agree bit for bit in per-point outputs AND the
    accumulator, on the first (default-shape) pass and on planned passes. Per
    point they equal the unplanned grid's; sums to rounding, and the oracle.
    Unsorted shuffled input puts > 4 nearest surfaces in most chunks (the dense
    row path); sorted input mostly 1-2 (the sparse entries)."""
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 911)
    pts = synthetic.depth_cloud(m64, qt, 262144 + 4321, seed=912, order="shuffled")
    poses = flash.hull_poses(m64, qe)
    res = []
    for shares in ((0.0, 0.0), (1.0 / 32, 1.0 / 16), (0.25, 0.5), (1.0, 0.0)):
        ctx = ctx_factory(m64, sort_points=sort_points)
        ctx.set_plan(True, *shares, 1 << 30)
        ctx.set_points(pts)
        runs = [ctx.eval(poses, per_point=True) for _ in range(3)]  # default shape, then planned
        assert ctx.pass_kernel_name().startswith("planned_pass_kernel")
        res.append(runs)
    c0, a0, p0 = res[0][0]
    for runs in res:
        for c, a, pp in runs:
            assert c == c0 and np.array_equal(a, a0)
            for x, y in zip(pp, p0):
                assert np.array_equal(x, y)
    legacy = ctx_factory(m64, sort_points=sort_points)
    legacy.set_plan(False)
    legacy.set_points(pts)
    cl, al, pl = legacy.eval(poses, per_point=True)
    assert not legacy.pass_kernel_name().startswith("planned")
    for x, y in zip(pl, p0):
        assert np.array_equal(x, y)
    assert np.allclose(al, a0, rtol=1e-11, atol=1e-12 * np.abs(a0).max())
    om = oracle_mod.OracleModel.from_manipulator(m64)
    _check_against(om.skin(poses, pts), p0[1], p0[0], p0[2], a0, om.cost_accum(poses, pts))


@pytest.mark.parametrize("model,limit,above", [("m64", 524288, False), ("irb", 393216, False), ("irb", 98304, True)])
def test_planned_pass_default_limit_per_model(m64, irb, ctx_factory, model, limit, above):
    """The planned pass's default size window follows the model (fsdf_set_plan
    max_points -1; DESIGN.md §7, profiles/r04/hpart_sweep_c2.jsonl): up to the
    upper limit a resident pass runs planned, one point more runs the unplanned
    grid; at the lower limit (98,304 points, both models) unplanned, one point
    more planned — with the same per-point bits on the points both clouds
    share."""
    import flash
    from flash import synthetic
    m = {"m64": m64, "irb": irb}[model]
    qt, qe = synthetic.perturbed_configuration(m, 505)
    poses = flash.hull_poses(m, qe)
    pts = synthetic.depth_cloud(m, qt, limit + 1, seed=506, order="shuffled")
    out = {}
    for mm, planned in ((limit, not above), (limit + 1, above)):
        ctx = ctx_factory(m)
        ctx.set_points(pts[:mm])
        out[mm] = ctx.eval(poses, per_point=True)
        assert ctx.pass_kernel_name().startswith("planned_pass_kernel") == planned, (mm, ctx.pass_kernel_name())
    for x, y in zip(out[limit][2], out[limit + 1][2]):
        assert np.array_equal(x, y[:limit])


def test_planned_pass_follows_cloud_changes(m64, ctx_factory):
    """A context's plan belongs to its cloud: after set_points with a smaller,
    then a larger cloud (chunk rows reallocated, plan rebuilt on the new cloud's
    first pass) every pass equals a fresh context's on that cloud bit for bit —
    no stale plan entry, no stale chunk row."""
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 707)
    poses = flash.hull_poses(m64, qe)
    big = synthetic.depth_cloud(m64, qt, 300000 + 77, seed=708, order="shuffled")
    small = synthetic.depth_cloud(m64, qt, 150000 + 5, seed=709, order="shuffled")
    ctx = ctx_factory(m64, sort_points=True)
    for pts in (big[:300000], small, big):
        fresh = ctx_factory(m64, sort_points=True)
        fresh.set_points(pts)
        want = fresh.eval(poses, per_point=True)
        ctx.set_points(pts)
        for _ in range(3):  # first pass (tier shape), then planned
            c, a, pp = ctx.eval(poses, per_point=True)
            assert ctx.pass_kernel_name().startswith("planned_pass_kernel")
            assert c == want[0] and np.array_equal(a, want[1])
            for x, y in zip(pp, want[2]):
                assert np.array_equal(x, y)


def test_passes_in_flight_bit_identical(m64, ctx_factory):
    """Independent passes in flight (bench.py --inflight): two
    contexts over the same resident cloud on two non-null HIP streams, passes
    interleaved without synchronisation — every accumulator and per-point output
    equals a serial context's bit for bit (planned window and 2^20 unplanned)."""
    import torch
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 808)
    poses = [flash.hull_poses(m64, qe), flash.hull_poses(m64, qe + 1e-3)]
    dev = torch.device("cuda", 0)
    for n in (200000, 1 << 20):
        pts = synthetic.depth_cloud(m64, qt, n, seed=809, order="shuffled")
        serial = ctx_factory(m64, sort_points=True)
        serial.set_points(pts)
        want = [serial.eval(p, per_point=True) for p in poses]
        d_pts = torch.as_tensor(pts, device=dev)
        streams = [torch.cuda.Stream(dev) for _ in range(2)]
        ctxs, accs, outs = [], [], []
        for c in range(2):
            cx = ctx_factory(m64, sort_points=True)
            cx.set_stream(streams[c].cuda_stream)
            cx.set_points_device(d_pts.data_ptr(), n)
            ctxs.append(cx)
            accs.append([torch.zeros(cx.accum_len, dtype=torch.float64, device=dev) for _ in range(2)])
            outs.append([(torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.float64, device=dev),
                          torch.empty((n, 3), dtype=torch.float64, device=dev)) for _ in range(2)])
        torch.cuda.synchronize()
        for i in range(24):  # first passes, then planned; never synchronised in between
            c, s = i % 2, (i // 2) & 1
            ctxs[c].eval_device(poses[s], accs[c][s].data_ptr(), *(b.data_ptr() for b in outs[c][s]))
        torch.cuda.synchronize()
        for c in range(2):
            for s in (0, 1):  # (per-point outputs in caller order, the default)
                assert np.array_equal(accs[c][s].cpu().numpy(), want[s][1])
                k, d, g = (b.cpu().numpy() for b in outs[c][s])
                assert np.array_equal(k, want[s][2][0]) and np.array_equal(d, want[s][2][1])
                assert np.array_equal(g, want[s][2][2])
        del d_pts


@pytest.mark.parametrize("sort_points", [True, False])
def test_point_ranges_edge_cases(m64, ctx_factory, sort_points):
    """fsdf_set_points_range at chunk-unaligned, single-point and empty ranges:
    bad ranges fail with FSDF_ERR_ARG and leave the context usable; an empty
    range gives zero cost and wrenches; every other range's per-point outputs
    equal the whole cloud's at the indices permutation() names (the Hilbert
    order's with sort_points, the caller's without), the ranges' permutations
    partition the cloud, and their costs and wrenches sum to the whole cloud's."""
    import flash
    from flash import synthetic
    from flash._lib import FlashNativeError
    qt, qe = synthetic.perturbed_configuration(m64, 731)
    poses = flash.hull_poses(m64, qe)
    n = 70001
    pts = synthetic.depth_cloud(m64, qt, n, seed=732, order="shuffled")
    whole = ctx_factory(m64, sort_points=sort_points)
    whole.set_points(pts)
    whole.set_output_order(False)
    c_all, acc_all, (ka, da, ga) = whole.eval(poses, per_point=True)
    ctx = ctx_factory(m64, sort_points=sort_points)
    for b, e in ((-1, 10), (10, 5), (0, n + 1)):
        with pytest.raises(FlashNativeError):
            ctx.set_points_range(pts, b, e)
    ctx.set_points_range(pts, 500, 500)
    cost, acc, _ = ctx.eval(poses)
    assert cost == 0.0 and not acc.any()
    cuts = [0, 1, 37, 64 * 100 + 5, 64 * 500, n - 1, n]
    seen = np.zeros(n, np.int32)
    c_sum, acc_sum = 0.0, np.zeros_like(acc_all)
    for b, e in zip(cuts[:-1], cuts[1:]):
        ctx.set_points_range(pts, b, e)
        cost, acc, (k, d, g) = ctx.eval(poses, per_point=True)
        perm = ctx.permutation()
        assert len(perm) == e - b
        if not sort_points:
            assert np.array_equal(perm, np.arange(b, e))
        seen[perm] += 1
        assert np.array_equal(k, ka[perm]) and np.array_equal(d, da[perm]) and np.array_equal(g, ga[perm])
        c_sum += cost
        acc_sum += acc
    assert (seen == 1).all()
    assert c_sum == pytest.approx(c_all, rel=RTOL_SUM)
    assert np.allclose(acc_sum, acc_all, rtol=1e-9, atol=1e-9 * max(1.0, np.abs(acc_all).max()))


@pytest.mark.parametrize("n", [20011, 131077, 530000])
def test_prior_seeds_change_no_bits(m64, ctx_factory, n):
    """Passes after a cloud's first seed each point's search from its nearest
    surface in the previous pass (PassOutputs::prior_in): every output — cost,
    accumulator, k*, d*, ∇d* — equals a first pass at the same configuration
    (no prior) bit for bit, on the 4-way tier, the planned pass and the
    one-wave grid; a new cloud (set_points) drops the prior."""
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 901)
    poses = [flash.hull_poses(m64, qe + d) for d in (0.0, 2e-3, -3e-3, 2e-3)]
    pts = synthetic.depth_cloud(m64, qt, n, seed=902, order="shuffled")
    warm = ctx_factory(m64, sort_points=True)
    warm.set_points(pts)
    runs = [warm.eval(p, per_point=True) for p in poses]
    cold = ctx_factory(m64, sort_points=True)
    for p, (c1, a1, (k1, d1, g1)) in zip(poses, runs):
        cold.set_points(pts)  # a first pass each time
        c0, a0, (k0, d0, g0) = cold.eval(p, per_point=True)
        assert c1 == c0 and np.array_equal(a1, a0)
        assert np.array_equal(k1, k0) and np.array_equal(d1, d0) and np.array_equal(g1, g0)


@pytest.mark.parametrize("n", [131077, 530000])
def test_regroup_points(m64, ctx_factory, n):
    """fsdf_regroup_points: the resident cloud regrouped by each point's nearest
    surface in the last pass (stable: the Hilbert order kept within a group).
    The permutation stays a permutation, the groups are contiguous, and later
    passes give every point's k*, d*, ∇d* bit for bit as an unregrouped
    context does, their sums to rounding; a ranged cloud regroups within its
    range; without a pass, or without a permutation, it refuses."""
    import flash
    from flash import synthetic
    from flash._lib import FlashNativeError
    qt, qe = synthetic.perturbed_configuration(m64, 911)
    pa, pb = flash.hull_poses(m64, qe), flash.hull_poses(m64, qe + 2e-3)
    pts = synthetic.depth_cloud(m64, qt, n, seed=912, order="shuffled")
    plain = ctx_factory(m64, sort_points=True)
    plain.set_points(pts)
    cb, accb, (kb, db, gb) = plain.eval(pb, per_point=True)  # caller order
    for begin, end in ((0, n), (64 * 100, n - 5)):
        ctx = ctx_factory(m64, sort_points=True)
        if (begin, end) == (0, n):
            ctx.set_points(pts)
        else:
            ctx.set_points_range(pts, begin, end)
        with pytest.raises(FlashNativeError):
            ctx.regroup_points()  # no pass yet
        ctx.set_output_order(True)
        _, _, (ka, _, _) = ctx.eval(pa, per_point=True)
        perm0 = ctx.permutation()
        ctx.regroup_points()
        perm1 = ctx.permutation()
        assert np.array_equal(np.sort(perm1), np.sort(perm0))
        pos0 = np.empty(perm0.max() + 1, np.int64)
        pos0[perm0] = np.arange(len(perm0))
        k_at = np.empty(perm0.max() + 1, np.int32)
        k_at[perm0] = ka
        kg, old = k_at[perm1], pos0[perm1]
        assert np.all(np.diff(kg) >= 0)  # contiguous groups, ascending surface
        same = np.diff(kg) == 0
        assert np.all(np.diff(old)[same] > 0)  # the previous order within a group
        c1, acc1, (k1, d1, g1) = ctx.eval(pb, per_point=True)
        assert np.array_equal(k1, kb[perm1]) and np.array_equal(d1, db[perm1]) and np.array_equal(g1, gb[perm1])
        if (begin, end) == (0, n):
            assert c1 == pytest.approx(cb, rel=1e-12)
            assert np.allclose(acc1, accb, rtol=1e-10, atol=1e-12 * np.abs(accb).max())
    unsorted = ctx_factory(m64, sort_points=False)
    unsorted.set_points(pts)
    unsorted.eval(pa)
    with pytest.raises(FlashNativeError):
        unsorted.regroup_points()


@pytest.mark.parametrize("n", [131077, 1 << 20])
def test_regroup_follows_last_pass(m64, ctx_factory, n):
    """The seed bytes a pass leaves behind (PassOutputs::prior_out) are that
    pass's k* at every point, though a seeded pass stores a byte only where k*
    changed: after passes at configurations far enough apart that many points
    change surface, fsdf_regroup_points groups by the LAST pass's k*; and again
    after more passes over the regrouped cloud."""
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 931)
    confs = [flash.hull_poses(m64, qe + d) for d in (0.0, 0.06, -0.05, 0.03)]
    pts = synthetic.depth_cloud(m64, qt, n, seed=932, order="shuffled")
    ctx = ctx_factory(m64, sort_points=True)
    ctx.set_points(pts)
    ctx.set_output_order(True)
    for rounds in range(2):
        ks = []
        for p in confs[2 * rounds:2 * rounds + 2]:
            _, _, (k, _, _) = ctx.eval(p, per_point=True)  # resident order
            ks.append(k.copy())
        changed = int(np.count_nonzero(ks[0] != ks[1]))
        assert changed > n // 1000, changed  # the second pass rewrote many seed bytes
        perm0 = ctx.permutation()
        ctx.regroup_points()
        perm1 = ctx.permutation()
        pos0 = np.empty(perm0.max() + 1, np.int64)
        pos0[perm0] = np.arange(len(perm0))
        kg = ks[1][pos0[perm1]]  # the last pass's k*, in the regrouped order
        assert np.all(np.diff(kg) >= 0)


def test_cost_functor_regroup(irb):
    """CostFunctor.regroup(): after the frame's first evaluation, later ones
    give the same cost and gradient to rounding."""
    from flash import synthetic
    from flash.gradientdescent import CostFunctor
    qt, qe = synthetic.perturbed_configuration(irb, 921)
    pts = synthetic.depth_cloud(irb, qt, 200003, seed=922, order="shuffled")
    cf = CostFunctor(irb, pts)
    x = np.asarray(qe, np.float64)
    c0, g0 = cf.value_and_gradient(x)
    cf.regroup()
    c1, g1 = cf.value_and_gradient(x)
    assert c1 == pytest.approx(c0, rel=1e-12)
    assert np.allclose(g1, g0, rtol=1e-9, atol=1e-12 * np.abs(g0).max())
