"""GPU: BASELINE configs at their full sizes.

* C4 (configs[3]): ONE 10·2^20-point IRB140 cloud sharded over 8 ranks, each
  rank a flash.distributed.ShardedCostFunctor on its contiguous shard with the
  per-pass all-reduce of the accumulator — here 8 gloo ranks sharing device 0
  (8 RCCL ranks need 8 GPUs; the driver's scaling runs use "nccl"). Against
  ONE context over the whole cloud: k*, d*, ∇d* bit-exact, the accumulator
  within 1e-9 relative, ∂c/∂x within 1e-7 (sums differ in order
  only).
* C3 (configs[2]): the deformable beanbag (RBF skin, 25 states) at 2^20 points
  in fp32 (the config's precision): culled ≡ brute force bit for bit, the
  accumulator's cost = Σ d*², and d* within the fp32 tolerance of the fp64
  oracle on a 20,000-point sample (and of an fp64 context on all points).
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

C4_POINTS = 10 * (1 << 20)
C4_RANKS = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _c4_state():
    from flash import Models, synthetic
    m = Models.irb140()
    qt, qe = synthetic.perturbed_configuration(m, 71)
    return m, qt, np.asarray(qe, np.float64)


def _c4_worker(rank, world, port, cloud_path, out_dir, mode="slice"):
    import sys
    from conftest import ROOT
    sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))
    import torch.distributed as dist
    from flash.distributed import ShardedCostFunctor, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m, _, x = _c4_state()
        cloud = np.load(cloud_path, mmap_mode="r")
        spatial = mode != "slice"
        if mode == "spatial":  # the whole cloud on every rank, a range of its Hilbert order kept
            f = ShardedCostFunctor(m, np.ascontiguousarray(cloud), rank=rank, world=world, device=0, spatial=True)
            a, b = f.range
        elif mode == "exchange":  # only this rank's slice uploaded; points moved to their key range's rank
            a, b = shard_range(len(cloud), rank, world)
            f = ShardedCostFunctor(m, np.ascontiguousarray(cloud[a:b]), rank=rank, world=world, device=0,
                                   exchange=True)
        else:
            a, b = shard_range(len(cloud), rank, world)
            f = ShardedCostFunctor(m, np.ascontiguousarray(cloud[a:b]), rank=rank, world=world, device=0)
        x2 = x.copy()
        x2[1] += 2e-3
        f.value_and_gradient(x2)  # a pass at another configuration first (resident cloud, schedule)
        c, g = f.value_and_gradient(x)
        acc = f.accum.cpu().numpy()
        k, d, gr = f.per_point(x)
        idx = f.global_index() if spatial else np.arange(a, b)
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), c=c, g=g, acc=acc, d=d, k=k, gr=gr, a=a, b=b, idx=idx)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["slice", "spatial", "exchange"])
def test_c4_ten_million_points_sharded_over_eight_ranks(mode, tmp_path):
    """Slices of the caller's order (round 4), density-preserving ranges of
    the whole cloud's Hilbert order (spatial: every rank uploads the whole
    cloud) and exchanged shards (exchange: every rank uploads only its slice,
    flash.distributed.exchange_points): per-point outputs placed at their
    whole-cloud indices are the single context's bit for bit; the exchanged
    shards, concatenated in rank order, are exactly the single context's
    Hilbert order."""
    import multiprocessing as mp
    from flash import synthetic
    from flash.gradientdescent import CostFunctor
    m, qt, x = _c4_state()
    cloud = synthetic.depth_cloud(m, qt, C4_POINTS, seed=72, order="shuffled")
    path = str(tmp_path / "cloud.npy")
    np.save(path, cloud)
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_c4_worker, args=(r, C4_RANKS, port, path, str(tmp_path), mode))
             for r in range(C4_RANKS)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    res = [dict(np.load(os.path.join(tmp_path, f"rank{r}.npz"))) for r in range(C4_RANKS)]
    assert res[0]["a"] == 0 and res[-1]["b"] == C4_POINTS
    assert all(res[r]["b"] == res[r + 1]["a"] for r in range(C4_RANKS - 1))
    # one context over the whole 10M cloud
    cf = CostFunctor(m, cloud)
    if mode == "exchange":  # (before any pass: the track! path regroups by itself)
        assert np.array_equal(np.concatenate([r["idx"] for r in res]), cf.ctx.permutation())
        assert max(len(r["idx"]) for r in res) <= 1.02 * C4_POINTS / C4_RANKS
    c1, g1 = cf.value_and_gradient(x)
    _, acc1, _ = cf._pass(x)
    k1, d1, gr1 = cf.per_point(x)
    for r in res:
        assert np.allclose(r["acc"], acc1, rtol=1e-9, atol=1e-9 * np.abs(acc1).max())
        assert r["c"] == pytest.approx(c1, rel=1e-9)
        assert np.allclose(r["g"], g1, rtol=1e-7, atol=1e-7 * np.abs(g1).max())
    idx = np.concatenate([r["idx"] for r in res])
    assert np.array_equal(np.sort(idx), np.arange(C4_POINTS))  # the shards partition the cloud
    k = np.empty_like(k1)
    d = np.empty_like(d1)
    gr = np.empty_like(gr1)
    k[idx] = np.concatenate([r["k"] for r in res])
    d[idx] = np.concatenate([r["d"] for r in res])
    gr[idx] = np.concatenate([r["gr"] for r in res])
    assert np.array_equal(k, k1) and np.array_equal(d, d1) and np.array_equal(gr, gr1)
    # cost = Σ d² over all 10M points (the reduction saw every shard once)
    assert c1 == pytest.approx(float(np.dot(d1, d1)), rel=1e-9)


def _c3_scene():
    import flash
    from flash import Models, synthetic
    bb = Models.beanbag()
    r = np.random.Generator(np.random.PCG64(5))  # examples/deformable_manipulator.ipynb:225-226, seeded
    x = np.zeros(flash.num_states(bb))
    x[:7] = bb.mechanism.zero_configuration()
    x[4:7] = 2 * r.random(3) ** 3
    x[7:] = 0.5 * (r.random(18) - 0.5)
    return bb, x, synthetic.skin_cloud(bb, x, 1 << 20, seed=6)


def _c3_poses(m, x):
    from flash.core import surface_poses
    return surface_poses(m, m.mechanism.normalize(x[:m.mechanism.num_positions]))


def _c3_eval(m, x, pts, precision, cull):
    from flash import _lib
    from flash import rbf as host_rbf
    c = _lib.Context(device=0, precision=precision, cull=cull, sort_points=True)
    c.set_surfaces([("rbf", len(s.surface_points) + len(s.skeleton_points)) for s in m.surfaces])
    c.set_points(pts)
    nq = m.mechanism.num_positions
    rows = host_rbf.rows(host_rbf.solve(m, m.mechanism.normalize(x[:nq]), x[nq:]))
    c.set_rbf_params(rows)
    out = c.eval(_c3_poses(m, x), per_point=True)
    c.close()
    return out, rows


def test_c3_beanbag_full_size_fp32(oracle_mod):
    m, x, pts = _c3_scene()
    assert len(pts) == 1 << 20
    (cost, acc, (k, d, g)), rows = _c3_eval(m, x, pts, 32, True)
    (cost_b, acc_b, (kb, db, gb)), _ = _c3_eval(m, x, pts, 32, False)
    assert np.array_equal(k, kb) and np.array_equal(d, db) and np.array_equal(g, gb)  # culled ≡ brute force
    assert np.all(k == 0) and np.all(np.isfinite(d))
    # the accumulator's cost is Σ d*² of the returned fp32 distances (f64 sums)
    assert cost == pytest.approx(float(np.dot(d, d)), rel=1e-9)
    assert acc[0] == cost
    # the fp64 oracle on a sample, and an fp64 context on every point
    sel = np.random.Generator(np.random.PCG64(7)).choice(len(pts), 20000, replace=False)
    om = oracle_mod.OracleModel.from_manipulator(m)
    od, ok, og = om.skin(_c3_poses(m, x), pts[sel], rbf_rows=rows)
    tol = 1e-4 * max(1.0, float(np.abs(od).max()))
    assert np.abs(d[sel] - od).max() < tol
    (cost64, _, (k64, d64, _)), _ = _c3_eval(m, x, pts, 64, True)
    assert np.abs(d - d64).max() < 1e-4 * max(1.0, float(np.abs(d64).max()))
    assert cost == pytest.approx(cost64, rel=1e-4)
    assert np.array_equal(d64[sel], od)  # the fp64 context is bit-exact with the oracle
    # ... and the fp32 context with the oracle's fp32 instantiation (oracle/skin_impl.h)
    od32, ok32, og32 = om.skin(_c3_poses(m, x), pts[sel], rbf_rows=rows, precision=32)
    assert np.array_equal(k[sel], ok32) and np.array_equal(d[sel], od32) and np.array_equal(g[sel], og32)


def test_exchange_ingest_one_rank_matches_set_points():
    """fsdf_cloud_box_device + fsdf_curve_keys_device + fsdf_set_points_keyed_device
    (exchange_points without a process group): the resident order and the
    per-point outputs of a sorted context's fsdf_set_points, bit for bit —
    also for a cloud whose slice arrives in another order."""
    import flash
    import torch
    from flash import Models, synthetic, _lib
    from flash.distributed import exchange_points
    m = Models.irb140()
    qt, qe = synthetic.perturbed_configuration(m, 81)
    cloud = synthetic.depth_cloud(m, qt, 300007, seed=82, order="shuffled")
    poses = flash.hull_poses(m, qe)
    spec = [(s.hull.vertices, s.hull.faces, s.hull.planes) for s in m.surfaces]
    a = _lib.Context(device=0, sort_points=True)
    a.set_model(spec)
    a.set_points(cloud)
    perm_a = a.permutation()
    a.set_output_order(True)
    _, acc_a, (ka, da, ga) = a.eval(poses, per_point=True)
    b = _lib.Context(device=0, sort_points=True)
    b.set_model(spec)
    rev = np.arange(len(cloud))[::-1].copy()  # the slice in reverse: the keyed order does not depend on it
    pts = torch.as_tensor(cloud[rev], device="cuda:0")
    idx = torch.as_tensor(rev, device="cuda:0")
    n_res, n_all = exchange_points([b], pts, idx)
    assert n_res == n_all == len(cloud)
    assert np.array_equal(b.permutation(), perm_a)
    b.set_output_order(True)
    _, acc_b, (kb, db, gb) = b.eval(poses, per_point=True)
    assert np.array_equal(ka, kb) and np.array_equal(da, db) and np.array_equal(ga, gb)
    assert np.array_equal(acc_a, acc_b)  # the same resident order: the same sums
    a.close()
    b.close()
