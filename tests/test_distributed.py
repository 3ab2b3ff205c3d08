"""The N>1 path on CPU: world_size-2 gloo ranks shard the cloud, compute their
local accumulators and all-reduce them; the result equals the 1-rank pass.
ShardedCostFunctor itself (sharding, in-place all-reduce, read-back, chain
rule) runs on CPU too, driving a stand-in engine whose passes are the oracle's
(the HIP engine is exercised by tests/test_gpu_distributed.py)."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    from conftest import ROOT
    for p in (os.path.join(ROOT, "point-cloud-signed-distance_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import flash
    from flash import Models, synthetic
    from flash.distributed import allreduce_accum, shard_range, chain_gradient
    import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = Models.irb140()
        qt, qe = synthetic.perturbed_configuration(m, 40)
        pts = synthetic.depth_cloud(m, qt, 3001, seed=41)
        a, b = shard_range(len(pts), rank, world)
        om = oracle.OracleModel.from_manipulator(m)
        local = torch.from_numpy(om.cost_accum(flash.hull_poses(m, qe), pts[a:b]))
        allreduce_accum(local)
        g = chain_gradient(m, qe, local.numpy(), 10)
        q.put((rank, local.numpy(), g))
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions():
    from flash.distributed import shard_range
    for n in (0, 1, 7, 64, 1000, 1 << 20):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))


def test_gloo_world2_allreduce_equals_single_rank():
    import multiprocessing as mp
    import flash
    from flash import Models, synthetic
    from flash.distributed import chain_gradient
    import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m = Models.irb140()
    qt, qe = synthetic.perturbed_configuration(m, 40)
    pts = synthetic.depth_cloud(m, qt, 3001, seed=41)
    full = oracle.OracleModel.from_manipulator(m).cost_accum(flash.hull_poses(m, qe), pts)
    for _, acc, g in res:
        assert np.allclose(acc, full, rtol=1e-11, atol=1e-12)
        assert np.allclose(g, chain_gradient(m, qe, full, 10), rtol=1e-10, atol=1e-12)
    assert np.array_equal(res[0][1], res[1][1])  # every rank holds the same sum


class OracleEngine:
    """Stand-in for the HIP context with the calls ShardedCostFunctor makes:
    host memory (device_type "cpu"), passes computed by the CPU oracle,
    accumulator and per-point outputs written through the raw pointers like
    fsdf_eval_device. Test infrastructure only."""
    device_type = "cpu"
    native_iterations = False

    def __init__(self, manip):
        import oracle
        self.om = oracle.OracleModel.from_manipulator(manip)
        self.accum_len = self.om.accum_len
        self.rows = None
        self.n = 0

    @staticmethod
    def _view(ptr, count, dtype):
        import ctypes
        buf = (ctypes.c_char * (count * np.dtype(dtype).itemsize)).from_address(ptr)
        return np.frombuffer(buf, dtype=dtype, count=count)

    def set_points_device(self, ptr, n):
        self.n = n
        self.pts = self._view(ptr, 3 * n, np.float64).reshape(n, 3).copy()
        self.perm = np.arange(n)

    @staticmethod
    def spatial_order(pts):
        """A deterministic spatial (Morton) order standing in for the device's Hilbert sort."""
        lo, hi = pts.min(0), pts.max(0)
        q = np.floor((pts - lo) / np.maximum(hi - lo, 1e-12) * 1023).astype(np.int64)
        key = np.zeros(len(pts), np.int64)
        for b in range(10):
            for a in range(3):
                key |= ((q[:, a] >> b) & 1) << (3 * b + a)
        return np.argsort(key, kind="stable")

    def set_points_range_device(self, ptr, n, begin, end):
        cloud = self._view(ptr, 3 * n, np.float64).reshape(n, 3).copy()
        order = self.spatial_order(cloud)
        self.perm = order[begin:end]
        self.order_pos, self.total = np.arange(begin, end), n
        self.pts = cloud[self.perm]
        self.n = end - begin

    def permutation(self):
        return self.perm.copy()

    # exchange shards (flash.distributed.exchange_points): box, keys, keyed resident order
    def cloud_box_device(self, ptr, n):
        pts = self._view(ptr, 3 * n, np.float64).reshape(n, 3)
        if n == 0:
            return np.array([np.inf] * 3 + [-np.inf] * 3)
        return np.concatenate([pts.min(0), pts.max(0)])

    def curve_keys_device(self, ptr, n, box, keys_ptr):
        """30-bit Morton keys in `box` (a stand-in for the device's Hilbert keys)."""
        pts = self._view(ptr, 3 * n, np.float64).reshape(n, 3)
        box = np.asarray(box)
        ext = box[3:] - box[:3]
        u = np.where(ext > 0, (pts - box[:3]) / np.where(ext > 0, ext, 1.0), 0.0)
        q = np.clip(np.floor(u * 1024.0), 0, 1023).astype(np.int64)
        key = np.zeros(n, np.int64)
        for b in range(10):
            for a in range(3):
                key |= ((q[:, a] >> b) & 1) << (3 * b + 2 - a)
        self._view(keys_ptr, n, np.int32)[:] = key

    def set_points_keyed_device(self, ptr, keys_ptr, idx_ptr, n):
        pts = self._view(ptr, 3 * n, np.float64).reshape(n, 3)
        keys = self._view(keys_ptr, n, np.int32).astype(np.int64)
        idx = self._view(idx_ptr, n, np.int64)
        order = np.lexsort((idx, keys))
        self.pts, self.perm, self.n = pts[order].copy(), idx[order].copy(), n
        self.keys = keys[order].copy()

    def set_plan(self, *a):
        pass

    def chunk_costs(self):
        """Deterministic per-chunk stand-in durations, uneven on purpose: chunks
        of the lower half of the cloud's order cost 1, of the upper half 9."""
        nc = -(-self.n // 64)
        return np.array([1.0 + 8.0 * (self.perm[64 * c] >= 0 and self.order_pos[64 * c] * 2 >= self.total)
                         for c in range(nc)])

    def set_rbf_params(self, rows):
        self.rows = np.asarray(rows, np.float64).copy()

    def eval_device(self, poses, accum_ptr, k_ptr=None, d_ptr=None, g_ptr=None):
        self._view(accum_ptr, self.accum_len, np.float64)[:] = self.om.cost_accum(poses, self.pts, rbf_rows=self.rows)
        if k_ptr:
            d, k, g = self.om.skin(poses, self.pts, rbf_rows=self.rows)
            self._view(k_ptr, self.n, np.int32)[:] = k
            self._view(d_ptr, self.n, np.float64)[:] = d
            self._view(g_ptr, 3 * self.n, np.float64)[:] = g.ravel()


def _scene(name):
    import flash
    from flash import Models, synthetic
    if name == "irb140":
        m = Models.irb140()
        qt, qe = synthetic.perturbed_configuration(m, 40)
        return m, synthetic.depth_cloud(m, qt, 3001, seed=41), qe
    m = Models.beanbag()  # RBF skin: the chain through the weight solve
    r = np.random.Generator(np.random.PCG64(43))
    x = np.zeros(flash.num_states(m))
    nq = m.mechanism.num_positions
    x[:nq] = m.mechanism.zero_configuration()
    x[4:7] = 0.05 * r.random(3)
    x[nq:] = 0.2 * (r.random(len(x) - nq) - 0.5)
    pts = r.normal(size=(1501, 3)) * 0.3
    return m, pts, x


def _functor_worker(rank, world, port, q, name):
    import sys
    from conftest import ROOT
    for p in (os.path.join(ROOT, "point-cloud-signed-distance_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from flash.distributed import ShardedCostFunctor, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m, pts, x = _scene(name)
        a, b = shard_range(len(pts), rank, world)
        f = ShardedCostFunctor(m, pts[a:b], rank, world, engine=OracleEngine(m))
        c, g = f.value_and_gradient(x)
        k, d, _ = f.per_point(x)
        q.put((rank, c, g, a, k, d))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["irb140", "beanbag_rbf"])
def test_gloo_world2_sharded_cost_functor(name):
    """ShardedCostFunctor on 2 gloo ranks == the same class on one rank (the
    whole cloud): cost and ∂c/∂x to 1e-10, every rank the same values, and the
    per-point outputs of the shards concatenate to the whole cloud's."""
    import multiprocessing as mp
    from flash.distributed import ShardedCostFunctor
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_functor_worker, args=(r, 2, port, q, name)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m, pts, x = _scene(name)
    one = ShardedCostFunctor(m, pts, engine=OracleEngine(m))
    c1, g1 = one.value_and_gradient(x)
    k1, d1, _ = one.per_point(x)
    for _, c, g, _, _, _ in res:
        assert c == pytest.approx(c1, rel=1e-10)
        assert np.allclose(g, g1, rtol=1e-9, atol=1e-10 * max(1.0, np.abs(g1).max()))
    assert res[0][1] == res[1][1] and np.array_equal(res[0][2], res[1][2])
    assert np.array_equal(np.concatenate([r[4] for r in res]), k1)
    assert np.array_equal(np.concatenate([r[5] for r in res]), d1)
    assert np.abs(g1).max() > 0


def _pipelined_worker(rank, world, port, q, name):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from flash.distributed import ShardedCostFunctor, shard_range
        m, pts, x = _scene(name)
        a, b = shard_range(len(pts), rank, world)
        f = ShardedCostFunctor(m, pts[a:b], rank, world, engine=OracleEngine(m))
        xs = [x + 1e-3 * i for i in range(4)]
        seq = [f.value_and_gradient(xi) for xi in xs]
        pip = f.value_and_gradient_many(xs)
        q.put((rank, seq, pip))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["irb140", "beanbag_rbf"])
def test_gloo_world2_pipelined_allreduce_same_bits(name):
    """value_and_gradient_many (the pass of x_{i+1} enqueued before the
    all-reduce of x_i is waited for; two accumulators, async collective) gives
    the same bits as one value_and_gradient per configuration, on 2 gloo ranks."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipelined_worker, args=(r, 2, port, q, name)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, seq, pip in res:
        assert len(seq) == len(pip) == 4
        for (c1, g1), (c2, g2) in zip(seq, pip):
            assert c1 == c2 and np.array_equal(g1, g2)
        assert len({c for c, _ in seq}) == 4  # the configurations differ


def test_spatial_bounds_partition_and_balance():
    from flash.distributed import spatial_bounds
    r = np.random.Generator(np.random.PCG64(5))
    for n in (0, 1, 63, 64, 65, 1000, 131072 + 7):
        for w in (1, 2, 3, 8):
            for costs in (None, r.random(-(-n // 64)) ** 4 if n else None):
                b = spatial_bounds(n, w, costs)
                assert len(b) == w and b[0][0] == 0 and b[-1][1] == n
                assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
                assert all(a % 64 == 0 or a == n for a, _ in b)
                if costs is not None and n:
                    per = [costs[a // 64:-(-e // 64)].sum() for a, e in b]
                    assert max(per) <= costs.sum() / w + costs.max() + 1e-9


def test_plan_window():
    """The planned pass's window for spatial shards (bench.py and
    ShardedCostFunctor share it): one rank keeps the default top, so the whole
    2^20 cloud runs unplanned; more ranks cover twice the average shard, and a
    rebalanced range 25 % past the average shard even above that top."""
    from flash.distributed import PLAN_TOP, plan_window
    n = 1 << 20
    assert plan_window(n, 1) == PLAN_TOP == 524288
    assert plan_window(n, 2) == 655360 and plan_window(n, 2) >= 530112  # round 5's rebalanced W = 2 range
    assert plan_window(n, 4) == 524288 and plan_window(n, 8) == 262144
    assert plan_window(1000, 8) == 98304 and plan_window(0, 1) == 98304
    for w in (2, 3, 4, 8, 16):
        assert plan_window(n, w) >= -(-n // w) * 5 // 4


def _spatial_worker(rank, world, port, q, name):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from flash.distributed import ShardedCostFunctor
        m, pts, x = _scene(name)
        f = ShardedCostFunctor(m, pts, rank, world, engine=OracleEngine(m), spatial=True)
        out = []
        for _ in range(2):  # equal chunk counts, then cost-balanced
            c, g = f.value_and_gradient(x)
            k, d, _ = f.per_point(x)
            out.append((list(f.bounds), c, g, f.global_index(), k, d))
            f.rebalance()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["irb140", "beanbag_rbf"])
def test_gloo_world2_spatial_shards(name):
    """Spatial shards (contiguous ranges of the cloud's spatial order, every
    rank given the whole cloud), before and after a cost-balancing rebalance():
    cost and ∂c/∂x equal the 1-rank functor's, and the per-point outputs placed
    at global_index() reproduce the whole cloud's."""
    import multiprocessing as mp
    from flash.distributed import ShardedCostFunctor
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_spatial_worker, args=(r, 2, port, q, name)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m, pts, x = _scene(name)
    one = ShardedCostFunctor(m, pts, engine=OracleEngine(m))
    c1, g1 = one.value_and_gradient(x)
    k1, d1, _ = one.per_point(x)
    bounds = [[o[0] for o in r[1]] for r in res]
    assert bounds[0] == bounds[1]  # every rank agrees on the ranges
    assert bounds[0][0] != bounds[0][1]  # the rebalance moved them (uneven stand-in costs)
    for step in range(2):
        k = np.full(len(pts), -1)
        d = np.zeros(len(pts))
        for _, out in res:
            b, c, g, idx, kk, dd = out[step]
            assert c == pytest.approx(c1, rel=1e-10)
            assert np.allclose(g, g1, rtol=1e-9, atol=1e-10 * max(1.0, np.abs(g1).max()))
            k[idx], d[idx] = kk, dd
        assert np.array_equal(k, k1) and np.array_equal(d, d1)


def _exchange_worker(rank, world, port, q, name):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from flash.distributed import ShardedCostFunctor, shard_range
        m, pts, x = _scene(name)
        # uneven slices of the caller's order: each rank uploads only its own
        cuts = [0, len(pts) // 5, (3 * len(pts)) // 4, len(pts)][:world] + [len(pts)]
        a, b = (cuts[rank], cuts[rank + 1]) if world == 3 else shard_range(len(pts), rank, world)
        eng = OracleEngine(m)
        f = ShardedCostFunctor(m, pts[a:b], rank, world, engine=eng, exchange=True)
        c, g = f.value_and_gradient(x)
        k, d, _ = f.per_point(x)
        q.put((rank, f.cloud_n, b - a, c, g, f.global_index(), k, d, int(eng.keys.min(initial=2**31)),
               int(eng.keys.max(initial=-1))))
        # a new frame (the same slice again): the same shards, the same bits
        f.set_sensed_points(pts[a:b])
        c2, _ = f.value_and_gradient(x)
        assert c2 == c
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_exchange_shards(world):
    """O(N/W) ingest (exchange_points): each rank uploads only its slice of
    the cloud; the ranks agree on the box, split the key range by an
    all-reduced histogram and exchange points over all_to_all. The shards
    partition the cloud into contiguous key ranges; cost and ∂c/∂x equal the
    1-rank functor's, and per-point outputs at global_index() reproduce it."""
    import multiprocessing as mp
    from flash.distributed import ShardedCostFunctor
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q, "irb140")) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m, pts, x = _scene("irb140")
    one = ShardedCostFunctor(m, pts, engine=OracleEngine(m))
    c1, g1 = one.value_and_gradient(x)
    k1, d1, _ = one.per_point(x)
    assert all(r[1] == len(pts) for r in res)
    k = np.full(len(pts), -1)
    d = np.zeros(len(pts))
    for _, _, _, c, g, idx, kk, dd, _, _ in res:
        assert c == pytest.approx(c1, rel=1e-10)
        assert np.allclose(g, g1, rtol=1e-9, atol=1e-10 * max(1.0, np.abs(g1).max()))
        k[idx], d[idx] = kk, dd
    assert np.array_equal(np.sort(np.concatenate([r[5] for r in res])), np.arange(len(pts)))
    assert np.array_equal(k, k1) and np.array_equal(d, d1)
    # contiguous key ranges in rank order, about N/W points each
    spans = [(r[8], r[9]) for r in res if len(r[5])]
    assert all(spans[i][1] <= spans[i + 1][0] for i in range(len(spans) - 1))
    assert max(len(r[5]) for r in res) <= 1.5 * len(pts) / world
