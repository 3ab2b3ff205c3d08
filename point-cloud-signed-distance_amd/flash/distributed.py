"""Point-sharded residual pass over several GPUs (one process per GPU).

The reference is single-threaded (no parallelism anywhere); its
cost is a plain sum over independent points (src/gradientdescent.jl:32) and k*
is per point, so the cloud shards trivially:
  * each rank holds a contiguous ⌈N/W⌉ slice of the cloud (uploaded once per frame);
  * every rank computes the same forward kinematics and ships the same K poses
    (no collective for parameters);
  * ONE all-reduce(sum, fp64) of the 1+6K accumulator per residual pass — over
    RCCL (torch.distributed backend "nccl") between GPUs, gloo on CPU tests.
The accumulator never leaves the device on the GPU path: fsdf_eval_device
writes it into a torch tensor that is all-reduced in place.

Overlap. The all-reduce is issued asynchronously (torch's RCCL stream waits
on the pass through an event; the compute stream does not wait for the
collective), and the functor keeps two accumulators, so the pass of the next
configuration runs while the previous one's all-reduce is in flight
(`value_and_gradient_many`, and bench.py's N > 1 step loop). A dependent
iteration (the NaiveSolver: x_{k+1} needs ∂c/∂x at x_k) cannot hide it —
there the host waits on the collective's completion only, not on a whole
stream synchronize. Results are bit-identical with and without the overlap:
every pass and every all-reduce sees the same inputs.
"""
from __future__ import annotations

import numpy as np

from ._lib import FlashNativeError

from .core import ConvexGeometry, Manipulator, ManipulatorState, prepare_pass
from .gradientdescent import (_regularizer, default_deformation_cost_weight, gradient_from_accum, native_capable,
                              normalize, register_native, unflatten)


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous slice [start, stop) of n points owned by `rank`."""
    per = -(-n // world)
    start = min(rank * per, n)
    return start, min(start + per, n)


CHUNK = 64  # points per wave-chunk of the pass (and per entry of fsdf_chunk_costs)
PLAN_TOP = 524288  # the planned pass's default window top for M64-class scenes (sdf_kernels.hip kPlanMaxFull)


def plan_window(n: int, world: int) -> int:
    """fsdf_set_plan max_points for a spatial shard of an n-point cloud over
    `world` ranks: the planned pass up to twice the average shard, also below
    the default window's 98,304-point bottom (its per-chunk durations are what
    rebalance() splits by; there it measured within 3 % of the unplanned 4-way
    tier). One rank keeps the default top (524,288: the
    whole 2^20 cloud runs the unplanned pass, whose step is shorter); more ranks
    let a rebalanced range grow 25 % past the average shard, also above that top
    — at two ranks a range of 530,112 points fell out of the window into the
    unplanned pass, 0.0643 ms against 0.0523 planned."""
    share = -(-n // max(world, 1))
    top = PLAN_TOP if world <= 1 else max(PLAN_TOP, -(-5 * share // 4))
    return int(min(max(2 * share, 98304), top))


def spatial_bounds(n: int, world: int, chunk_costs=None) -> list[tuple[int, int]]:
    """Shard ranges [begin, end) over a cloud's SPATIAL order (the device's
    Hilbert order, fsdf_set_points_range): contiguous, 64-point-chunk aligned,
    partitioning [0, n). Without costs every rank gets the same number of
    chunks; with `chunk_costs` (one per chunk of the whole cloud's order — the
    ranks' fsdf_chunk_costs concatenated) the boundaries split the prefix sum of
    the costs evenly, so each rank's summed chunk time is ~1/world of the
    total. A range of the spatial order is a compact region of space: its
    64-point chunks are as dense as the whole cloud's, where a slice of an
    arbitrary (e.g. shuffled) order gives every rank a sparse 1/world sample of
    the whole scene whose chunks each meet more hulls."""
    nc = -(-n // CHUNK)
    if world <= 1 or nc == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    if chunk_costs is None:
        w = np.ones(nc)
        w[-1] = (n - CHUNK * (nc - 1)) / CHUNK
    else:
        w = np.asarray(chunk_costs, np.float64).reshape(-1)
        if w.shape[0] != nc:
            raise ValueError(f"spatial_bounds: {w.shape[0]} chunk costs for {nc} chunks")
        w = np.maximum(w, 1e-9)
    cum = np.cumsum(w)
    cuts = [0]
    for r in range(1, world):
        c = int(np.searchsorted(cum, cum[-1] * r / world, side="left")) + 1  # first chunk of rank r
        cuts.append(min(max(c, cuts[-1]), nc))
    cuts.append(nc)
    return [(min(CHUNK * a, n), min(CHUNK * b, n)) for a, b in zip(cuts[:-1], cuts[1:])]


def gather_chunk_costs(local_costs, group=None, device=None) -> np.ndarray:
    """The ranks' per-chunk costs concatenated in rank order (the whole cloud's
    chunk order when the shards are spatial_bounds ranges): one all_gather of
    the padded arrays — a control-path collective, once per rebalance. device:
    the rank's GPU for an RCCL group (default: the current device)."""
    import torch
    import torch.distributed as dist
    local = np.asarray(local_costs, np.float64).reshape(-1)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return local
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    cnt = torch.tensor([local.shape[0]], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    m = int(max(int(c.item()) for c in cnts))
    buf = torch.zeros(max(m, 1), dtype=torch.float64, device=dev)
    buf[:local.shape[0]] = torch.from_numpy(local).to(dev)
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf, group=group)
    return np.concatenate([b[:int(c.item())].cpu().numpy() for b, c in zip(bufs, cnts)])


KEY_BITS = 30  # the device's curve keys (sort.hip: 10 bits per axis)


def exchange_points(ctxs, local_pts, local_index, group=None, bins_log2: int = 16):
    """O(N/W) ingest of one frame's cloud into spatial shards. Every rank holds
    a 1/W slice of the sensed cloud (`local_pts` [m,3] f64 tensor on the rank's
    device, `local_index` [m] int64: each point's index in the whole cloud):
      1. the whole cloud's bounding box: each slice's box (fsdf_cloud_box_device)
         and one 6-double all-reduce (MAX of (-lo, hi));
      2. each point's 30-bit Hilbert key in that box (fsdf_curve_keys_device —
         the keys a single context's sort_points orders by);
      3. splitters: a 2^bins_log2-bin histogram of the keys' top bits,
         all-reduced; rank r owns the bins where the cumulative count crosses
         r/W of the points — W contiguous key ranges of about N/W points;
      4. one all-to-all moves every point (xyz, key, whole-cloud index) to the
         rank owning its key;
      5. each context makes the received points resident in (key, whole-cloud
         index) order (fsdf_set_points_keyed_device): the single-context sorted
         order restricted to the rank's key range, the whole-cloud indices as
         the permutation.
    No rank ever holds more than its slice plus its shard: per-rank H2D and
    device sort are O(N/W) (the whole-cloud ranges of fsdf_set_points_range
    upload and sort all N points on every rank). A gloo group exchanges host
    copies (the CPU tests); RCCL exchanges device tensors over xGMI. Returns
    (this rank's resident count, the whole cloud's point count)."""
    import torch
    import torch.distributed as dist
    grouped = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if grouped else 1
    cdev = local_pts.device if (not grouped or dist.get_backend(group) == "nccl") else torch.device("cpu")
    ctx = ctxs[0]
    m = int(local_pts.shape[0])
    local_pts = local_pts.contiguous()
    box = ctx.cloud_box_device(local_pts.data_ptr(), m)
    t = torch.tensor(np.concatenate([-box[:3], box[3:]]), dtype=torch.float64, device=cdev)
    n_all = torch.tensor([m], dtype=torch.int64, device=cdev)
    if grouped:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        dist.all_reduce(n_all, op=dist.ReduceOp.SUM, group=group)
    t = t.cpu().numpy()
    gbox = np.concatenate([-t[:3], t[3:]])
    keys = torch.empty(max(m, 1), dtype=torch.int32, device=local_pts.device)
    ctx.curve_keys_device(local_pts.data_ptr(), m, gbox, keys.data_ptr())
    keys = keys[:m]
    if world == 1:
        recv_pts, recv_keys, recv_idx = local_pts, keys, local_index.to(torch.int64).contiguous()
    else:
        bins = (keys >> (KEY_BITS - bins_log2)).to(torch.int64).to(cdev)
        hist = torch.bincount(bins, minlength=1 << bins_log2)
        dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
        cum = torch.cumsum(hist, 0)
        total = int(cum[-1].item())
        targets = torch.tensor([total * r // world for r in range(1, world)], dtype=torch.int64, device=cdev)
        cuts = torch.searchsorted(cum, targets, right=True)  # first bin of ranks 1 .. W-1
        dest = torch.bucketize(bins, cuts, right=True)
        order = torch.argsort(dest, stable=True)
        send = torch.bincount(dest, minlength=world)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=group)
        sc, rc = send.tolist(), recv.tolist()
        nr = sum(rc)
        src_pts = local_pts.to(cdev)[order].contiguous()
        src_keys = keys.to(cdev)[order].contiguous()
        src_idx = local_index.to(cdev).to(torch.int64)[order].contiguous()
        recv_pts = torch.empty((nr, 3), dtype=torch.float64, device=cdev)
        recv_keys = torch.empty(nr, dtype=torch.int32, device=cdev)
        recv_idx = torch.empty(nr, dtype=torch.int64, device=cdev)
        dist.all_to_all_single(recv_pts.view(-1), src_pts.view(-1), [3 * c for c in rc], [3 * c for c in sc],
                               group=group)
        dist.all_to_all_single(recv_keys, src_keys, rc, sc, group=group)
        dist.all_to_all_single(recv_idx, src_idx, rc, sc, group=group)
        if cdev != local_pts.device:
            recv_pts, recv_keys, recv_idx = (recv_pts.to(local_pts.device), recv_keys.to(local_pts.device),
                                             recv_idx.to(local_pts.device))
    n_res = int(recv_pts.shape[0])
    for c in ctxs:
        c.set_points_keyed_device(recv_pts.data_ptr(), recv_keys.data_ptr(), recv_idx.data_ptr(), n_res)
    return n_res, int(n_all.item())


def allreduce_accum(accum, group=None, async_op=False):
    """Sum the per-rank accumulators in place (torch tensor, any device).
    async_op=True returns the collective's work handle (None without a process
    group): `.wait()` orders the caller's current stream (RCCL) or the host
    (gloo) after it. With a process group the collective runs at every world
    size, one rank included (the RCCL branch's stream ordering is then the one
    a multi-GPU run takes; tests/test_gpu_distributed.py::test_nccl_world1_pipelined)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        work = dist.all_reduce(accum, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
        return work if async_op else accum
    return None if async_op else accum


class RcclComm:
    """A communicator of RCCL itself (the librccl torch loads), whose sum
    all-reduce is enqueued on a HIP stream the caller names — in order with
    the pass on that stream, no collective stream and no cross-stream events
    (torch's ProcessGroupNCCL runs every collective on a stream of its own,
    ordered by an event each way). Built collectively over the process
    group: rank 0's ncclGetUniqueId is broadcast, every rank joins with
    ncclCommInitRank (the current HIP device)."""

    _lib = None

    @classmethod
    def _load(cls):
        if cls._lib is None:
            import ctypes
            import os
            import torch
            lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"))
            cls._Uid = type("ncclUniqueId", (ctypes.Structure,), {"_fields_": [("internal", ctypes.c_char * 128)]})
            lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(cls._Uid)]
            lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, cls._Uid, ctypes.c_int]
            lib.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_void_p]
            lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
            for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclCommDestroy"):
                getattr(lib, f).restype = ctypes.c_int
            cls._lib = lib
        return cls._lib

    def __init__(self, group=None):
        import ctypes
        import torch.distributed as dist
        lib = self._load()
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        uid = self._Uid()
        if rank == 0 and lib.ncclGetUniqueId(ctypes.byref(uid)) != 0:
            raise RuntimeError("ncclGetUniqueId failed")
        box = [bytes(uid.internal) if rank == 0 else None]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        uid.internal = box[0]
        self.comm = ctypes.c_void_p()
        if lib.ncclCommInitRank(ctypes.byref(self.comm), world, uid, rank) != 0:
            raise RuntimeError("ncclCommInitRank failed")

    def allreduce(self, ptr: int, count: int, stream: int) -> None:
        """In-place sum of `count` f64 at device pointer `ptr`, on HIP stream `stream` (0: the null stream)."""
        if self._lib.ncclAllReduce(ptr, ptr, count, 8, 0, self.comm, stream) != 0:  # ncclFloat64, ncclSum
            raise RuntimeError("ncclAllReduce failed")

    def close(self) -> None:
        if self.comm:
            self._lib.ncclCommDestroy(self.comm)
            self.comm = None


def chain_gradient(manip: Manipulator, x: np.ndarray, accum: np.ndarray, weight, solves=()) -> np.ndarray:
    """∂c/∂x from an (all-reduced) accumulator (see gradientdescent.gradient_from_accum)."""
    return gradient_from_accum(manip, np.asarray(x, np.float64), np.asarray(accum), list(solves), weight)


class ShardedCostFunctor:
    """CostFunctor over this rank's shard; value/gradient are global (all-reduced)."""

    def __init__(self, manipulator: Manipulator, local_points, rank: int = 0, world: int = 1, device: int = 0,
                 precision: int = 64, group=None, deformation_cost_weight=default_deformation_cost_weight,
                 engine=None, inflight: int = 1, spatial: bool = False, bounds=None, exchange: bool = False,
                 index_offset: int | None = None, collective: str = "torch"):
        """engine: an already-built context-like object to drive instead of
        manipulator.engine(device, precision) — with engine.device_type == "cpu"
        the accumulator lives in host memory and no HIP stream is used (the CPU
        gloo tests drive this class's sharding / all-reduce / read-back / chain
        rule through a stand-in engine; the product engine is the HIP context).
        inflight = 2 (HIP contexts only): a second context over the shard on a
        stream of its own (manipulator.engine(..., slot=1)) takes every other
        launch, so value_and_gradient_many's consecutive passes run together
        (bit-identical).
        spatial = True: `local_points` is the WHOLE cloud (every rank passes the
        same one) and this rank keeps range `bounds[rank]` (default
        spatial_bounds(n, world): equal chunk counts) of its spatial order
        (fsdf_set_points_range); rebalance() moves the boundaries to equal
        measured cost. Per-point outputs are then in the shard's resident
        order, global_index() names their indices in the whole cloud.
        exchange = True: O(N/W) ingest — `local_points` is only this rank's
        slice of the cloud (any split; index_offset = the whole-cloud index of
        its first point, default: the slices concatenated in rank order) and
        exchange_points() moves every point to the rank whose key range holds it
        (per-point outputs and global_index() as for spatial shards;
        set_sensed_points() swaps a new frame's slice in the same way).
        collective = "rccl" (HIP contexts over an RCCL group): each pass's
        all-reduce is RCCL itself, in order on the pass's stream (RcclComm) —
        no collective stream, no events; "torch" (default): torch.distributed's
        asynchronous all_reduce (profiles/r06/collective/). close() releases
        the RCCL communicator."""
        import contextlib
        import torch
        self.torch = torch
        self.manipulator = manipulator
        self.group = group
        self.weight = deformation_cost_weight
        self.state = ManipulatorState(manipulator)
        self.ctx = engine if engine is not None else manipulator.engine(device, precision)
        on_host = getattr(self.ctx, "device_type", "cuda") == "cpu"
        self.dev = torch.device("cpu") if on_host else torch.device("cuda", device)
        pts = torch.as_tensor(np.ascontiguousarray(local_points, np.float64).reshape(-1, 3), device=self.dev)
        self._pts = pts  # the context reads the resident copy (set_points_device does not own it)
        self.rank, self.world, self.spatial, self.exchange = rank, world, spatial and not exchange, exchange
        if collective not in ("torch", "rccl"):
            raise ValueError(f"collective: 'torch' or 'rccl', not {collective!r}")
        if collective == "rccl" and on_host:
            raise ValueError("collective='rccl' needs a HIP context")
        self._rccl = RcclComm(group) if collective == "rccl" else None
        self._index_offset = index_offset
        if exchange:
            self._exchange(pts)
        elif spatial:
            self.cloud_n = pts.shape[0]
            self.bounds = list(bounds) if bounds is not None else spatial_bounds(self.cloud_n, world)
            self.range = self.bounds[rank]
            self._plan_window(self.ctx)
            self.ctx.set_points_range_device(pts.data_ptr(), pts.shape[0], *self.range)
        else:
            self.ctx.set_points_device(pts.data_ptr(), pts.shape[0])
        # two accumulators: the next pass may run while the previous all-reduce is in flight
        self.accums = [torch.zeros(self.ctx.accum_len, dtype=torch.float64, device=self.dev) for _ in range(2)]
        self.accum = self.accums[0]
        self._slot = 0
        # pinned read-back of the all-reduced accumulator (a pageable .cpu()
        # goes through the runtime's staging buffer: ~10 us per iteration on
        # the single-GPU path, profiles/r02/experiments/r02pin)
        # (one per accumulator slot: value_and_gradient_many reads slot i's while slot i+1's pass runs)
        self.h_accums = [torch.empty(self.ctx.accum_len, dtype=torch.float64, pin_memory=not on_host)
                         for _ in range(2)]
        self.h_accum = self.h_accums[0]
        # the in-flight all-reduce of each accumulator slot: a slot is written
        # again (next launch, per_point) only after its collective completed
        self._pending = [None, None]
        if on_host:
            self.stream = None
            self._on_stream = lambda slot=0: contextlib.nullcontext()
            self._sync = lambda slot=0: None
            self.ctxs, self.streams = [self.ctx], [None]
        else:
            two = inflight > 1 and engine is None
            # (in flight: both contexts on streams of their own — HIP's null stream,
            # torch's default, would serialise their passes)
            self.stream = torch.cuda.Stream(self.dev) if two else torch.cuda.current_stream(self.dev)
            self.ctx.set_stream(self.stream.cuda_stream)
            self.ctxs, self.streams = [self.ctx], [self.stream]
            if two:
                c2 = manipulator.engine(device, precision, slot=1)
                s2 = torch.cuda.Stream(self.dev)
                c2.set_stream(s2.cuda_stream)
                self.ctxs.append(c2)
                if exchange:
                    self._exchange(pts)
                elif spatial:
                    self._plan_window(c2)
                    c2.set_points_range_device(pts.data_ptr(), pts.shape[0], *self.range)
                else:
                    c2.set_points_device(pts.data_ptr(), pts.shape[0])
                self.streams.append(s2)
            self._on_stream = lambda slot=0: torch.cuda.stream(self.streams[slot % len(self.streams)])
            self._sync = lambda slot=0: self.streams[slot % len(self.streams)].synchronize()
        # native iterations (fsdf_eval_state_device + fsdf_state_gradient: FK,
        # RBF solve, poses, pass; chain rule after the all-reduce)
        self._native = native_capable(manipulator) and getattr(self.ctx, "native_iterations", True)

    def _exchange(self, pts):
        """exchange_points() of this rank's slice `pts` into every context."""
        torch = self.torch
        m = int(pts.shape[0])
        off = self._index_offset
        if off is None:  # the slices in rank order: this rank's offset = the earlier ranks' sizes
            import torch.distributed as dist
            sizes = [m]
            if dist.is_available() and dist.is_initialized() and self.world > 1:
                cdev = self.dev if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
                t = torch.tensor([m], dtype=torch.int64, device=cdev)
                ts = [torch.zeros_like(t) for _ in range(self.world)]
                dist.all_gather(ts, t, group=self.group)
                sizes = [int(x.item()) for x in ts]
            off = sum(sizes[:self.rank])
        idx = torch.arange(off, off + m, dtype=torch.int64, device=self.dev)
        ctxs = getattr(self, "ctxs", [self.ctx])
        self.n_resident, self.cloud_n = exchange_points(ctxs, pts, idx, self.group)
        for c in ctxs:  # (the planned pass over shards of about cloud_n / world points)
            self._plan_window(c)

    def set_sensed_points(self, local_points):
        """A new frame's cloud (exchange shards: this rank's slice of it; spatial
        shards: the whole cloud, the ranges kept): the shards are rebuilt, the
        functor and the device model kept."""
        torch = self.torch
        for slot in (0, 1):
            self._wait_slot(slot)
        self._sync(0)
        pts = torch.as_tensor(np.ascontiguousarray(local_points, np.float64).reshape(-1, 3), device=self.dev)
        self._pts = pts
        if self.exchange:
            self._exchange(pts)
        elif self.spatial:
            self.cloud_n = pts.shape[0]
            for c in self.ctxs:
                c.set_points_range_device(pts.data_ptr(), pts.shape[0], *self.range)
        else:
            for c in self.ctxs:
                c.set_points_device(pts.data_ptr(), pts.shape[0])

    def _ensure_native(self, ctx=None):
        ctx = self.ctx if ctx is None else ctx
        if getattr(ctx, "_mechanism_of", None) != (self.manipulator, self.weight):
            register_native(self.manipulator, ctx, self.weight)

    def _wait_slot(self, slot):
        """Order the slot's stream (RCCL; gloo: the host) after the slot's
        pending all-reduce, which may still read its accumulator."""
        work = self._pending[slot]
        if work is not None:
            with self._on_stream(slot):
                work.wait()
            self._pending[slot] = None

    def launch(self, x, slot=None):
        """Enqueue one residual pass into accumulator `slot` (default: the
        other one than last time) and its all-reduce, asynchronously. Returns
        (slot, work); `finish` turns it into the host accumulator. A slot whose
        previous all-reduce is still in flight is waited for first (its
        accumulator is that collective's buffer)."""
        if slot is None:
            slot = self._slot ^ 1
        self._slot = slot
        self._wait_slot(slot)
        acc = self.accums[slot]
        ctx = self.ctxs[slot % len(self.ctxs)]  # (inflight: slot 1's passes on the second context)
        with self._on_stream(slot):
            if self._native:
                self._ensure_native(ctx)
                ctx.eval_state_device(np.asarray(x, np.float64), acc.data_ptr())
            else:
                unflatten(self.state, x)
                normalize(self.state)
                poses, self._solves = prepare_pass(ctx, self.manipulator, self.state.q,
                                                   self.state.deformation_data)
                ctx.eval_device(poses, acc.data_ptr())
            if self._rccl is not None:  # in order on this stream: nothing to wait for later
                self._rccl.allreduce(acc.data_ptr(), acc.numel(), self.streams[slot % len(self.streams)].cuda_stream)
                work = None
            else:
                work = allreduce_accum(acc, self.group, async_op=True)
        self._pending[slot] = work
        self.accum = acc
        return slot, work

    def finish(self, pending, out=None):
        """Wait for a launched pass's all-reduce and copy its accumulator to
        host memory (`out`, default the pinned buffer); the host blocks on
        this copy only."""
        slot, work = pending
        out = self.h_accums[slot] if out is None else out
        with self._on_stream(slot):
            if work is not None:
                work.wait()  # RCCL: the stream waits for the collective; gloo: the host does
            if self._pending[slot] is work:
                self._pending[slot] = None
            out.copy_(self.accums[slot], non_blocking=True)
            self._sync(slot)
        return out.numpy()

    def _gradient(self, x, acc, solves, slot=0):
        if self._native:
            ctx = self.ctxs[slot % len(self.ctxs)]  # the context that ran the pass (its FK / solve is current)
            self._ensure_native(ctx)
            return ctx.state_gradient(x, acc)  # (re-prepares x's FK / solve if a later pass was enqueued)
        unflatten(self.state, x)  # the state of THIS x (a pipelined later launch moved it)
        normalize(self.state)
        c = float(acc[0]) + _regularizer(self.state, self.weight)
        return c, chain_gradient(self.manipulator, x, acc, self.weight, solves)

    def _plan_window(self, ctx):
        """Spatial shards run the planned pass over plan_window()'s range."""
        if hasattr(ctx, "set_plan"):
            ctx.set_plan(True, -1.0, -1.0, plan_window(self.cloud_n, self.world))

    def global_index(self) -> np.ndarray:
        """The whole cloud's index of each resident point (spatial and exchange
        shards; for a plain shard its own caller order is resident, indices
        0..n-1 of it)."""
        return self.ctx.permutation()

    def rebalance(self):
        """Move the spatial shard boundaries so that every rank's summed chunk
        time (the planned pass's measured per-chunk durations, fsdf_chunk_costs,
        all-gathered once) is ~1/world of the total, and re-upload this rank's
        range. Call on every rank, after at least one pass over the current
        ranges. Returns the new bounds."""
        if not self.spatial:
            raise ValueError("rebalance: not a spatial shard")
        try:
            local = self.ctx.chunk_costs()
        except FlashNativeError:  # a regrouped range (its chunks are not the whole cloud's): keep the ranges
            local = np.zeros(0)
        # (every rank joins the all-gather; a short list on any rank keeps every rank's ranges)
        costs = gather_chunk_costs(local, self.group, device=None if self.dev.type == "cpu" else self.dev)
        nc = -(-self.cloud_n // CHUNK)
        if costs.shape[0] != nc:  # (no planned pass measured every chunk: keep the ranges)
            return self.bounds
        for slot in (0, 1):
            self._wait_slot(slot)
        self._sync(0)
        self.bounds = spatial_bounds(self.cloud_n, self.world, costs)
        self.range = self.bounds[self.rank]
        for c in self.ctxs:
            c.set_points_range_device(self._pts.data_ptr(), self.cloud_n, *self.range)
        return self.bounds

    def per_point(self, x):
        """(k*, d*, ∇d*) of this rank's shard at x, like CostFunctor.per_point (device
        outputs, caller order; a spatial shard: its resident order, global_index())."""
        torch = self.torch
        n = self.ctx.n
        k = torch.empty(max(n, 1), dtype=torch.int32, device=self.dev)
        d = torch.empty(max(n, 1), dtype=torch.float64, device=self.dev)
        g = torch.empty((max(n, 1), 3), dtype=torch.float64, device=self.dev)
        unflatten(self.state, x)
        normalize(self.state)
        poses, self._solves = prepare_pass(self.ctx, self.manipulator, self.state.q, self.state.deformation_data)
        self._wait_slot(0)  # accumulator 0 may still be read by its last all-reduce
        self._slot, self.accum = 0, self.accums[0]
        with self._on_stream(0):
            self.ctx.eval_device(poses, self.accum.data_ptr(), k.data_ptr(), d.data_ptr(), g.data_ptr())
            if self._rccl is not None:
                self._rccl.allreduce(self.accum.data_ptr(), self.accum.numel(), self.streams[0].cuda_stream)
            else:
                allreduce_accum(self.accum, self.group)
            return k[:n].cpu().numpy(), d[:n].cpu().numpy(), g[:n].cpu().numpy()

    def close(self):
        """Release the RCCL communicator (collective='rccl'); before the process group is destroyed."""
        if self._rccl is not None:
            self._sync(0)
            self._rccl.close()
            self._rccl = None

    def value_and_gradient(self, x):
        x = np.asarray(x, np.float64)
        pending = self.launch(x)
        acc = self.finish(pending)
        return self._gradient(x, acc, getattr(self, "_solves", ()), pending[0])

    def value_and_gradient_many(self, xs):
        """[(c, ∂c/∂x)] at independent configurations, pipelined: the pass at
        xs[i+1] is enqueued before the host waits for the all-reduce of xs[i],
        so the collective's latency hides behind the next pass. Bit-identical
        to [value_and_gradient(x) for x in xs]."""
        xs = [np.asarray(x, np.float64) for x in xs]
        out = []
        pending, solves = None, ()
        for x in xs:
            nxt = self.launch(x)  # the other accumulator than `pending`'s
            nxt_solves = getattr(self, "_solves", ())
            if pending is not None:
                xp, pp = pending  # (its own slot's pinned buffer: the other slot's pass is in flight)
                out.append(self._gradient(xp, self.finish(pp), solves, pp[0]))
            pending, solves = (x, nxt), nxt_solves
        if pending is not None:
            out.append(self._gradient(pending[0], self.finish(pending[1]), solves, pending[1][0]))
        return out
