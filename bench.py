#!/usr/bin/env python3
"""Benchmark: SDF+grad point-evals/s, 1M-point cloud x 64-primitive model (M64).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config m64|c2|c4]
                    [--points P | --global-points G]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

A step is ONE residual pass of the hot path over the resident cloud: the pose
kernel (the 12·S pose doubles ride in its arguments), the pass kernel (per
point: nearest hull d*, k*, ∇d* written to HBM + the cost/wrench partial sums),
the fixed-order reduce kernel and, for N > 1, the RCCL all-reduce of the
1+6S-double accumulator. Steps run one pass at a time (the
headline `value`), as a track! iteration does; at N = 1 the line also carries
the dependent step (pass + accumulator read-back + host wait, every step) and,
labelled as such, the aggregate of two independent passes in flight
(config.inflight_throughput).

Sharding (contiguous point ranges, uploaded once per frame):
  (default)           weak scaling of the metric's cloud (`value`): every rank
                      its own 2^20-point M64 cloud (rank r seeded seed+17(r+1);
                      rank 0's is the N = 1 cloud), the 1+6S-double all-reduce
                      every step — the path partitions into independent point
                      ranges joined by that one collective. For W > 1 the strong
                      figure is measured in the same run and reported beside it
                      (`strong`): ONE 2^20-point cloud split into W spatial
                      shards — contiguous ranges of the whole cloud's Hilbert
                      order (fsdf_set_points_range), rebalanced after the settle
                      to equal measured chunk time — with the per-frame ingest
                      both ways (`config.ingest_per_frame`)
  --slice-shards      the strong side figure over slices of the caller's order (A/B)
  --points P          weak scaling only: every rank owns its own P-point cloud
  --global-points G   strong scaling only, of a G-point cloud
  --config c4         BASELINE config 4: IRB140, ONE 10·2^20-point cloud, strong
                      scaling (`value`), the weak figure beside it (`weak`)
For W > 1 the per-pass all-reduce is also timed on its own (`allreduce_ms`:
host-synchronised all-reduces of the accumulator, mean over `steps`), and the
backend that ran is named (`config.backend`).

Rank 0 prints one JSON line (contract in the task description) with:
  roofline      the pass kernel on the HBM roofline: algorithmic bytes per launch
                (24 B in + 36 B out per point) / its mean HIP-event
                time vs 8 TB/s; `traffic` = PMC bytes per launch of the committed
                profile (profiles/latest_pmc.json); `valu_issue_frac` = executed
                VALU wave-instructions (PMC) x 2 cycles / (1,024 SIMDs x 2.4 GHz x
                kernel time); the brute-force-equivalent F_alg rate is under
                `valu_effective` (it counts work the culling never executes)
  cpu_baseline  the C oracle on a bounded sample of the same cloud, on this
                host's cores: culled (sphere lower bounds, exact) as `value`,
                brute force (the reference's loop) beside it
  config        set-points (copy + Hilbert sort) per frame, a measured track!
                frame (pinned host cloud -> set_points -> fsdf_descend, 30
                iterations of estimate_state's default solver; device and host
                solver loops) and the full CostFunctor iteration (host FK + pass +
                accumulator read-back + chain rule), measured in the same run
  telemetry     the GPU's clocks, power and temperatures (sysfs / hipDeviceProp)
                at the start and end of the timed region
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
# FP64 vector: 256 CUs x 4 SIMD-32 x 2.4 GHz, wave64 FMA at 16 lanes/clk = AMD's 78.6 TF
FP64_VALU_PEAK_TFLOPS = 78.6
FP32_VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md
SIMDS, CLOCK_HZ, CYCLES_PER_WAVE_OP = 1024, 2.4e9, 2   # MI355X_MICROARCH.md §Wave scheduling
ITERS_PER_FRAME = 30           # src/tracking.jl:10-13 default NaiveSolver iteration_limit (manipulator.ipynb: 30)

SERIAL = {}  # run_cloud's serial re-run of the timed passes (one at a time)
SIDE_RES = {}  # run_cloud's N = 1 side figures (dependent step, passes in flight)
REGROUP_MS = None  # run_cloud's per-frame fsdf_regroup_points time (ms per context)
TELEMETRY = {}  # device_telemetry() at the start and the end of the timed region (first run_cloud)

CONFIGS = {
    # name: (model, default points, scaling, description)
    "m64": ("arm_grid", 1 << 20, "weak",
            "M64: 8 IRB140 arms (7 link hulls + ATI hull each) on a 2x4 grid, 64 convex hulls, 48 DOF; seeded "
            "synthetic depth cloud (SURVEY.md §8d generator G)"),
    "c2": ("irb140", 1 << 20, "weak", "C2: IRB140 rigid model (7 hulls, 6 DOF), 2^20 synthetic points"),
    "c4": ("irb140", 10 << 20, "strong", "C4: IRB140 rigid model, ONE 10*2^20-point cloud sharded over the GPUs"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--settle-ms", type=float, default=200.0,
                   help="untimed passes for this long before the W warmup steps: the GPU's clocks ramp up over "
                        "the first tens of ms of load (2^20 pass kernel 0.103 ms after 5 passes, 0.093 after 300, "
                        "profiles/r04/warmup_ab.txt)")
    p.add_argument("--inflight", type=int, default=1,
                   help="passes in flight in the timed region: C contexts over the same resident cloud, each on its "
                        "own HIP stream, step i on context i %% C (each context's results bit-identical to serial "
                        "steps; profiles/r04/inflight.jsonl). Default 1: one pass at a time, as a track! iteration "
                        "runs (each iteration needs the gradient of the one before)")
    p.add_argument("--inflight-side", type=int, default=2,
                   help="N = 1: after the timed region, also measure the aggregate throughput of this many "
                        "independent passes in flight (config.inflight_throughput; 0 = skip). Not the headline: "
                        "only independent configurations (line-search trials, several hypotheses) can overlap")
    p.add_argument("--accum-ring", type=int, default=2,
                   help="W > 1: accumulators per context in the timed loop (rounded up to even); a buffer is "
                        "reused only after its previous all-reduce completed, so a deeper ring leaves the pass "
                        "stream fewer waits on the collective stream")
    p.add_argument("--collective", default="torch", choices=("torch", "rccl"),
                   help="W > 1: the per-step all-reduce through torch.distributed (its own collective stream, "
                        "asynchronous, ordered by events) or RCCL itself in order on the pass's stream "
                        "(flash.distributed.RcclComm)")
    p.add_argument("--config", default="m64", choices=sorted(CONFIGS))
    g = p.add_mutually_exclusive_group()
    g.add_argument("--points", type=int, default=None, help="points per GPU (weak scaling)")
    g.add_argument("--global-points", type=int, default=None, help="one cloud split over the GPUs (strong scaling)")
    p.add_argument("--precision", type=int, default=64, choices=(64, 32))
    p.add_argument("--no-cull", action="store_true")
    p.add_argument("--order", default="shuffled", choices=("raster", "shuffled"),
                   help="input order of the synthetic cloud (shuffled = adversarial)")
    p.add_argument("--no-sort", action="store_true", help="keep the input order resident (no Hilbert sort)")
    p.add_argument("--no-per-point", action="store_true", help="reduction-only pass (no per-point outputs)")
    p.add_argument("--no-regroup", action="store_true",
                   help="keep the Hilbert resident order (no fsdf_regroup_points after the frame's first passes)")
    p.add_argument("--caller-order", action="store_true",
                   help="per-point outputs scattered to the caller's order (default: resident order, coalesced; "
                        "the permutation is fsdf_get_permutation)")
    p.add_argument("--cpu-seconds", type=float, default=8.0, help="target wall time of each CPU baseline leg")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-full-iteration", action="store_true")
    p.add_argument("--slice-shards", action="store_true",
                   help="W > 1 strong scaling: contiguous slices of the caller's (shuffled) order instead of ranges "
                        "of the whole cloud's Hilbert order (the round-4 partition; A/B)")
    p.add_argument("--seed", type=int, default=1234)
    return p.parse_args()


def cpu_baseline(manip, pts, q_eval, target_s):
    """Oracle (test infrastructure, the checker/baseline only) on a bounded
    sample: SURVEY.md §8d — culled and brute force, all host threads (the box's
    OpenMP share) and one thread, median of timed runs after a warm-up."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import statistics
    import flash
    import oracle
    om = oracle.OracleModel.from_manipulator(manip)
    poses = flash.hull_poses(manip, q_eval)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or 1))

    def rate(nt, per_run_s, runs, culled):
        n = 1024
        t = time.perf_counter()
        om.skin(poses, pts[:n], threads=nt, culled=culled)  # warm-up + sizing
        dt = time.perf_counter() - t
        n = int(min(len(pts), max(n, n * per_run_s / max(dt, 1e-6))))
        ts = []
        for _ in range(runs):
            t = time.perf_counter()
            om.skin(poses, pts[:n], threads=nt, culled=culled)
            ts.append(time.perf_counter() - t)
        return n, statistics.median(ts), sum(ts)

    n, med, tot = rate(threads, target_s / 5, 5, True)
    nb, medb, totb = rate(threads, target_s / 5, 5, False)
    n1, med1, _ = rate(1, 1.0, 3, True)
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": n / med, "unit": "point-evals/s", "cores": threads, "kind": "port",
            "brute_force_value": nb / medb, "single_thread_value": n1 / med1,
            "sample": f"first {n} points of rank 0's cloud, oracle with exact sphere-bound culling (same results "
                      f"as brute force), median of 5 runs ({tot:.1f} s wall) on {threads} threads; brute force over "
                      f"all {om.K} hulls (the reference's loop): {nb} points, median of 5 ({totb:.1f} s); "
                      f"culled on 1 thread: {n1} points, median of 3; host CPU: {model}"}


def device_telemetry(device):
    """The GPU's state where the host can read it: hipDeviceProp (CU count,
    peak engine / memory clock, PCI bus id) and, for the DRM card at that bus
    id (every card when it is unknown), the current DPM levels (pp_dpm_sclk /
    pp_dpm_mclk, the '*' line), power cap / draw and temperatures from hwmon.
    Fields the box does not expose are left out."""
    import ctypes
    import glob
    out = {}
    bus = None
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        for name, attr in (("cu_count", 63), ("clock_khz", 5), ("mem_clock_khz", 60)):  # hipDeviceAttribute_t
            v = ctypes.c_int(0)
            if hip.hipDeviceGetAttribute(ctypes.byref(v), attr, device) == 0:
                out[name] = v.value
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, device) == 0:
            bus = buf.value.decode().lower()
            out["pci_bus_id"] = bus
    except OSError:
        pass

    def read(p):
        try:
            with open(p) as f:
                return f.read().strip()
        except OSError:
            return None

    cards = []
    for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
        sclk = read(os.path.join(dev, "pp_dpm_sclk"))
        if sclk is None:
            continue
        rec = {"card": dev.split("/")[-2]}
        if bus is not None:  # this process's GPU only (a node's sysfs lists every card)
            if not os.path.realpath(dev).lower().endswith(bus):
                continue
        for key, fn in (("sclk", "pp_dpm_sclk"), ("mclk", "pp_dpm_mclk")):
            txt = read(os.path.join(dev, fn)) or ""
            cur = [ln.split(":", 1)[1].replace("*", "").strip() for ln in txt.splitlines() if ln.endswith("*")]
            if cur:
                rec[key] = cur[0]
        for hw in glob.glob(os.path.join(dev, "hwmon", "hwmon*")):
            for key, fn, scale in (("power_cap_w", "power1_cap", 1e-6), ("power_w", "power1_average", 1e-6),
                                   ("power_input_w", "power1_input", 1e-6)):
                v = read(os.path.join(hw, fn))
                if v and v.lstrip("-").isdigit():
                    rec[key] = round(int(v) * scale, 1)
            for tp in sorted(glob.glob(os.path.join(hw, "temp*_input"))):
                v = read(tp)
                lab = read(tp.replace("_input", "_label")) or os.path.basename(tp)
                if v and v.lstrip("-").isdigit():
                    rec["temp_" + lab + "_c"] = int(v) / 1000.0
        cards.append(rec)
    if cards:
        out["cards"] = cards
    return out


def full_iteration_ms(manip, ctx, q, iters=20):
    """One CostFunctor.value_and_gradient iteration on the resident cloud, as
    track! runs it for a rigid scene: fsdf_value_and_gradient = native FK +
    surface poses, the pass, accumulator read-back, chain rule to ∂c/∂q (the
    configuration moves every iteration)."""
    surf = manip.surfaces
    ctx.set_mechanism(manip.mechanism, [s.body for s in surf], [s.frame.R for s in surf], [s.frame.t for s in surf])
    x = np.array(q, np.float64)
    for i in range(iters + 3):
        if i == 3:
            t = time.perf_counter()
        x = x + 1e-6
        ctx.value_and_gradient(x)
    return (time.perf_counter() - t) / iters * 1e3


def measured_frame(manip, ctx, pts_host, q, torch, frames=5):
    """The reference's unit of tracking work, measured end to end: per frame
    the sensed cloud from pinned host memory -> fsdf_set_points (H2D + device
    Hilbert sort) -> fsdf_descend with estimate_state's default solver
    (NaiveSolver rate 0.1, max_step 0.5, 30 iterations, src/tracking.jl:12-15;
    tolerance 1e-3, flash/tracking.py) from q over c/N (src/tracking.jl:20);
    the library regroups after the frame's first pass by its own rule. The
    device solver loop (every iteration on the GPU, one read-back per frame)
    and, beside it, the host loop (one synchronisation per iteration). Median
    of `frames` frames after one untimed (allocations)."""
    import statistics
    surf = manip.surfaces
    ctx.set_mechanism(manip.mechanism, [s.body for s in surf], [s.frame.R for s in surf], [s.frame.t for s in surf])
    n = len(pts_host)
    pinned = torch.empty((n, 3), dtype=torch.float64, pin_memory=True)
    pinned.copy_(torch.from_numpy(np.ascontiguousarray(pts_host, np.float64)))
    host_pts = pinned.numpy()
    x0 = np.array(q, np.float64)

    def frame(device_loop):
        ctx.set_solver(device_loop)
        t0 = time.perf_counter()
        ctx.set_points(host_pts)
        t1 = time.perf_counter()
        x, f, its = ctx.descend(x0, ITERS_PER_FRAME, 0.1, 0.5, 1e-3, None, float(n))
        t2 = time.perf_counter()
        return (t2 - t0) * 1e3, (t1 - t0) * 1e3, its, f, x

    out = {}
    for name, dev_loop in (("device_loop", "require"), ("host_loop", False)):
        frame(dev_loop)
        rec = [frame(dev_loop) for _ in range(frames)]
        ms = statistics.median(r[0] for r in rec)
        sp = statistics.median(r[1] for r in rec)
        its = rec[0][2]
        out[name] = {"frame_ms": ms, "set_points_ms": sp, "iterations": its,
                     "ms_per_iteration": (ms - sp) / max(its, 1),
                     "tracking_point_evals_per_s": n * its / (ms / 1e3), "f": rec[0][3]}
    # a frame loop over queued clouds: frame t+1's upload (fsdf_prefetch_points,
    # page-locked, the context's copy stream) and sort run under frame t's
    # iterations, set_points_prefetched then swaps buffers (two pinned buffers
    # of the same cloud alternate; the library's default solver: the device loop)
    pinned2 = torch.empty((n, 3), dtype=torch.float64, pin_memory=True)
    pinned2.copy_(pinned)
    bufs = [host_pts, pinned2.numpy()]
    ctx.set_solver(True)
    ctx.prefetch_points(bufs[0])
    rec = []
    for f_ in range(frames + 1):
        t0 = time.perf_counter()
        ctx.set_points_prefetched()
        ctx.prefetch_points(bufs[(f_ + 1) & 1])
        t1 = time.perf_counter()
        x, fv, its = ctx.descend(x0, ITERS_PER_FRAME, 0.1, 0.5, 1e-3, None, float(n))
        t2 = time.perf_counter()
        if f_ > 0:  # (after one untimed frame)
            rec.append(((t2 - t0) * 1e3, (t1 - t0) * 1e3, its, fv))
    ctx.set_points_prefetched()  # (the trailing prefetch)
    ms = statistics.median(r[0] for r in rec)
    sp = statistics.median(r[1] for r in rec)
    out["device_loop_prefetched"] = {"frame_ms": ms, "set_points_ms": sp, "iterations": rec[0][2],
                                   "ms_per_iteration": (ms - sp) / max(rec[0][2], 1),
                                   "tracking_point_evals_per_s": n * rec[0][2] / (ms / 1e3), "f": rec[0][3],
                                   "note": "frame t+1's upload overlapping frame t's iterations "
                                           "(fsdf_prefetch_points / fsdf_set_points_prefetched, Tracker / track)"}
    a, b = out["device_loop"], out["host_loop"]
    out["same_result"] = bool(a["iterations"] == b["iterations"] and a["f"] == b["f"] and
                              out["device_loop_prefetched"]["f"] == b["f"])
    out["note"] = (f"{n} points, pinned host cloud -> set_points (H2D + sort) -> fsdf_descend(rate 0.1, max_step 0.5, "
                   f"{ITERS_PER_FRAME} iterations, tolerance 1e-3) from q_eval; median of {frames} frames; "
                   "device_loop: solver step on the GPU (solver.hip), host_loop: fsdf_set_solver(0)")
    ctx.set_solver(True)  # (the library's default)
    out["default"] = "device_loop"  # (fsdf_set_solver's default: the device loop for rigid scenes)
    out["frame_loop"] = "device_loop_prefetched"  # (what flash.tracking.track / Tracker.step(next_points) run)
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # FSDF_BENCH_BACKEND / FSDF_BENCH_DEVICE: rehearsal of the N>1 path on a
        # one-GPU box (gloo, every rank on one device); RCCL ("nccl") otherwise.
        # The device is set before the process group exists (RCCL binds to it)
        local = int(os.environ.get("FSDF_BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group(os.environ.get("FSDF_BENCH_BACKEND", "nccl"))
    elif os.environ.get("FSDF_BENCH_GROUP_AT_1"):
        # rehearsal of the W > 1 step loop on one GPU: an RCCL group of one rank,
        # so the timed steps take the grouped path (stream switch + asynchronous
        # all-reduce every step) and show its host cost against the device's
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29633", rank=0, world_size=1)
    dev = torch.device("cuda", local)
    backend = dist.get_backend() if dist.is_initialized() else None

    import flash
    from flash import Models, synthetic
    from flash._lib import FlashNativeError
    from flash.distributed import allreduce_accum, gather_chunk_costs, plan_window, shard_range, spatial_bounds

    model_name, default_points, scaling, workload = CONFIGS[args.config]
    if args.global_points is not None:
        scaling = "strong"
    elif args.points is not None:
        scaling = "weak"
    # W > 1 with the default workload. M64 / C2 (the metric's 1M-point cloud):
    # the headline is weak scaling — every rank its own 2^20-point cloud, the
    # pass's per-DOF all-reduce over the backend every step — and the strong
    # figure (ONE 2^20 cloud split into W spatial shards) is measured beside it;
    # C4 (ONE 10*2^20 cloud over the GPUs) is strong by definition, the weak
    # figure beside it
    explicit = args.points is not None or args.global_points is not None
    also_weak = world > 1 and not explicit and scaling == "strong"
    also_strong = world > 1 and not explicit and scaling == "weak"
    manip = getattr(Models, model_name)()
    q_true, q_eval = synthetic.perturbed_configuration(manip, args.seed)

    # strong scaling: every rank makes the same whole cloud and keeps a range of
    # its Hilbert order (spatial shards, rebalanced to equal measured chunk time
    # after the settle); --slice-shards: slices of the caller's (shuffled) order
    bounds = None

    def strong_shard(g):
        nonlocal bounds
        cloud = synthetic.depth_cloud(manip, q_true, g, seed=args.seed + 17, order=args.order)
        if world > 1 and not args.slice_shards:
            bounds = spatial_bounds(g, world)
            return cloud
        a, b = shard_range(g, rank, world)
        return np.ascontiguousarray(cloud[a:b])

    def weak_cloud(p):
        return synthetic.depth_cloud(manip, q_true, p, seed=args.seed + 17 * (rank + 1), order=args.order)

    if scaling == "strong":
        global_points = args.global_points if args.global_points is not None else default_points
        pts = strong_shard(global_points)
    else:
        p = args.points if args.points is not None else default_points
        pts = weak_cloud(p)
        global_points = p * world
    q_alt = q_eval + 1e-3  # alternate between two configurations step to step
    poses = [flash.hull_poses(manip, q_eval), flash.hull_poses(manip, q_alt)]

    C = max(1, args.inflight)
    SIDE = args.inflight_side if (world == 1 and args.inflight_side > 1) else 0
    CS = max(C, SIDE)  # contexts: the timed region uses the first C, the in-flight side figure the first SIDE
    ctxs = [manip.engine(device=local, precision=args.precision, cull=not args.no_cull,
                         sort_points=not args.no_sort, slot=c) for c in range(CS)]
    # every context on a stream of its own, none of them HIP's null stream (whose
    # implicit synchronisation would serialise the passes in flight); the first
    # is made torch's current stream, so the collectives and timing events order
    # after it
    streams = [torch.cuda.Stream(dev) for _ in range(CS)]
    stream_handles = [st_.cuda_stream for st_ in streams]
    RCCL = None
    if args.collective == "rccl" and dist.is_initialized():
        from flash.distributed import RcclComm
        RCCL = RcclComm()
    torch.cuda.set_stream(streams[0])
    stream = streams[0]
    for c, cx in enumerate(ctxs):
        cx.set_output_order(not args.caller_order)
        cx.set_stream(streams[c].cuda_stream)
    ctx = ctxs[0]
    # two accumulators per context (the all-reduce of one overlaps the next pass)
    RING = max(2, args.accum_ring + (args.accum_ring & 1))  # (even: a buffer always holds one configuration)
    accums = [[torch.zeros(ctx.accum_len, dtype=torch.float64, device=dev) for _ in range(RING)] for _ in range(CS)]
    h_acc = torch.empty(ctx.accum_len, dtype=torch.float64, pin_memory=True)
    accum = accums[0][0]

    def run_cloud(pts_host, shard_bounds=None):
        """Upload the cloud (timed per frame, every context), then W untimed + K
        timed steps bracketed by barrier + synchronize; returns the max-over-ranks
        (elapsed s, whole-pass ms, pass-kernel ms, set_points ms). shard_bounds:
        spatial shards — every context keeps this rank's range of the whole
        cloud's Hilbert order (fsdf_set_points_range), and after the settle the
        ranks rebalance the ranges to equal measured chunk time (the list is
        updated in place)."""
        d_pts = torch.as_tensor(pts_host, device=dev)
        torch.cuda.synchronize()

        if shard_bounds is not None:  # (flash.distributed.ShardedCostFunctor._plan_window: measured chunk costs)
            for cx in ctxs:
                cx.set_plan(True, -1.0, -1.0, plan_window(len(pts_host), world))

        def upload(cx):
            if shard_bounds is not None:
                cx.set_points_range_device(d_pts.data_ptr(), len(pts_host), *shard_bounds[rank])
            else:
                cx.set_points_device(d_pts.data_ptr(), len(pts_host))
        for cx in ctxs:  # (every context, the side figure's too)
            upload(cx)  # first upload (allocations)
        set_ms = []
        for _ in range(3):  # once per frame: copy (+ Hilbert sort), every context of the timed region
            t_set = time.perf_counter()
            for cx in ctxs[:C]:
                upload(cx)
            set_ms.append((time.perf_counter() - t_set) * 1e3)
        # (outputs sized for the whole cloud: a rebalance may grow this rank's range)
        n_ = len(pts_host)
        outs, bufs = [], []
        for _ in range(CS):
            if args.no_per_point:
                outs.append((0, 0, 0))
            else:
                b_ = (torch.empty(max(n_, 1), dtype=torch.int32, device=dev),
                      torch.empty(max(n_, 1), dtype=torch.float64, device=dev),
                      torch.empty((max(n_, 1), 3), dtype=torch.float64, device=dev))
                bufs.append(b_)
                outs.append(tuple(x.data_ptr() for x in b_))

        # step i: context i % C, its accumulator (i // C) & 1, configuration
        # (i // C) & 1. W > 1: an asynchronous all-reduce ordered after the
        # context's stream — step i+1's pass runs while step i's collective is
        # in flight (flash/distributed.py); a buffer is reused only after its
        # previous collective completed
        pending = [[None] * RING for _ in range(CS)]

        # (no process group — N = 1: no collective to order, and every context
        # is bound to its own stream by set_stream, so the step is the library
        # call alone; torch's stream switch cost ~5 us of host time per step,
        # enough to starve the device between 0.1 ms passes)
        acc_ptrs = [[accums[c][r_].data_ptr() for r_ in range(RING)] for c in range(CS)]
        grouped = dist.is_available() and dist.is_initialized()
        alen = ctx.accum_len

        def step(i, nctx=C):
            c, s_, r_ = i % nctx, (i // nctx) & 1, (i // nctx) % RING
            if not grouped:
                ctxs[c].eval_device(poses[s_], acc_ptrs[c][r_], *outs[c])
                return
            if RCCL is not None:  # in order on the context's stream: no waits, no events
                ctxs[c].eval_device(poses[s_], acc_ptrs[c][r_], *outs[c])
                RCCL.allreduce(acc_ptrs[c][r_], alen, stream_handles[c])
                return
            with torch.cuda.stream(streams[c]):
                if pending[c][r_] is not None:
                    pending[c][r_].wait()
                ctxs[c].eval_device(poses[s_], acc_ptrs[c][r_], *outs[c])
                pending[c][r_] = allreduce_accum(accums[c][r_], async_op=True)

        def drain():
            for c in range(CS):
                for r_ in range(RING):
                    if pending[c][r_] is not None:
                        with torch.cuda.stream(streams[c]):
                            pending[c][r_].wait()
                        pending[c][r_] = None

        def join(nctx=C):  # the first context's stream waits for every other context's stream
            for st in streams[1:nctx]:
                stream.wait_stream(st)

        # once per frame, after its first passes: the resident cloud regrouped by
        # each point's last nearest surface where the library's rule says it
        # pays (fsdf_regroup_auto: the pass ran one wave per chunk — the grid
        # above the planned window, bound by its summed work; the planned pass
        # and the hull-partitioned tiers are bound by their heaviest chunks,
        # which grouping makes heavier, profiles/r05/regroup/), timed and charged
        # to the frame beside set_points; before the settle (spatial shards:
        # after the rebalance, whose chunk costs must be the whole cloud's
        # Hilbert chunks), so every timed and profiled pass runs on the
        # regrouped cloud. The track! path (fsdf_descend, value_and_gradient)
        # applies the same rule by itself (measured_frame below).
        def regroup_all():
            if args.no_regroup:
                return None
            # (every context: the same pass, then the same regroup, so that their
            # resident orders — and the in-flight check's accumulators — agree;
            # the first regroup also grows the context's scratch, the second —
            # an explicit one, the rule having decided — is timed)
            ms = None
            for rep in range(2):
                for c in range(CS):
                    ctxs[c].eval_device(poses[0], accums[c][0].data_ptr(), *outs[c])
                torch.cuda.synchronize()
                t_r = time.perf_counter()
                if rep == 0:
                    applied = [cx.regroup_auto() for cx in ctxs]
                    if not all(applied):
                        assert not any(applied), "contexts over one cloud disagree on the regroup"
                        return None
                else:
                    for cx in ctxs:
                        cx.regroup_points()
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t_r) * 1e3 / CS
            for i in range(16 * CS):  # other chunks: their first passes plan and order anew
                c = i % CS
                ctxs[c].eval_device(poses[(i // CS) & 1], accums[c][(i // CS) & 1].data_ptr(), *outs[c])
            torch.cuda.synchronize()
            return ms

        global REGROUP_MS
        spatial = shard_bounds is not None and world > 1
        if not spatial:
            REGROUP_MS = regroup_all()
        # settle: untimed passes (no collectives: the ranks' counts differ) until
        # the clocks have ramped, wall-clock bound
        t_settle = time.perf_counter()
        i = 0
        while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
            c = i % C
            ctxs[c].eval_device(poses[(i // C) & 1], accums[c][(i // C) & 1].data_ptr(), *outs[c])
            i += 1
            if i % 16 == 0:
                torch.cuda.synchronize()
        if spatial:
            # rebalance: the ranks' measured per-chunk durations (the planned
            # pass's, in the whole cloud's chunk order — before any regroup)
            # all-gathered once; new ranges at equal summed chunk time, every
            # rank re-uploads its range; then the regroup
            torch.cuda.synchronize()
            costs = gather_chunk_costs(ctx.chunk_costs(), device=dev)
            if costs.shape[0] == -(-len(pts_host) // 64):
                shard_bounds[:] = spatial_bounds(len(pts_host), world, costs)
                for cx in ctxs:
                    upload(cx)
                for i in range(16 * C):  # a new range: its first passes plan anew
                    c = i % C
                    ctxs[c].eval_device(poses[(i // C) & 1], accums[c][(i // C) & 1].data_ptr(), *outs[c])
                torch.cuda.synchronize()
            REGROUP_MS = regroup_all()
        del d_pts
        # K passes one at a time on context 0 (no collective), right after the
        # settle: the kernel's own launch duration (the roofline's, as rocprofv3
        # sees it in tools/rocprof_round.sh) and one step's latency
        torch.cuda.synchronize()
        ctx.profile_pass(True)
        t_s = time.perf_counter()
        for i in range(args.steps):
            ctx.eval_device(poses[i & 1], accums[0][i & 1].data_ptr(), *outs[0])
        torch.cuda.synchronize()
        serial_step = (time.perf_counter() - t_s) / args.steps * 1e3
        k_, p_, l_ = ctx.pass_times()
        ctx.profile_pass(False)
        global SERIAL
        SERIAL = {"step_ms": serial_step, "kernel_ms": k_ / max(l_, 1), "pass_and_reduce_ms": p_ / max(l_, 1)}
        torch.cuda.synchronize()
        for i in range(args.warmup):
            step(i)
        drain()
        torch.cuda.synchronize()
        for cx in ctxs:
            cx.profile_pass(True)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        first_run = not TELEMETRY
        if first_run:
            TELEMETRY["timed_start"] = device_telemetry(local)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(stream)
        for i in range(args.steps):
            step(i)
        t_enq = time.perf_counter() - t0  # host time to enqueue the K steps (< the region: device-bound)
        drain()
        join()
        ev1.record(stream)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        if first_run:
            TELEMETRY["timed_end"] = device_telemetry(local)
        kernel_ms = pass_ms = 0.0
        launches = 0
        for cx in ctxs:
            k_, p_, l_ = cx.pass_times()
            kernel_ms, pass_ms, launches = kernel_ms + k_, pass_ms + p_, launches + l_
            cx.profile_pass(False)
        elapsed_ = max(wall, ev0.elapsed_time(ev1) / 1e3)
        # N = 1 side figures, after the timed region: (a) a dependent step — the
        # pass, then the accumulator read back to pinned host memory and the host
        # waits, every step (what a track! iteration pays besides its host FK and
        # chain rule); (b) SIDE independent passes in flight (aggregate throughput)
        global SIDE_RES
        SIDE_RES = {"host_enqueue_ms_per_step": t_enq / args.steps * 1e3}
        if world == 1:
            for i in range(3):
                ctx.eval_device(poses[i & 1], accums[0][i & 1].data_ptr(), *outs[0])
                h_acc.copy_(accums[0][i & 1], non_blocking=True)
                stream.synchronize()
            t_d = time.perf_counter()
            for i in range(args.steps):
                ctx.eval_device(poses[i & 1], accums[0][i & 1].data_ptr(), *outs[0])
                h_acc.copy_(accums[0][i & 1], non_blocking=True)
                stream.synchronize()
            SIDE_RES["dependent_step_ms"] = (time.perf_counter() - t_d) / args.steps * 1e3
        if SIDE > 1:
            for i in range(4 * SIDE):
                step(i, SIDE)
            drain()
            join(SIDE)
            torch.cuda.synchronize()
            t_f = time.perf_counter()
            for i in range(args.steps):
                step(i, SIDE)
            drain()
            join(SIDE)
            torch.cuda.synchronize()
            SIDE_RES["inflight_ms_per_pass"] = (time.perf_counter() - t_f) / args.steps * 1e3
            if args.steps >= 2 * SIDE:
                for c in range(1, SIDE):
                    for s_ in (0, 1):
                        assert torch.equal(accums[c][s_], accums[0][s_]), "in-flight contexts disagree"
        t = torch.tensor([elapsed_, pass_ms / max(launches, 1), kernel_ms / max(launches, 1),
                          float(np.median(set_ms))], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        # sanity: the last pass is finite and non-trivial; every context's
        # accumulators equal context 0's (the same configurations)
        acc = accums[0][0].cpu().numpy()
        assert np.isfinite(acc).all() and acc[0] > 0
        if args.steps >= 2 * C:
            for c in range(1, C):
                for s_ in (0, 1):
                    assert torch.equal(accums[c][s_], accums[0][s_]), "in-flight contexts disagree"
        return float(t[0]), float(t[1]), float(t[2]), float(t[3])

    elapsed, timed_pass_ms, timed_kernel_ms, set_points_ms = run_cloud(pts, bounds)
    n = ctx.n  # this rank's resident points
    serial = dict(SERIAL)
    side = dict(SIDE_RES)
    # the roofline prices the kernel alone on the device (its serial launches,
    # measured above with HIP events on its stream); with passes in flight each
    # launch shares the device with its neighbour and lasts longer
    kernel_avg_ms, pass_avg_ms = serial["kernel_ms"], serial["pass_and_reduce_ms"]

    allreduce_ms = None
    dependent_ms = side.get("dependent_step_ms")
    if world > 1:
        # a dependent iteration (track!: x_{k+1} needs the all-reduced accumulator
        # of x_k): pass, collective, host read-back, every step — the latency the
        # overlap above cannot hide
        outs0 = (0, 0, 0)
        for _ in range(3):
            ctx.eval_device(poses[0], accum.data_ptr(), *outs0)
            allreduce_accum(accum)
            accum[0].item()
        dist.barrier()
        t_dep = time.perf_counter()
        for i in range(args.steps):
            ctx.eval_device(poses[i & 1], accum.data_ptr(), *outs0)
            allreduce_accum(accum)
            accum[0].item()
        dependent_ms = (time.perf_counter() - t_dep) / args.steps * 1e3
        # the all-reduce alone, host-synchronised per call (latency-bound: ~3 KB)
        for _ in range(3):
            allreduce_accum(accum)
        torch.cuda.synchronize()
        t_ar = time.perf_counter()
        for _ in range(args.steps):
            allreduce_accum(accum)
            torch.cuda.synchronize()
        allreduce_ms = (time.perf_counter() - t_ar) / args.steps * 1e3

    # W > 1 spatial shards: the per-frame ingest, measured both ways on every rank
    # (max over ranks, median of 3 after one warm-up), from pinned host memory:
    # round 5's whole-cloud ranges (every rank uploads and sorts all N points,
    # fsdf_set_points_range) and round 6's exchanged shards (each rank uploads
    # its N/W slice; box all-reduce, keys, histogram splitters, one RCCL
    # all-to-all, keyed sort: flash.distributed.exchange_points)
    def measure_ingest(pts):
        from flash.distributed import exchange_points
        a, b = shard_range(len(pts), rank, world)
        whole = torch.empty((len(pts), 3), dtype=torch.float64, pin_memory=True)
        whole.copy_(torch.from_numpy(np.ascontiguousarray(pts)))
        cx = manip.engine(device=local, precision=args.precision, cull=not args.no_cull, sort_points=True, slot=CS)
        cx.set_stream(torch.cuda.current_stream().cuda_stream)

        def timed_max(fn, reps=4):
            ts = []
            for _ in range(reps):
                dist.barrier()
                torch.cuda.synchronize()
                t_ = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                tt = torch.tensor([(time.perf_counter() - t_) * 1e3], dtype=torch.float64, device=dev)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                ts.append(float(tt.item()))
            return float(np.median(ts[1:]))

        counts = []

        def exchange():
            d_sl = whole[a:b].to(dev, non_blocking=True)
            idx = torch.arange(a, b, dtype=torch.int64, device=dev)
            counts.append(exchange_points([cx], d_sl, idx)[0])

        ms_exchange = timed_max(exchange)
        ms_range = timed_max(lambda: cx.set_points_range(whole.numpy(), *bounds[rank]))
        nmax = torch.tensor([counts[-1]], dtype=torch.int64, device=dev)
        dist.all_reduce(nmax, op=dist.ReduceOp.MAX)
        rec = {"exchange_ms": ms_exchange, "whole_cloud_range_ms": ms_range,
                  "exchange_shard_points_max": int(nmax.item()), "slice_points": b - a,
                  "note": "per-frame ingest from pinned host memory, max over ranks: exchanged shards (N/W upload per "
                          "rank + box all-reduce + keys + histogram splitters + one all-to-all over the backend + "
                          "keyed sort) vs whole-cloud ranges (every rank uploads and sorts all N points)"}
        del whole
        return rec

    ingest = measure_ingest(pts) if world > 1 and bounds is not None else None

    weak = None
    if also_weak:
        del pts
        pts_w = weak_cloud(default_points)
        w_elapsed, w_pass, w_kernel, _ = run_cloud(pts_w)
        weak = {"value": default_points * world * args.steps / w_elapsed, "points_per_gpu": default_points,
                "global_points": default_points * world, "ms_per_step": w_elapsed / args.steps * 1e3,
                "pass_ms": w_pass, "pass_kernel_ms": w_kernel,
                "note": "weak scaling beside the strong value: every rank its own 2^20-point cloud"}

    strong = None
    if also_strong:
        del pts
        pts_s = strong_shard(default_points)  # (spatial: sets bounds; --slice-shards: this rank's slice)
        s_elapsed, s_pass, s_kernel, s_set = run_cloud(pts_s, bounds)
        n_s = torch.tensor([ctxs[0].n], dtype=torch.int64, device=dev)
        dist.all_reduce(n_s, op=dist.ReduceOp.MAX)
        strong = {"value": default_points * args.steps / s_elapsed, "global_points": default_points,
                  "points_per_gpu_max": int(n_s.item()), "ms_per_step": s_elapsed / args.steps * 1e3,
                  "pass_ms": s_pass, "pass_kernel_ms": s_kernel, "set_points_ms_per_frame": s_set,
                  "partition": ("spatial: contiguous ranges of the whole cloud's Hilbert order (fsdf_set_points_range), "
                                "rebalanced after the settle to equal measured chunk time" if bounds is not None else
                                "slices of the caller's order"),
                  "shard_bounds": bounds,
                  "note": "strong scaling beside the weak value: ONE 2^20-point cloud split over the W ranks"}
        if bounds is not None:
            ingest = measure_ingest(pts_s)

    iter_ms = frame_rec = None
    if rank == 0 and world == 1 and not args.no_full_iteration:
        ctx.set_stream(None)
        ctx.set_output_order(False)
        iter_ms = full_iteration_ms(manip, ctx, q_eval)
        frame_rec = measured_frame(manip, ctx, pts, q_eval, torch)

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = global_points * args.steps / elapsed
        tsz = 8 if args.precision == 64 else 4
        bytes_in = 3 * tsz * n
        bytes_per_launch = bytes_in + (0 if args.no_per_point else 36 * n)
        # per launch of the pass kernel, its own HIP events on the stream it runs on
        hbm_achieved = bytes_per_launch / (kernel_avg_ms / 1e3) / 1e9
        # F_alg per point-eval = Σ_hulls (21 + 7 F_k) + 15 (brute-force plane tests)
        f_alg = sum(21 + 7 * len(s.hull.faces) for s in manip.surfaces) + 15
        eff_tflops = f_alg * n / (kernel_avg_ms / 1e3) / 1e12
        peak_valu = FP64_VALU_PEAK_TFLOPS if args.precision == 64 else FP32_VALU_PEAK_TFLOPS
        traffic, traffic_src, executed, issue = None, None, None, None
        pmc = os.path.join(ROOT, "profiles", "latest_pmc.json")
        # the committed PMC profile is of the single-GPU default run only
        default_run = (world == 1 and args.config == "m64" and n == 1 << 20 and args.precision == 64
                       and not args.no_cull and not args.no_sort and not args.no_per_point
                       and args.order == "shuffled" and not args.caller_order)
        ran = ctx.pass_kernel_name()
        pmc_kernel = None
        if os.path.exists(pmc) and default_run:
            with open(pmc) as f:
                rec = json.load(f)
            pmc_kernel = rec.get("kernel", "").replace("fsdf::", "")
            # counters of another kernel variant (an older profile) are not this run's: refuse them
            if rec.get("workload") == "bench.py default" and pmc_kernel == ran:
                traffic, traffic_src = rec.get("traffic_bytes_per_launch"), rec.get("source")
                executed = rec.get("executed")
                if executed and executed.get("valu_insts_per_launch"):
                    issue = executed["valu_insts_per_launch"] * CYCLES_PER_WAVE_OP / (
                        SIMDS * CLOCK_HZ * kernel_avg_ms / 1e3)
        out = {
            "metric": "SDF+grad point-evals/sec, 1M-pt cloud x 64-prim model (M64)",
            "value": value,
            "unit": "point-evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_ms": args.settle_ms,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f64" if args.precision == 64 else "f32",
            "data": "synthetic",
            "config": {
                "workload": workload, "name": args.config,
                "points_per_gpu": n, "global_points": global_points, "surfaces": ctx.K,
                "dof": manip.mechanism.num_positions,
                "input_order": args.order, "sort_points": not args.no_sort,
                "cull": not args.no_cull, "per_point_outputs": not args.no_per_point,
                "output_order": "caller" if args.caller_order else "resident (+ permutation)",
                "parallelism": (f"points sharded x{world} ({scaling} scaling), {backend} all-reduce of "
                                f"{ctx.accum_len} f64 per pass" if world > 1 else
                                f"one GPU ({scaling} figure of the metric's cloud); at W > 1 one "
                                f"{ctx.accum_len}-f64 all-reduce per pass"),
                "partition": (None if world == 1 else "one cloud per rank" if scaling == "weak" else
                              "spatial: contiguous ranges of the whole cloud's Hilbert order (fsdf_set_points_range), "
                              "rebalanced after the settle to equal measured chunk time" if bounds is not None else
                              "slices of the caller's order"),
                "shard_bounds": bounds if scaling == "strong" else None,
                "backend": backend,
                "grouped_at_one_rank": (world == 1 and backend is not None) or None,
                "allreduce_ms": allreduce_ms,
                "allreduce_overlap": ("asynchronous all-reduce, two accumulators: step i+1's pass overlaps step "
                                      "i's collective" if world > 1 else None),
                "accum_ring": RING if (world > 1 or backend) else None,
                "collective": (args.collective if backend else None),
                "inflight": C,
                "inflight_note": (f"{C} independent passes in flight: {C} contexts over the same resident cloud, each on "
                                  f"its own HIP stream, step i on context i % {C} (two configurations alternate); every "
                                  f"context's accumulators checked equal" if C > 1 else
                                  "one pass at a time (the timed region), as a track! iteration runs"),
                "inflight_throughput": ({"passes_in_flight": SIDE, "ms_per_pass": side["inflight_ms_per_pass"],
                                         "value": global_points / (side["inflight_ms_per_pass"] / 1e3),
                                         "note": f"NOT the headline: {SIDE} independent passes in flight on {SIDE} "
                                                 "contexts / streams (two configurations alternating), measured after "
                                                 "the timed region; only independent configurations can overlap, a "
                                                 "dependent track! iteration cannot"}
                                        if "inflight_ms_per_pass" in side else None),
                "serial_step_ms": serial["step_ms"],
                "host_enqueue_ms_per_step": side.get("host_enqueue_ms_per_step"),
                "serial_step_note": "K passes one at a time on one context, untimed, before the timed region (no "
                                    "collective, per-point outputs written): one pass's latency",
                "dependent_step_ms": dependent_ms,
                "dependent_step_note": ("pass + all-reduce + host read-back per step, no overlap (a track! "
                                        "iteration's latency; no per-point outputs)" if world > 1 else
                                        "pass (per-point outputs written) + accumulator read back to pinned host "
                                        "memory + host wait, every step (a track! iteration's device latency; its "
                                        "host FK and chain rule are in full_iteration_ms)"),
                "set_points_ms_per_frame": set_points_ms,
                "ingest_per_frame": ingest,
                "measured_frame": frame_rec,
                "regroup_ms_per_frame": REGROUP_MS,
                "regroup_note": ("fsdf_regroup_auto once per frame after its first passes (the library's rule: the pass "
                                 "ran one wave per chunk): the resident cloud grouped by each point's last nearest "
                                 "surface (Hilbert order within a group); "
                                 "the timed passes run on it, seeded from the previous pass's k* (per-point results "
                                 "unchanged)" if REGROUP_MS is not None else "not applied (--no-regroup, the "
                                 "planned pass or a hull-partitioned tier, an RBF scene or an unsorted cloud)"),
                "full_iteration_ms": iter_ms,
                "full_iteration_note": "CostFunctor.value_and_gradient on the resident cloud (fsdf_value_and_gradient: "
                                       "host FK + surface poses, pass, accumulator read-back, chain rule; rank 0, "
                                       "N=1 only)",
            },
            "roofline": {
                "bound": "hbm", "achieved": hbm_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": hbm_achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                "kernel": ran, "kernel_ms": kernel_avg_ms,
                "kernel_ms_source": ("HIP events on the kernel's stream, K passes one at a time between the settle "
                                     "and the timed region (the kernel alone on the device, as in the committed "
                                     "rocprofv3 summary)"),
                # the pass kernel's mean HIP-event time inside the timed region (= kernel_ms
                # when passes run one at a time; longer with passes in flight)
                "kernel_ms_timed_region": timed_kernel_ms,
                # algorithmic bytes of all timed launches / the timed region
                "achieved_aggregate": bytes_per_launch * args.steps / elapsed / 1e9,
                "pass_and_reduce_ms": pass_avg_ms,
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "valu_issue_frac": issue,
                "executed_pmc": executed,
                "pmc_kernel": pmc_kernel,
            },
            # not a roofline fraction: the brute-force work the culling skips, per kernel time
            "valu_effective": {"flop_per_eval": f_alg, "achieved_tflops": eff_tflops, "peak_tflops": peak_valu,
                               "ratio": eff_tflops / peak_valu,
                               "note": "brute-force F_alg (every plane of every hull, SURVEY.md §8d) per launch / "
                                       "kernel time; culling skips most of it, so the ratio exceeds 1"},
        }
        out["telemetry"] = TELEMETRY
        if weak is not None:
            out["weak"] = weak
        if strong is not None:
            out["strong"] = strong
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(manip, pts, q_eval, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if RCCL is not None:
        RCCL.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
