#!/usr/bin/env python3
"""Strong-scaling shards of the bench cloud, each stepped alone on ONE GPU
(GPU box). For W = 1, 2, 4, 8 ranks the 2^20-point M64 bench
cloud (shuffled, as bench.py makes it) is split three ways:

  slice     contiguous slices of the caller's (shuffled) order — each rank a
            sparse 1/W sample of the whole scene, Hilbert-sorted on its own
            (the round-4 partition: bench.py / flash.distributed.shard_range);
  spatial   contiguous equal-count ranges of the whole cloud's Hilbert order
            (fsdf_set_points_range, flash.distributed.spatial_bounds);
  balanced  the same with boundaries at equal summed chunk time, from the
            per-chunk durations each rank's range measured under `spatial`
            (ShardedCostFunctor.rebalance's rule, the costs concatenated).

Per rank the serial step (pose + pass + reduce, one pass at a time, per-point
outputs written, the bench's two alternating configurations) and the pass
kernel (HIP events) are timed after a settle; one JSON line per (W, split)
with the max over ranks — the step a W-GPU strong-scaling run would wait for
(the all-reduce aside). A projection of the scaling curve, not a multi-GPU
measurement.

    python tools/spatial_shards.py [--ws 1,2,4,8] [--steps 40] > spatial_shards.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ws", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--points", type=int, default=1 << 20)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--splits", default="slice,spatial,balanced")
    ap.add_argument("--no-plan", action="store_true", help="unplanned pass at every shard size (fsdf_set_plan off)")
    ap.add_argument("--regroup", action="store_true",
                    help="fsdf_regroup_points after each shard's first passes (spatial splits)")
    a = ap.parse_args()
    import torch
    import flash
    from flash import Models, synthetic
    from flash.distributed import plan_window, shard_range, spatial_bounds
    dev = torch.device("cuda", 0)
    m = Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m, a.seed)
    poses = [flash.hull_poses(m, qe), flash.hull_poses(m, qe + 1e-3)]
    cloud = synthetic.depth_cloud(m, qt, a.points, seed=a.seed + 17, order="shuffled")
    n = len(cloud)
    d_cloud = torch.as_tensor(cloud, device=dev)
    ctx = m.engine(device=0, precision=64, cull=True, sort_points=True)
    ctx.set_output_order(True)
    if a.no_plan:
        ctx.set_plan(False)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    acc = torch.zeros(ctx.accum_len, dtype=torch.float64, device=dev)
    bufs = [torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.float64, device=dev),
            torch.empty((n, 3), dtype=torch.float64, device=dev)]
    outs = [b.data_ptr() for b in bufs]
    t0 = time.perf_counter()
    ctx.set_points_device(d_cloud.data_ptr(), n)
    while time.perf_counter() - t0 < 0.3:  # clocks settle
        ctx.eval_device(poses[0], acc.data_ptr(), *outs)
        torch.cuda.synchronize()

    def load(split, bounds, r):
        b, e = bounds[r]
        if split == "slice":
            if not a.no_plan:  # (the model's default window, as bench.py's --slice-shards)
                ctx.set_plan(True, -1.0, -1.0, -1)
            sl = torch.as_tensor(np.ascontiguousarray(cloud[b:e]), device=dev)
            ctx.set_points_device(sl.data_ptr(), e - b)
        else:
            if not a.no_plan:  # (the window bench.py and ShardedCostFunctor give spatial shards)
                ctx.set_plan(True, -1.0, -1.0, plan_window(n, len(bounds)))
            ctx.set_points_range_device(d_cloud.data_ptr(), n, b, e)

    def step_rank(regroup=False):
        for i in range(8):  # first pass (tier shape), plan, planned passes
            ctx.eval_device(poses[i & 1], acc.data_ptr(), *outs)
        torch.cuda.synchronize()
        # the chunk costs of the range in the whole cloud's Hilbert chunk order —
        # before any regroup, which permutes the chunks (round-5 advice: costs
        # read after the regroup mis-placed the balanced cuts)
        pre_costs = ctx.chunk_costs()
        if regroup:
            ctx.regroup_points()
            for i in range(8):  # other chunks: plan anew
                ctx.eval_device(poses[i & 1], acc.data_ptr(), *outs)
            torch.cuda.synchronize()
        best = (1e9, 1e9)
        for _ in range(a.rounds):
            ctx.profile_pass(True)
            ts = time.perf_counter()
            for i in range(a.steps):
                ctx.eval_device(poses[i & 1], acc.data_ptr(), *outs)
            torch.cuda.synchronize()
            step = (time.perf_counter() - ts) / a.steps * 1e3
            kms, _, launches = ctx.pass_times()
            ctx.profile_pass(False)
            best = (min(best[0], step), min(best[1], kms / max(launches, 1)))
        return best, pre_costs

    for w in (int(x) for x in a.ws.split(",")):
        eq_costs = None
        for split in a.splits.split(","):
            if split == "slice":
                bounds = [shard_range(n, r, w) for r in range(w)]
            elif split == "spatial":
                bounds = spatial_bounds(n, w)
            else:
                if eq_costs is None or w == 1:
                    continue
                bounds = spatial_bounds(n, w, eq_costs)
            steps, kernels, costs, kinds = [], [], [], []
            for r in range(w):
                load(split, bounds, r)
                (s, k), cc = step_rank(a.regroup and split != "slice")
                steps.append(s)
                kernels.append(k)
                kinds.append(ctx.pass_kernel_name())
                costs.append(cc)
            if split == "spatial":
                cat = np.concatenate(costs).astype(np.float64)
                if cat.shape[0] == -(-n // 64):
                    eq_costs = cat
            heavy = [float(c.max()) / 100.0 if len(c) else None for c in costs]
            summed = [float(c.sum()) / 100.0 if len(c) else None for c in costs]
            print(json.dumps({"W": w, "split": split, "points": n, "max_step_ms": max(steps),
                              "max_kernel_ms": max(kernels), "step_ms": steps, "kernel_ms": kernels,
                              "bounds": bounds, "heaviest_chunk_us": heavy, "summed_chunk_us": summed,
                              "kernels": sorted(set(kinds)), "planned": not a.no_plan, "regroup": a.regroup,
                              "projected_value": n / (max(steps) / 1e3)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
