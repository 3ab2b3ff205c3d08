#!/usr/bin/env python3
"""Hull-partitioned pass tiers against cloud size, per model (run on the GPU box).

For every size and every mode — the unplanned grid (fsdf_set_plan off) at a
forced tier (4 waves per chunk, 2, one wave per chunk; fsdf_set_partition) or
at the model's default tier, and the planned pass (the product default) — the
bench's step (pose + pass + reduce on the
resident, Hilbert-sorted cloud, per-point outputs written; two alternating
configurations) is timed, interleaved over rounds on one context, and the pass
kernel's own HIP-event time recorded; then the model's default tier and what
it picks. One JSON line per (size, tier); min over rounds.

    python tools/hpart_sweep.py --model irb140 --sizes 65536,131072,196608,262144,393216,524288
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))

# tier: (4-way limit, 2-way limit, planned pass) — the first three run the
# unplanned grid (fsdf_set_plan off) at a forced tier, "unplanned" at the
# model's default tier; "planned" forces the planned pass (per-chunk plan from
# measured durations, fsdf_set_plan) at every size; "default" is the product
# default (planned up to the model's size limit, unplanned above)
TIERS = {"4-way": (1 << 40, 0, False), "2-way": (0, 1 << 40, False), "one-wave": (0, 0, False),
         "unplanned": (-1, -1, False), "planned": (-1, -1, True), "default": (-1, -1, None)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="irb140", choices=("irb140", "arm_grid"))
    ap.add_argument("--sizes", default="65536,131072,196608,262144,393216,524288")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--tiers", default="", help="comma-separated subset of " + ",".join(TIERS))
    ap.add_argument("--four-share", type=float, default=-1.0, help="< 0: the library's default counts")
    ap.add_argument("--two-share", type=float, default=-1.0)
    ap.add_argument("--dump-costs", default="", help="npz path: the planned pass's per-chunk durations per size")
    a = ap.parse_args()
    import torch
    import flash
    from flash import Models, synthetic
    dev = torch.device("cuda", 0)
    m = getattr(Models, a.model)()
    qt, qe = synthetic.perturbed_configuration(m, a.seed)
    poses = [flash.hull_poses(m, qe), flash.hull_poses(m, qe + 1e-3)]
    ctx = m.engine(device=0, precision=64, cull=True, sort_points=True)
    ctx.set_output_order(True)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    accum = torch.zeros(ctx.accum_len, dtype=torch.float64, device=dev)
    dumps = {}
    for n in (int(s) for s in a.sizes.split(",")):
        pts = synthetic.depth_cloud(m, qt, n, seed=a.seed + 17, order="shuffled")
        d_pts = torch.as_tensor(pts, device=dev)
        ctx.set_points_device(d_pts.data_ptr(), n)
        bufs = (torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.float64, device=dev),
                torch.empty((n, 3), dtype=torch.float64, device=dev))
        outs = tuple(b.data_ptr() for b in bufs)
        best = {}
        for _ in range(a.rounds):
            for tier, (l4, l2, plan) in TIERS.items():
                if a.tiers and tier not in a.tiers.replace("+", ",").split(","):
                    continue
                ctx.set_partition(l4, l2)
                ctx.set_plan(plan is not False, a.four_share, a.two_share, -1 if plan is None else 1 << 30)
                for i in range(5):
                    ctx.eval_device(poses[i & 1], accum.data_ptr(), *outs)
                torch.cuda.synchronize()
                ctx.profile_pass(True)
                t0 = time.perf_counter()
                for i in range(a.steps):
                    ctx.eval_device(poses[i & 1], accum.data_ptr(), *outs)
                torch.cuda.synchronize()
                step = (time.perf_counter() - t0) / a.steps * 1e3
                kms, pms, launches = ctx.pass_times()
                ctx.profile_pass(False)
                row = best.setdefault(tier, {"step_ms": 1e9, "pass_kernel_ms": 1e9})
                row["step_ms"] = min(row["step_ms"], step)
                row["pass_kernel_ms"] = min(row["pass_kernel_ms"], kms / launches)
                row["kernel"] = ctx.pass_kernel_name()
        if a.dump_costs:
            ctx.set_partition(-1, -1)
            ctx.set_plan(True, 0.0, 0.0, 1 << 30)  # one wave per chunk: raw durations
            for i in range(3):
                ctx.eval_device(poses[i & 1], accum.data_ptr(), *outs)
            dumps[f"n{n}"] = ctx.chunk_costs()
        ctx.set_partition(-1, -1)
        ctx.set_plan(True)
        lim4, lim2, parts = ctx.get_partition(n)
        for tier, row in best.items():
            print(json.dumps({"model": a.model, "hulls": ctx.K, "points": n, "tier": tier, **row,
                              "shares": [a.four_share, a.two_share],
                              "default_limits": [lim4, lim2], "default_parts": parts}), flush=True)
        del d_pts, bufs
    if a.dump_costs:
        np.savez_compressed(a.dump_costs, **dumps)


if __name__ == "__main__":
    main()
