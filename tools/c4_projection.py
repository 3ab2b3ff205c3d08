#!/usr/bin/env python3
"""BASELINE config 4 (ONE 10·2^20-point IRB140 cloud over W GPUs) as a
projection from ONE GPU (GPU box). For W = 1, 2, 4, 8
every rank's share of the work is run alone on the one GPU, and the line per W
carries the max over ranks — what a W-GPU run would wait for:

  per pass   each rank's shard (a contiguous Hilbert-key range of the whole
             cloud, the shards exchange_points builds: equal point counts)
             stepped one pass at a time (pose + pass + reduce, per-point outputs
             written) after a settle — pass_ms = the max step;
  per frame  the ingest a frame costs each rank, two ways:
             whole-cloud ranges (round 5, fsdf_set_points_range): every rank
               uploads the WHOLE cloud from pinned host memory and sorts all N
               points — measured;
             exchange (round 6, flash.distributed.exchange_points): the rank
               uploads only its N/W slice (pinned H2D), boxes and keys it, and
               makes its received shard resident (keyed sort of N/W points) —
               measured; the all-to-all in between moves ~(W-1)/W of the
               rank's slice (xyz + key + index = 36 B a point) over xGMI: NOT
               measurable on one GPU, reported as bytes and as an estimate at a
               stated per-GPU all-to-all bandwidth (--a2a-gbs).
  frame_ms   ingest + 30 passes (estimate_state's default iteration_limit).

    python tools/c4_projection.py [--ws 1,2,4,8] [--points 10485760] > c4_projection.jsonl
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ws", default="1,2,4,8")
    ap.add_argument("--points", type=int, default=10 << 20)
    ap.add_argument("--model", default="irb140", choices=("irb140", "m64"))
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--a2a-gbs", type=float, default=50.0,
                    help="assumed all-to-all bandwidth per GPU (GB/s, each direction) for the exchange estimate")
    a = ap.parse_args()
    import torch
    import flash
    from flash import Models, synthetic
    from flash.distributed import KEY_BITS, plan_window
    dev = torch.device("cuda", 0)
    m = Models.irb140() if a.model == "irb140" else Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m, a.seed)
    poses = [flash.hull_poses(m, qe), flash.hull_poses(m, qe + 1e-3)]
    cloud = synthetic.depth_cloud(m, qt, a.points, seed=a.seed + 17, order="shuffled")
    n = len(cloud)
    pinned = torch.empty((n, 3), dtype=torch.float64, pin_memory=True)
    pinned.copy_(torch.from_numpy(cloud))
    ctx = m.engine(device=0, precision=64, cull=True, sort_points=True)
    ctx.set_output_order(True)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    acc = torch.zeros(ctx.accum_len, dtype=torch.float64, device=dev)
    bufs = [torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.float64, device=dev),
            torch.empty((n, 3), dtype=torch.float64, device=dev)]
    outs = [b.data_ptr() for b in bufs]
    d_cloud = pinned.to(dev, non_blocking=True)
    torch.cuda.synchronize()
    # the whole cloud's keys (global box) once: the shards every W builds
    box = ctx.cloud_box_device(d_cloud.data_ptr(), n)
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    ctx.curve_keys_device(d_cloud.data_ptr(), n, box, keys.data_ptr())
    bins = (keys >> (KEY_BITS - 16)).to(torch.int64)
    cum = torch.cumsum(torch.bincount(bins, minlength=1 << 16), 0)
    index = torch.arange(n, dtype=torch.int64, device=dev)
    t0 = time.perf_counter()
    ctx.set_points_device(d_cloud.data_ptr(), n)
    while time.perf_counter() - t0 < 0.3:  # clocks settle
        ctx.eval_device(poses[0], acc.data_ptr(), *outs)
        torch.cuda.synchronize()

    def timed(fn, reps=a.reps):
        ts = []
        for _ in range(reps + 1):
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        return statistics.median(ts[1:])

    def step_rank():
        for i in range(8):  # first pass (tier shape), plan, planned passes
            ctx.eval_device(poses[i & 1], acc.data_ptr(), *outs)
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for i in range(a.steps):
            ctx.eval_device(poses[i & 1], acc.data_ptr(), *outs)
        torch.cuda.synchronize()
        return (time.perf_counter() - ts) / a.steps * 1e3

    for w in (int(x) for x in a.ws.split(",")):
        targets = torch.tensor([n * r // w for r in range(1, w)], dtype=torch.int64, device=dev)
        cuts = torch.searchsorted(cum, targets, right=True)
        dest = torch.bucketize(bins, cuts, right=True)
        steps, ingest_range, ingest_exch, a2a_bytes, sizes = [], [], [], [], []
        for r in range(w):
            sel = torch.nonzero(dest == r).flatten()
            sh_pts, sh_keys, sh_idx = d_cloud[sel].contiguous(), keys[sel].contiguous(), index[sel].contiguous()
            ns = int(sel.numel())
            sizes.append(ns)
            ctx.set_plan(True, -1.0, -1.0, plan_window(n, w))
            # ingest, round 5: the whole cloud from pinned host memory, sorted, a range kept
            b0, e0 = (0, ns)  # (any range of the size: the cost is the whole-cloud upload + sort)
            ingest_range.append(timed(lambda: ctx.set_points_range(pinned.numpy(), b0, e0)))
            # ingest, round 6: the rank's slice H2D + box + keys, then its shard resident
            s0, s1 = n * r // w, n * (r + 1) // w
            sl_host = pinned[s0:s1]
            sl_dev = torch.empty((s1 - s0, 3), dtype=torch.float64, device=dev)
            sl_keys = torch.empty(max(s1 - s0, 1), dtype=torch.int32, device=dev)

            def slice_part():
                sl_dev.copy_(sl_host, non_blocking=True)
                torch.cuda.synchronize()
                bx = ctx.cloud_box_device(sl_dev.data_ptr(), s1 - s0)
                ctx.curve_keys_device(sl_dev.data_ptr(), s1 - s0, bx, sl_keys.data_ptr())

            t_slice = timed(slice_part)
            t_keyed = timed(lambda: ctx.set_points_keyed_device(sh_pts.data_ptr(), sh_keys.data_ptr(),
                                                                  sh_idx.data_ptr(), ns))
            ingest_exch.append((t_slice, t_keyed))
            # bytes this rank sends: its slice's points owned by other ranks (36 B each)
            own = int(((dest[s0:s1] == r)).sum().item())
            a2a_bytes.append(36 * ((s1 - s0) - own))
            steps.append(step_rank())
        pass_ms = max(steps)
        exch_meas = max(t + k for t, k in ingest_exch)
        a2a_ms = max(a2a_bytes) / (a.a2a_gbs * 1e9) * 1e3
        rec = {"W": w, "model": a.model, "points": n, "shard_points": sizes,
               "pass_ms": pass_ms, "step_ms": steps, "projected_pass_value": n / (pass_ms / 1e3),
               "ingest_whole_cloud_range_ms": max(ingest_range),
               "ingest_exchange_measured_ms": exch_meas,
               "ingest_exchange_parts_ms": [[round(t, 4), round(k, 4)] for t, k in ingest_exch],
               "a2a_bytes_per_rank_max": max(a2a_bytes), "a2a_ms_estimate": a2a_ms,
               "a2a_assumed_gbs": a.a2a_gbs,
               "frame_ms_whole_cloud_range": max(ingest_range) + a.steps * pass_ms,
               "frame_ms_exchange": exch_meas + a2a_ms + a.steps * pass_ms,
               "note": "projection from one GPU: every rank's shard stepped alone, max over ranks; the all-to-all is "
                       "an estimate (bytes / assumed bandwidth), not measured"}
        print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
