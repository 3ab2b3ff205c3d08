#!/usr/bin/env python3
"""The bench step (pose -> pass -> reduce, fsdf_eval_device) launched eagerly
against the same launches captured into a HIP graph and replayed (GPU box).
M64, 2^20 points, resident-order per-point outputs, two configurations
alternating as in bench.py. Answers whether a graph shortens the per-step
launch chain (the launches' own durations are what they are; a graph can only
remove host submission and inter-launch gaps).

    python tools/graph_probe.py [--points N] [--steps K]
"""
import argparse
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    import flash
    from flash import Models, synthetic
    m = Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m, 1234)
    poses = [flash.hull_poses(m, qe), flash.hull_poses(m, qe + 1e-3)]
    pts = synthetic.depth_cloud(m, qt, a.points, seed=1234 + 17, order="shuffled")
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    ctx = m.engine(device=0, sort_points=True)
    ctx.set_stream(s.cuda_stream)
    ctx.set_points(pts)
    ctx.set_output_order(True)
    n = ctx.n
    acc = [torch.zeros(ctx.accum_len, dtype=torch.float64, device=dev) for _ in range(2)]
    k = torch.empty(n, dtype=torch.int32, device=dev)
    d = torch.empty(n, dtype=torch.float64, device=dev)
    g = torch.empty(3 * n, dtype=torch.float64, device=dev)
    outs = (k.data_ptr(), d.data_ptr(), g.data_ptr())

    def step(i):
        ctx.eval_device(poses[i & 1], acc[i & 1].data_ptr(), *outs)

    for i in range(40):  # first passes, regroup, block orders, clocks up
        step(i)
        if i == 1:
            ctx.regroup_auto()
    torch.cuda.synchronize()
    ref = [x.clone() for x in acc]

    per = 2 * 10  # steps per captured graph
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        for i in range(per):
            step(i)
    torch.cuda.synchronize()
    graph.replay()
    torch.cuda.synchronize()
    same = all(torch.equal(x, y) for x, y in zip(acc, ref))

    def timed(fn, reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s)
        for r in range(reps):
            fn(r)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    res = {"eager": [], "graph": []}
    K = (a.steps // per) * per
    for _ in range(a.rounds):
        res["eager"].append(timed(step, K) / K)
        res["graph"].append(timed(lambda r: graph.replay(), K // per) / K)
    out = {"points": n, "steps": K, "steps_per_graph": per, "same_accumulator": same,
           "eager_ms_per_step": res["eager"], "graph_ms_per_step": res["graph"],
           "eager_median": statistics.median(res["eager"]), "graph_median": statistics.median(res["graph"])}
    print(json.dumps(out), flush=True)
    ctx.set_stream(None)
    return 0


if __name__ == "__main__":
    sys.exit(main())
