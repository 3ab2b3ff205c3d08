#!/usr/bin/env python3
"""Measured speed-up of splitting a chunk over 2 / 4 waves (GPU box; verdict r4
item 5: the planned pass's x5/2 and x8/5 rescale of split chunks' durations).

The planned pass records each chunk's wall time from its first wave's start to
its emit; a chunk split over P waves stores that time x5/2 (P = 4) or x8/5
(P = 2) as its serial-equivalent duration (sdf_kernels.hip planned_pass_kernel).
Here the same resident cloud runs (a) every chunk on one wave (plan shares 0, 0)
and (b) the default plan, R passes each, alternating; per chunk the median
one-wave time and the median split wall time (the stored duration divided by
the rescale) give the split's speed-up, for the chunks the default plan split.

    python tools/split_speedup.py [--model arm_grid|irb140] [--points N] [--rounds R]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))

# the serial-equivalent rescale the kernel applies to split chunks (capi.hip run_planned:
# scenes with >= 32 hulls, fewer); round 4's build used 5/2 and 8/5 for both
RESCALE = {True: {4: 15 / 8, 2: 4 / 3}, False: {4: 5 / 2, 2: 8 / 5}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="arm_grid")
    ap.add_argument("--points", type=int, default=1 << 19)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--seed", type=int, default=1234)
    a = ap.parse_args()
    import flash
    from flash import Models, synthetic, _lib
    m = getattr(Models, a.model)()
    qt, qe = synthetic.perturbed_configuration(m, a.seed)
    pts = synthetic.depth_cloud(m, qt, a.points, seed=a.seed + 17, order="shuffled")
    poses = flash.hull_poses(m, qe)
    ctx = _lib.Context(device=0, sort_points=True)
    ctx.set_model([(s.hull.vertices, s.hull.faces, s.hull.planes) for s in m.surfaces])
    ctx.set_points(pts)
    nc = -(-len(pts) // 64)
    # the round-4 default composition's counts (capi.hip kPlanDefault4 / 2, or the spare-slot rule),
    # as fixed shares: the split set is then the heaviest chunks, whatever the keyed plan would pick
    slots = 256 * 16
    n4 = min(nc, max(96, max(0, slots - nc) // 3))
    n2 = min(nc - n4, 192)
    one, split = [], []
    for r in range(a.rounds):
        for shares, sink in (((0.0, 0.0), one), ((n4 / nc, n2 / nc), split)):
            ctx.set_plan(True, shares[0], shares[1], len(pts))
            for _ in range(20):  # first pass plans, the plan is rebuilt after 16
                ctx.eval(poses)
            sink.append(ctx.chunk_costs().astype(np.float64))
    one = np.median(np.array(one), axis=0)
    split_d = np.median(np.array(split), axis=0)
    order = np.argsort(-one, kind="stable")
    rescale = RESCALE[len(m.surfaces) >= 32]
    out = {"model": a.model, "points": len(pts), "chunks": nc, "rounds": a.rounds, "n4": n4, "n2": n2,
           "heaviest_one_wave_us": float(one.max()) / 100.0, "mean_one_wave_us": float(one.mean()) / 100.0}
    for parts, sel in ((4, order[:n4]), (2, order[n4:n4 + n2])):
        wall = split_d[sel] / rescale[parts]
        s = one[sel] / wall
        out[f"speedup_{parts}way"] = {"median": float(np.median(s)), "p10": float(np.percentile(s, 10)),
                                      "p90": float(np.percentile(s, 90)),
                                      "heaviest10_median": float(np.median(s[:10]))}
    print(json.dumps(out), flush=True)
    ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
