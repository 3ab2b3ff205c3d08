#!/usr/bin/env python3
"""End-to-end tracking timing (GPU box): the track! frame loop
(examples/irb_and_squishable.ipynb cells 11-12) over F synthetic frames of a
moving model, each frame = one cloud swap (upload + device sort) + I solver
iterations (native FK + pose assembly, residual pass, accumulator read-back,
chain rule). Prints ms per iteration, ms per frame, tracking error.

    python tools/track_bench.py [--model m64|irb140|c5] [--points N] [--frames F] [--iters I]

c5 = the notebook's own scene (irb_and_squishable: 7 hulls + the deformable
squishable RBF skin + table, 63 states): the IRB's joints move between
frames, the squishable's deformations are estimated with them.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "point-cloud-signed-distance_amd"), os.path.join(ROOT, "tools")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="m64", choices=("m64", "irb140", "c5"))
    ap.add_argument("--points", type=int, default=1 << 20)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import flash
    from flash import Models, synthetic
    from flash.tracking import NaiveSolver, Tracker
    rng = np.random.Generator(np.random.PCG64(91))
    if a.model == "c5":
        from bench_configs import rbf_cloud
        m, x0 = Models.irb_and_squishable()
        nq = m.mechanism.num_positions
        x0 = np.asarray(x0, np.float64)
        x0[nq:] = 0.005 * rng.normal(size=len(x0) - nq)  # a squished squishable
        xb = x0.copy()
        xb[7:13] += rng.uniform(-0.1, 0.1, size=6)  # the IRB's six revolute joints (after its floating base)
        xs = [x0 + (xb - x0) * t / max(a.frames - 1, 1) for t in range(a.frames)]
        clouds = [rbf_cloud(m, x, a.points, 92 + t) for t, x in enumerate(xs)]
        qs = xs
    else:
        m = Models.arm_grid() if a.model == "m64" else Models.irb140()
        qa, _ = synthetic.perturbed_configuration(m, 90)
        qb = qa + rng.uniform(-0.1, 0.1, size=qa.shape)
        qs = [qa + (qb - qa) * t / max(a.frames - 1, 1) for t in range(a.frames)]
        clouds = [synthetic.depth_cloud(m, q, a.points, seed=92 + t, order="shuffled") for t, q in enumerate(qs)]
    n = flash.num_states(m)
    state = flash.ManipulatorState(m)
    nq = m.mechanism.num_positions
    state.q[:] = qs[0][:nq] + 0.02
    state.deformation_data[:] = qs[0][nq:] if len(qs[0]) > nq else state.deformation_data
    # step rules: irb140.ipynb's rate 20 for the rigid arms; irb_and_squishable.ipynb
    # cell 11's rate 0.5 / max_step 0.1 for its own scene (30 iterations per frame here)
    rate = 0.5 if a.model == "c5" else 20.0
    tr = Tracker(m, state, NaiveSolver(n, rate=rate, max_step=0.1, iteration_limit=a.iters))
    tr.step(clouds[0])  # warm-up frame (allocations)
    tr.frame_ms.clear(); tr.set_points_ms.clear(); tr.iterations.clear()
    errs = []
    for q, pts in zip(qs[1:], clouds[1:]):
        x = tr.step(pts)
        errs.append(float(np.abs(x[:nq] - q[:nq]).max()))
    out = {"model": a.model, "points": a.points, "frames": a.frames - 1, "iters_per_frame": a.iters,
           "ms_per_iteration": tr.iteration_ms(), "ms_per_frame": float(np.mean(tr.frame_ms)),
           "set_points_ms": float(np.mean(tr.set_points_ms)),
           "point_evals_per_s_end_to_end": a.points * sum(tr.iterations) / (sum(tr.frame_ms) / 1e3),
           "max_abs_q_error_per_frame": errs}
    print(json.dumps(out))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
