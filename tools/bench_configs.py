#!/usr/bin/env python3
"""Throughput of every BASELINE.json config on ONE GPU (the metric line itself
is bench.py's; these are the companion numbers DESIGN.md §7 reports).

  C2  IRB140 rigid, 2^20 synthetic points, f64
  C3  deformable beanbag (RBF, 25 states), 2^20 points, f32 (and f64)
  C4  IRB140, 10*2^20/8 = 1,310,720 points = one GPU's shard of the 8-GPU config, f64
  C5  irb_and_squishable (7 hulls + squishable RBF + table, 63 states), 2^20 points (the reference's
      recorded squishable cloud tiled + G, flash.synthetic.c5_cloud), f32 vs f64
  M64 the metric model, for reference
Each: one residual pass incl. the RBF parameter upload; mean pass-kernel time
(HIP events) and whole-pass wall time over R passes (the Python prepare_pass
path); set_points once (sorted). Then the product's unit of work per config —
a track! frame through the native solver loop (CostFunctor.descend =
fsdf_descend: estimate_state's NaiveSolver rate 0.1, max_step 0.5, 30
iterations, tolerance 0 so every frame runs all 30, src/tracking.jl:12-15) on
the resident cloud: ms per iteration with the host loop and, for rigid scenes,
the device loop (csrc/solver.hip), and tracking point-evals/s.

    python tools/bench_configs.py [--reps 20] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def rbf_cloud(m, x, n, seed):
    """Points near the skins (projected surface samples + noise) and a uniform box."""
    from flash.synthetic import skin_cloud
    return skin_cloud(m, x, n, seed)


def run(name, m, x, pts, precision, reps):
    import flash
    from flash.core import prepare_pass
    ctx = m.engine(device=0, precision=precision)
    ctx.set_points(pts)
    nq = m.mechanism.num_positions
    q = m.mechanism.normalize(x[:nq])
    poses, _ = prepare_pass(ctx, m, q, x[nq:])
    ctx.eval(poses)
    ctx.profile_pass(True)
    t = time.perf_counter()
    for _ in range(reps):
        poses, _ = prepare_pass(ctx, m, q, x[nq:])
        ctx.eval(poses)
    wall = (time.perf_counter() - t) / reps
    ms, launches = ctx.pass_time()
    ctx.profile_pass(False)
    kms = ms / launches
    row = {"config": name, "points": len(pts), "surfaces": len(m.surfaces), "states": flash.num_states(m),
           "precision": precision, "pass_kernel_ms": kms, "evals_per_s_kernel": len(pts) / kms * 1e3,
           "pass_wall_ms_incl_host": wall * 1e3, "evals_per_s_wall": len(pts) / wall}
    row.update(track_frame(m, x, pts, precision))
    print(json.dumps(row), flush=True)
    return row


def track_frame(m, x, pts, precision, iters=30, frames=3):
    """Median of `frames` native solver frames (after one untimed) on the
    resident cloud: fsdf_descend with the host loop and, where the scene allows
    it (rigid: no RBF skin, no deformation), the device loop."""
    import statistics
    from flash.gradientdescent import CostFunctor
    from flash._lib import FlashNativeError
    cf = CostFunctor(m, pts, precision=precision)
    x0 = np.asarray(x, np.float64)
    out = {}
    for name, mode in (("host_loop", False), ("device_loop", "require")):
        cf.ctx.set_solver(mode)
        try:
            cf.descend(x0, iters, 0.1, 0.5, 0.0, None, float(len(pts)))
        except FlashNativeError:
            continue  # (device loop: RBF scenes iterate on the host)
        ts = []
        for _ in range(frames):
            t = time.perf_counter()
            _, f, its = cf.descend(x0, iters, 0.1, 0.5, 0.0, None, float(len(pts)))
            ts.append((time.perf_counter() - t) * 1e3)
        ms = statistics.median(ts)
        out[f"frame_{name}_ms_per_iteration"] = ms / its
        out[f"frame_{name}_tracking_evals_per_s"] = len(pts) * its / (ms / 1e3)
    cf.ctx.set_solver(True)  # (the default)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from flash import Models, synthetic
    rows = []
    irb = Models.irb140()
    qt, qe = synthetic.perturbed_configuration(irb, 2)
    rows.append(run("C2 irb140", irb, qe, synthetic.depth_cloud(irb, qt, 1 << 20, seed=3, order="shuffled"), 64, a.reps))
    rows.append(run("C4 irb140 shard", irb, qe, synthetic.depth_cloud(irb, qt, 10 * (1 << 20) // 8, seed=4,
                                                                      order="shuffled"), 64, a.reps))
    bb = Models.beanbag()
    import flash
    r = np.random.Generator(np.random.PCG64(5))
    x = np.zeros(flash.num_states(bb))
    x[:7] = bb.mechanism.zero_configuration()
    x[4:7] = 2 * r.random(3) ** 3
    x[7:] = 0.5 * (r.random(18) - 0.5)
    pts = rbf_cloud(bb, x, 1 << 20, 6)
    for prec in (32, 64):
        rows.append(run("C3 beanbag", bb, x, pts, prec, a.reps))
    sc, x0 = Models.irb_and_squishable()
    # the reference's recorded cloud tiled/jittered + G on the scene's hulls
    real = np.load(os.path.join(ROOT, "tests", "golden", "squishable_unsquished.npz"))["xyz"]
    pts = synthetic.c5_cloud(sc, x0, 1 << 20, real, seed=7)
    for prec in (32, 64):
        rows.append(run("C5 irb_and_squishable", sc, x0, pts, prec, a.reps))
    m64 = Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m64, 1234)
    rows.append(run("M64", m64, qe, synthetic.depth_cloud(m64, qt, 1 << 20, seed=9, order="shuffled"), 64, a.reps))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
