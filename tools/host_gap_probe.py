#!/usr/bin/env python3
"""Where the host solver loop's per-iteration idle gap goes (GPU box).

Run against a diagnostic build whose fsdf_descend prints its host clocks
(`make dev DEV_OUT=../../abr/lib_host_times.so EXTRA=-DFSDF_HOST_TIMES=1`):

    FLASHSDF_LIB=$PWD/abr/lib_host_times.so python tools/host_gap_probe.py

Per model: one estimate_state frame (30 iterations of the default NaiveSolver,
tolerance 0) on a 2^20-point resident cloud, host loop, three times; the build
prints prepare (FK + surface poses), launches (pose + pass + reduce), wait
(device work + wake-up) and chain rule means per iteration (stderr).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def main():
    from flash import Models, synthetic
    from flash.gradientdescent import CostFunctor
    for name in ("arm_grid", "irb140"):
        m = getattr(Models, name)()
        qt, qe = synthetic.perturbed_configuration(m, 41)
        pts = synthetic.depth_cloud(m, qt, 1 << 20, seed=42)
        cf = CostFunctor(m, pts)
        cf.ctx.set_solver(False)
        x0 = np.asarray(qe, np.float64)
        for rep in range(4):
            t = time.perf_counter()
            _, f, its = cf.descend(x0, 30, 0.1, 0.5, 0.0, None, float(len(pts)))
            ms = (time.perf_counter() - t) * 1e3
            print(f"{name} frame {rep}: {ms:.3f} ms, {its} iterations, {ms / its * 1e3:.1f} us/iteration", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
