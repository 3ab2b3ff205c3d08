#!/usr/bin/env python3
"""Frames of the bench workload (M64, 2^20 points, 30 iterations of the default
solver, host loop) with and without the next frame's upload running under the
iterations (fsdf_prefetch_points), for a kernel + memory-copy trace:

    rocprofv3 --kernel-trace --memory-copy-trace --stats -d OUT -o run -- python3 tools/prefetch_probe.py
"""
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def main():
    import torch
    from flash import Models, synthetic
    m = Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m, 1234)
    pts = synthetic.depth_cloud(m, qt, 1 << 20, seed=1234 + 17)
    n = len(pts)
    bufs = []
    for _ in range(2):
        p = torch.empty((n, 3), dtype=torch.float64, pin_memory=True)
        p.copy_(torch.from_numpy(pts))
        bufs.append(p)
    ctx = m.engine(0, 64)
    surf = m.surfaces
    ctx.set_mechanism(m.mechanism, [s.body for s in surf], [s.frame.R for s in surf], [s.frame.t for s in surf])
    x0 = np.asarray(qe, np.float64)
    for mode in ("plain", "prefetch", "plain", "prefetch"):
        ts, sp = [], []
        if mode == "prefetch":
            ctx.prefetch_points(bufs[0].numpy())
        for f in range(6):
            t0 = time.perf_counter()
            if mode == "prefetch":
                ctx.set_points_prefetched()
                ctx.prefetch_points(bufs[(f + 1) & 1].numpy())
            else:
                ctx.set_points(bufs[f & 1].numpy())
            t1 = time.perf_counter()
            ctx.descend(x0, 30, 0.1, 0.5, 1e-3, None, float(n))
            t2 = time.perf_counter()
            if f:
                ts.append((t2 - t0) * 1e3)
                sp.append((t1 - t0) * 1e3)
        if mode == "prefetch":
            ctx.set_points_prefetched()
        print(f"{mode}: frame {statistics.median(ts):.3f} ms, ingest {statistics.median(sp):.3f} ms, "
              f"iterations {(statistics.median(ts) - statistics.median(sp)) / 30 * 1e3:.1f} us each", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
