#!/usr/bin/env python3
"""The first pass over a new cloud, with and without seeds carried from the
previous cloud (GPU box). M64, 2^20 points, the bench's clouds: per rep a new
cloud (a different seed of the generator) is made resident and evaluated once;
the pass kernel's HIP-event time of that first pass is reported for
  carried   one context over a sequence of clouds (fsdf_set_points carries the
            last pass's k* into the next cloud's seeds through a voxel grid)
  fresh     a context that has never held a cloud (no seeds: bounds only)
and, after the first pass, the steady pass time.

    python tools/seed_probe.py
"""
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def main():
    import flash
    from flash import Models, synthetic
    m = Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m, 1234)
    poses = flash.hull_poses(m, qe)
    clouds = [synthetic.depth_cloud(m, qt + 0.002 * r, 1 << 20, seed=1234 + 17 + r) for r in range(6)]
    carried = m.engine(0, 64, slot=0)
    carried.set_points(clouds[-1])
    carried.eval(poses)

    def first_pass(ctx, pts):
        ctx.set_points(pts)
        ctx.profile_pass(True)
        ctx.eval(poses)
        k1, _, _ = ctx.pass_times()
        ctx.profile_pass(False)
        ctx.profile_pass(True)
        for _ in range(5):
            ctx.eval(poses)
        k5, _, l5 = ctx.pass_times()
        ctx.profile_pass(False)
        return k1, k5 / max(l5, 1)

    out = {"carried": [], "fresh": []}
    for r, pts in enumerate(clouds):
        t = time.perf_counter()
        while time.perf_counter() - t < 0.05:  # (clocks up)
            carried.eval(poses)
        out["carried"].append(first_pass(carried, pts))
        fresh = m.engine(0, 64, slot=10 + r)
        out["fresh"].append(first_pass(fresh, pts))
    for k, v in out.items():
        print(f"{k}: first pass {statistics.median(a for a, _ in v):.4f} ms, then {statistics.median(b for _, b in v):.4f} ms "
              f"(median of {len(v)})", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
