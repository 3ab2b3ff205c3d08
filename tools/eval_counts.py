#!/usr/bin/env python3
"""Kernel work counters of the bench pass (GPU box): hull evaluations, seed
evaluations, walk steps per (points) for the library in FLASHSDF_LIB."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def main():
    import flash
    from flash import Models, synthetic, _lib
    m = Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m, 1234)
    poses = flash.hull_poses(m, qe)
    full = synthetic.depth_cloud(m, qt, 1 << 20, seed=1234 + 17, order="shuffled")
    for n in (1 << 20, 1 << 17):
        c = _lib.Context(device=0, precision=64, cull=True, sort_points=True)
        c.set_model([(s.hull.vertices, s.hull.faces, s.hull.planes) for s in m.surfaces])
        c.set_points(full[:n])
        c.eval(poses)
        c.kernel_stats(True)
        c.eval(poses)
        st = c.kernel_stats(False)
        print(json.dumps({"lib": os.path.basename(os.environ.get("FLASHSDF_LIB", "default")), "points": n,
                          **{k: st[k] for k in ("wave_iters", "hull_evals", "seed_evals", "slow_waves",
                                                "walk_steps", "screen_rejects")}}), flush=True)
        c.close()


if __name__ == "__main__":
    main()
