#!/usr/bin/env python3
"""Pass time against the heavy-wave split budget and cloud size (GPU box).

    python tools/split_sweep.py [--budgets 0 1 2 3 4] [--points ...] [--json out.json]

M64 bench cloud (shuffled + device Hilbert sort), f64, per-point outputs in
resident order; per (points, budget) the mean pass-kernel and whole-pass
(pass kernel through the split kernels) times over 30 passes, HIP events."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--budgets", type=int, nargs="+", default=[0, 1, 2, 3, 4])
    ap.add_argument("--points", type=int, nargs="+", default=[1 << 20, 1 << 19, 1 << 18, 1 << 17, 1 << 16])
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import torch
    import flash
    from flash import Models, synthetic, _lib
    m = Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m, 1234)
    poses = [flash.hull_poses(m, qe), flash.hull_poses(m, qe + 1e-3)]
    full = synthetic.depth_cloud(m, qt, max(args.points), seed=1234 + 17, order="shuffled")
    dev = torch.device("cuda", 0)
    rows = []
    for n in args.points:
        pts = np.ascontiguousarray(full[:n])
        c = _lib.Context(device=0, precision=64, cull=True, sort_points=True)
        c.set_model([(s.hull.vertices, s.hull.faces, s.hull.planes) for s in m.surfaces])
        c.set_points(pts)
        c.set_output_order(True)
        acc = torch.zeros(c.accum_len, dtype=torch.float64, device=dev)
        ks = torch.empty(n, dtype=torch.int32, device=dev)
        dd = torch.empty(n, dtype=torch.float64, device=dev)
        gg = torch.empty((n, 3), dtype=torch.float64, device=dev)
        for b in args.budgets:
            c.set_split_budget(b)
            for i in range(5):
                c.eval_device(poses[i & 1], acc.data_ptr(), ks.data_ptr(), dd.data_ptr(), gg.data_ptr())
            c.synchronize()
            c.profile_pass(True)
            for i in range(args.reps):
                c.eval_device(poses[i & 1], acc.data_ptr(), ks.data_ptr(), dd.data_ptr(), gg.data_ptr())
            k_ms, p_ms, cnt = c.pass_times()
            c.profile_pass(False)
            r = {"points": n, "budget": b, "pass_kernel_ms": k_ms / cnt, "pass_ms": p_ms / cnt,
                 "Gevals_per_s": n / (p_ms / cnt) / 1e6}
            print(json.dumps(r), flush=True)
            rows.append(r)
        c.close()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
