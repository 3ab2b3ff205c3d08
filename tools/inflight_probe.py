#!/usr/bin/env python3
"""Independent passes in flight on one GPU (run on the GPU box): C contexts over
the same resident cloud, each on its own HIP stream, step i on context i % C —
against one context's serial steps. Prints per-pass wall time (step period) for
C = 1, 2, 3 at each size, and checks that every context's accumulator equals
the serial one bit for bit.

    python tools/inflight_probe.py --sizes 131072,262144,524288,1048576
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="131072,262144,524288,1048576")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--plan-max", type=int, default=-1, help="fsdf_set_plan max_points (-1: the default window)")
    ap.add_argument("--counts", default="1,2,3", help="contexts in flight to measure (commas or +)")
    a = ap.parse_args()
    import torch
    import flash
    from flash import Models, synthetic, _lib
    dev = torch.device("cuda", 0)
    m = Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m, a.seed)
    poses = [flash.hull_poses(m, qe), flash.hull_poses(m, qe + 1e-3)]
    for n in (int(s) for s in a.sizes.split(",")):
        pts = synthetic.depth_cloud(m, qt, n, seed=a.seed + 17, order="shuffled")
        d_pts = torch.as_tensor(pts, device=dev)
        res = {"points": n, "plan_max": a.plan_max}
        ref = None
        for C in (int(c) for c in a.counts.replace("+", ",").split(",")):
            streams = [torch.cuda.Stream(dev) for _ in range(C)]
            ctxs, accs, outs = [], [], []
            for c in range(C):
                ctx = _lib.Context(device=0, precision=64, cull=True, sort_points=True)
                ctx.set_surfaces([("hull", (s_.hull.vertices, s_.hull.faces, s_.hull.planes)) for s_ in m.surfaces])
                ctx.set_output_order(True)
                ctx.set_plan(True, -1, -1, a.plan_max)
                ctx.set_stream(streams[c].cuda_stream)
                ctx.set_points_device(d_pts.data_ptr(), n)
                ctxs.append(ctx)
                accs.append([torch.zeros(ctx.accum_len, dtype=torch.float64, device=dev) for _ in range(2)])
                bufs = (torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.float64, device=dev),
                        torch.empty((n, 3), dtype=torch.float64, device=dev))
                outs.append((bufs, tuple(b.data_ptr() for b in bufs)))

            def step(i):
                c = i % C
                s = (i // C) & 1
                ctxs[c].eval_device(poses[s], accs[c][s].data_ptr(), *outs[c][1])

            t_end = time.perf_counter() + 0.3  # settle
            i = 0
            while time.perf_counter() < t_end:
                step(i)
                i += 1
                if i % 32 == 0:
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(3):
                t0 = time.perf_counter()
                for i in range(a.steps):
                    step(i)
                torch.cuda.synchronize()
                best = min(best, (time.perf_counter() - t0) / a.steps * 1e3)
            got = [accs[c][s].cpu().numpy() for c in range(C) for s in (0, 1)]
            if ref is None:
                ref = got[:2]
            same = all(np.array_equal(g, ref[j % 2]) for j, g in enumerate(got))
            res[f"C{C}_ms_per_pass"] = best
            res[f"C{C}_bits_equal"] = same
            for ctx in ctxs:
                ctx.close()
            del ctxs, accs, outs
        print(json.dumps(res), flush=True)
        del d_pts


if __name__ == "__main__":
    main()
