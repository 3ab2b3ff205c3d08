#!/usr/bin/env python3
"""Back-to-back bench-cloud passes WITHOUT pass profiling, for a kernel trace of
the step's launch gaps (the bench times the pass kernel with HIP events, which
are themselves packets in the stream):

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/step_trace.py [--points N]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch
    import flash
    from flash import Models, synthetic, _lib
    m = Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m, 1234)
    poses = [flash.hull_poses(m, qe), flash.hull_poses(m, qe + 1e-3)]
    pts = synthetic.depth_cloud(m, qt, a.points, seed=1234 + 17, order="shuffled")
    ctx = _lib.Context(device=0, precision=64, cull=True, sort_points=True)
    ctx.set_model([(s.hull.vertices, s.hull.faces, s.hull.planes) for s in m.surfaces])
    ctx.set_output_order(True)
    ctx.set_points(pts)
    dev = torch.device("cuda", 0)
    accum = torch.zeros(ctx.accum_len, dtype=torch.float64, device=dev)
    bufs = (torch.empty(a.points, dtype=torch.int32, device=dev), torch.empty(a.points, dtype=torch.float64, device=dev),
            torch.empty((a.points, 3), dtype=torch.float64, device=dev))
    for i in range(a.steps):
        ctx.eval_device(poses[i & 1], accum.data_ptr(), *(b.data_ptr() for b in bufs))
    torch.cuda.synchronize()
    ctx.close()
    print("ok", float(accum[0]))


if __name__ == "__main__":
    main()
