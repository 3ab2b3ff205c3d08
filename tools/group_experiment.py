#!/usr/bin/env python3
"""Experiment (GPU box): does regrouping the resident cloud by nearest surface
shorten the pass? Orders compared on the bench cloud (M64):
  hilbert  the device Hilbert sort (sort_points=True, the shipped order)
  kstar    Hilbert order stably re-sorted by k* of a first pass (host-side
           reorder, uploaded with sort_points=False)
Prints pass-kernel time per order (HIP events) and, with a -DFSDF_WAVE_TIMES=1
build (FLASHSDF_LIB), the per-wave evaluation counts.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def timed(ctx, poses, reps=30):
    for i in range(5):
        ctx.eval(poses[i & 1])
    ctx.profile_pass(True)
    for i in range(reps):
        ctx.eval(poses[i & 1])
    ms, n = ctx.pass_time()
    ctx.profile_pass(False)
    return ms / max(n, 1)


def wave_stats(lib, ctx, poses, npts):
    nw = -(-npts // 64)
    buf = np.zeros(32 + 4 * 4 * 16384 + 2 * 16384, np.uint64)
    if lib.fsdf_kernel_stats(ctx._ctx, 1, None) != 0:
        return None
    ctx.eval(poses)
    lib.fsdf_kernel_stats(ctx._ctx, 0, buf.ctypes.data_as(ctypes.c_void_p))
    t = buf[32:32 + 2 * min(nw, 4 * 16384)].reshape(-1, 2).astype(np.int64)
    ev = buf[32 + 8 * 16384:32 + 8 * 16384 + 2 * min(nw, 4 * 16384)].reshape(-1, 2).astype(np.int64)
    if not t[:, 0].any():
        return None
    dur = (t[:, 1] - t[:, 0]) * 0.01
    span = (t[:, 1].max() - t[:, 0].min()) * 0.01
    return {"span_us": float(span), "dur_max_us": float(dur.max()), "dur_mean_us": float(dur.mean()),
            "evals_mean": float(ev[:, 0].mean()), "evals_max": int(ev[:, 0].max()),
            "seeds_mean": float(ev[:, 1].mean()),
            "waves_by_evals": {int(e): int((ev[:, 0] == e).sum()) for e in np.unique(ev[:, 0])}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, nargs="+", default=[1 << 20, 1 << 17])
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import flash
    from flash import Models, synthetic, _lib
    lib = _lib.load()
    m = Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m, 1234)
    poses = [flash.hull_poses(m, qe), flash.hull_poses(m, qe + 1e-3)]
    hulls = [(s.hull.vertices, s.hull.faces, s.hull.planes) for s in m.surfaces]
    res = []
    for n in args.points:
        pts = synthetic.depth_cloud(m, qt, n, seed=1234 + 17, order="shuffled")
        c = _lib.Context(device=0, precision=64, cull=True, sort_points=True)
        c.set_model(hulls)
        c.set_points(pts)
        c.set_output_order(False)
        _, _, (ks, _, _) = c.eval(poses[0], per_point=True)
        perm = c.permutation()
        r = {"points": n, "hilbert_ms": timed(c, poses), "hilbert_waves": wave_stats(lib, c, poses[0], n)}
        c.close()
        order = perm[np.argsort(ks[perm], kind="stable")]
        c2 = _lib.Context(device=0, precision=64, cull=True, sort_points=False)
        c2.set_model(hulls)
        c2.set_points(pts[order])
        r["kstar_ms"] = timed(c2, poses)
        r["kstar_waves"] = wave_stats(lib, c2, poses[0], n)
        _, _, (ks2, _, _) = c2.eval(poses[0], per_point=True)
        r["kstar_exact"] = bool(np.array_equal(ks2, ks[order]))
        c2.close()
        print(json.dumps(r), flush=True)
        res.append(r)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
