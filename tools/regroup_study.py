#!/usr/bin/env python3
"""Resident order grouped by the previous pass's nearest surface (GPU box).

The pass's unit of cost is a wave's hull evaluation: a 64-point
chunk whose points have several nearest surfaces evaluates several hulls. A
tracking frame runs many passes over one cloud at nearby configurations, and
the nearest surface k* of a point rarely changes between them, so the resident
order could group points by the last pass's k* — within windows of the Hilbert
order, to keep chunks compact — and cut the evaluations per chunk.

This study needs no kernel change: the Hilbert-ordered cloud (a sorted
context's resident order) is regrouped on the host and uploaded to contexts
that keep the given order (sort_points off); every variant's pass is timed
(one pass at a time, the bench's two alternating configurations) with its
kernel work counters, and its per-point outputs are checked against the
Hilbert order's bit for bit. One JSON line per variant.

    python tools/regroup_study.py [--points N] [--windows 0,256,1024,4096,-1]
      window 0: Hilbert order as is; -1: one global grouping by k*
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
    ap.add_argument("--model", default="arm_grid")
    ap.add_argument("--points", type=int, default=1 << 20)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--windows", default="0,256,1024,4096,16384,-1")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    import flash
    from flash import Models, synthetic, _lib
    dev = torch.device("cuda", 0)
    m = getattr(Models, a.model)()
    qt, qe = synthetic.perturbed_configuration(m, a.seed)
    poses = [flash.hull_poses(m, qe), flash.hull_poses(m, qe + 1e-3)]
    pts = synthetic.depth_cloud(m, qt, a.points, seed=a.seed + 17, order="shuffled")
    n = len(pts)
    hulls = [(s.hull.vertices, s.hull.faces, s.hull.planes) for s in m.surfaces]
    ref = _lib.Context(device=0, sort_points=True)
    ref.set_model(hulls)
    ref.set_points(pts)
    ref.set_output_order(True)
    _, acc_h, (k_h, d_h, g_h) = ref.eval(poses[0], per_point=True)
    perm = ref.permutation()
    hil = np.ascontiguousarray(pts[perm])  # the Hilbert order
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    acc = torch.zeros(ref.accum_len, dtype=torch.float64, device=dev)
    out = [torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.float64, device=dev),
           torch.empty((n, 3), dtype=torch.float64, device=dev)]
    outs = [t.data_ptr() for t in out]
    ctxs = {}
    for w in (int(x) for x in a.windows.split(",")):
        if w == 0:
            o = np.arange(n)
        elif w < 0:
            o = np.lexsort((np.arange(n), k_h))
        else:
            o = np.lexsort((np.arange(n), k_h, np.arange(n) // w))
        c = _lib.Context(device=0, sort_points=False)
        c.set_model(hulls)
        c.set_stream(stream.cuda_stream)
        c.set_points(np.ascontiguousarray(hil[o]))
        _, acc_c, (k_c, d_c, g_c) = c.eval(poses[0], per_point=True)
        exact = bool(np.array_equal(k_c, k_h[o]) and np.array_equal(d_c, d_h[o]) and np.array_equal(g_c, g_h[o]))
        ch = k_h[o][: (n // 64) * 64].reshape(-1, 64)
        distinct = float(np.mean([len(np.unique(r)) for r in ch]))
        ctxs[w] = (c, exact, distinct, float(np.abs(acc_c - acc_h).max() / max(1.0, np.abs(acc_h).max())))
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:  # clocks settle
        for c, *_ in ctxs.values():
            c.eval_device(poses[0], acc.data_ptr(), *outs)
        torch.cuda.synchronize()
    res = {w: [] for w in ctxs}
    for _ in range(a.rounds):  # interleaved
        for w, (c, *_r) in ctxs.items():
            for i in range(8):
                c.eval_device(poses[i & 1], acc.data_ptr(), *outs)
            torch.cuda.synchronize()
            c.profile_pass(True)
            ts = time.perf_counter()
            for i in range(a.steps):
                c.eval_device(poses[i & 1], acc.data_ptr(), *outs)
            torch.cuda.synchronize()
            step = (time.perf_counter() - ts) / a.steps * 1e3
            kms, _, launches = c.pass_times()
            c.profile_pass(False)
            res[w].append((step, kms / max(launches, 1)))
    for w, (c, exact, distinct, acc_rel) in ctxs.items():
        c.kernel_stats(True)
        c.eval_device(poses[0], acc.data_ptr(), *outs)
        torch.cuda.synchronize()
        st = c.kernel_stats(False)
        waves = max(st.get("wave_iters", 0), 1)
        print(json.dumps({"window": w, "points": n, "exact_per_point": exact, "acc_max_rel_diff": acc_rel,
                          "distinct_kstar_per_chunk": distinct,
                          "step_ms": min(s for s, _ in res[w]), "kernel_ms": min(k for _, k in res[w]),
                          "kernel": c.pass_kernel_name(),
                          "hull_evals_per_wave": st.get("hull_evals", 0) / waves,
                          "seed_evals_per_wave": st.get("seed_evals", 0) / waves,
                          "slow_per_wave": st.get("slow_waves", 0) / waves,
                          "candidates_per_wave": st.get("wave_candidates", 0) / waves}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
