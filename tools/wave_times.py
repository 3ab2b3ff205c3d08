#!/usr/bin/env python3
"""Per-wave wall-clock timeline of one pass (GPU box, diagnostic build):

    make -C point-cloud-signed-distance_amd/csrc dev DEV_OUT=../../ab/lib_wt.so EXTRA=-DFSDF_WAVE_TIMES=1
    FLASHSDF_LIB=$PWD/ab/lib_wt.so python tools/wave_times.py [--points N] [--json out.json]

Each wave-iteration of the first grid pass records s_memrealtime (100 MHz)
at its start and end. Prints the pass span, the wave-duration distribution,
and how much of the span the last-started waves occupy (the tail).
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=1 << 20)
    ap.add_argument("--order", default="shuffled")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import flash
    from flash import Models, synthetic, _lib

    m = Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m, 1234)
    poses = flash.hull_poses(m, qe)
    pts = synthetic.depth_cloud(m, qt, args.points, seed=1234 + 17, order=args.order)
    c = _lib.Context(device=0, precision=64, cull=True, sort_points=True)
    c.set_plan(False)  # the per-wave timeline is written by the block-structured pass only
    c.set_model([(s.hull.vertices, s.hull.faces, s.hull.planes) for s in m.surfaces])
    c.set_points(pts)
    for _ in range(3):
        c.eval(poses)
    lib = _lib.load()
    nw = -(-args.points // 64)
    buf = np.zeros(32 + 32 * 16384, np.uint64)
    assert lib.fsdf_kernel_stats(c._ctx, 1, None) == 0
    c.eval(poses)
    assert lib.fsdf_kernel_stats(c._ctx, 0, buf.ctypes.data_as(ctypes.c_void_p)) == 0
    c.close()
    t = buf[32:32 + 2 * min(nw, 4 * 16384)].reshape(-1, 2).astype(np.int64)
    ev = buf[32 + 8 * 16384:32 + 8 * 16384 + 2 * min(nw, 4 * 16384)].reshape(-1, 2).astype(np.int64)
    ph = buf[32 + 18 * 16384:32 + 18 * 16384 + 2 * min(nw, 4 * 16384)].reshape(-1, 2).astype(np.uint64)
    ev_raw = buf[32 + 8 * 16384:32 + 8 * 16384 + 2 * min(nw, 4 * 16384)].reshape(-1, 2).astype(np.uint64)

    def fields(a):  # (n, 2) packed 16-bit fields -> (n, 8)
        return np.stack([(a[:, j // 4] >> np.uint64(16 * (j % 4))) & np.uint64(0xffff) for j in range(8)],
                        1).astype(np.int64)
    evf = fields(ev_raw)  # evals, rejects, slow, walk steps, seeds, need lanes, candidates, full scans
    phf = fields(ph) * 0.01  # us: stage, screen, fast, search, cull, rbf, emit, -
    e2 = buf[32 + 26 * 16384:32 + 26 * 16384 + min(nw, 4 * 16384)].astype(np.uint64)
    ev2 = np.stack([(e2 >> np.uint64(16 * j)) & np.uint64(0xffff) for j in range(4)], 1).astype(np.int64)
    # slow lane-evaluations | of which the hull won the lane | lanes spared the search by h_max
    nw2 = min(nw, 16384)
    p2 = buf[32 + 30 * 16384:32 + 30 * 16384 + 2 * nw2].reshape(-1, 2).astype(np.uint64)
    sub = np.zeros((min(nw, 4 * 16384), 8))
    sub[:nw2] = fields(p2)
    sub[:, [0, 1, 4, 5]] *= 0.01  # us
    sub_names = ["t_cert", "t_walk_cot", "vertex_lane_certs", "fan_iters", "t_screen_loop", "t_fixup",
                 "edge_lane_certs", "interior_lane_certs"]
    ev = np.stack([evf[:, 0], evf[:, 4]], 1)
    nb = -(-args.points // 256)
    bt = buf[32 + 16 * 16384:32 + 16 * 16384 + 2 * min(nb, 16384)].reshape(-1, 2).astype(np.int64)
    if not t[:, 0].any():
        print("no wave times recorded (not a -DFSDF_WAVE_TIMES=1 build?)")
        return 1
    t0 = t[:, 0].min()
    start = (t[:, 0] - t0) * 0.01  # us
    end = (t[:, 1] - t0) * 0.01
    dur = end - start
    span = end.max()
    q = np.percentile(dur, [10, 50, 90, 99, 100])
    # busy fraction of wave slots over time (1024 WG slots x 4 waves)
    grid = np.linspace(0, span, 41)
    live = [int(((start <= g) & (end > g)).sum()) for g in grid[:-1]]
    order = np.argsort(start)
    late = order[-len(order) // 20:]  # last 5 % of waves to start
    res = {"points": args.points, "waves": int(len(dur)), "span_us": float(span),
           "dur_us_p10_p50_p90_p99_max": [float(x) for x in q], "dur_us_mean": float(dur.mean()),
           "sum_dur_us": float(dur.sum()),
           "last5pct_start_us": float(start[late].min()), "last5pct_end_max_us": float(end[late].max()),
           "live_waves_over_time": live,
           "corr_dur_vs_index": float(np.corrcoef(dur, np.arange(len(dur)))[0, 1]),
           "evals_mean": float(ev[:, 0].mean()), "evals_max": int(ev[:, 0].max()),
           "corr_dur_vs_evals": float(np.corrcoef(dur, ev[:, 0])[0, 1]),
           "us_per_eval_by_evals": {int(e): float(dur[ev[:, 0] == e].mean() / max(e, 1))
                                    for e in np.unique(ev[:, 0])},
           "waves_by_evals": {int(e): int((ev[:, 0] == e).sum()) for e in np.unique(ev[:, 0])},
           "block_us_mean": float((bt[:, 1] - bt[:, 0]).mean() * 0.01),
           "block_minus_slowest_wave_us_mean": float(((bt[:, 1] - bt[:, 0]) * 0.01 - dur[:len(bt) * 4].reshape(-1, 4).max(1)).mean()),
           "block_start_to_first_wave_us_mean": float(((t[:len(bt) * 4, 0].reshape(-1, 4).min(1) - bt[:, 0]) * 0.01).mean()),
           "heaviest_waves": [[float(dur[i]), int(ev[i, 0]), int(ev[i, 1])] for i in np.argsort(-dur)[:12]]}
    ev_names = ["evals", "rejects", "slow", "walk_steps", "seeds", "need_lanes", "candidates", "full_scans"]
    ph_names = ["stage", "screen", "fast", "search", "cull", "rbf", "emit", "walk"]
    heavy = np.argsort(-dur)[:16]
    res["heaviest_detail"] = [{"us": round(float(dur[i]), 2), **{n: int(evf[i, j]) for j, n in enumerate(ev_names)},
                               **{"t_" + n: round(float(phf[i, j]), 2) for j, n in enumerate(ph_names)}}
                              for i in heavy]
    tot = phf[:, :8].sum(0)
    res["phase_us_total_frac"] = {n: round(float(tot[j] / dur.sum()), 4) for j, n in enumerate(ph_names)}
    ne = max(int(evf[:, 0].sum()), 1)
    res["per_eval_us"] = {n: round(float(phf[:, j].sum() / ne), 3) for j, n in enumerate(ph_names[:4])}
    res["event_totals"] = {n: int(evf[:, j].sum()) for j, n in enumerate(ev_names)}
    e2n = ["slow_lane_evals", "slow_lane_evals_won", "lanes_spared_by_hmax", "t_needs_phase_c_10ns"]
    res["search_lanes"] = {n: int(ev2[:, j].sum()) for j, n in enumerate(e2n)}
    for i, r in zip(heavy, res["heaviest_detail"]):
        r.update({n: int(ev2[i, j]) for j, n in enumerate(e2n)})
        r.update({n: round(float(sub[i, j]), 2) for j, n in enumerate(sub_names)})
    res["sub_phase_totals"] = {n: round(float(sub[:, j].sum()), 2) for j, n in enumerate(sub_names)}
    ws = max(int(evf[:, 3].sum()), 1)
    res["per_walk_step"] = {"us_cert": round(float(sub[:, 0].sum() / ws), 3),
                            "us_cot": round(float(sub[:, 1].sum() / ws), 3),
                            "fan_iters": round(float(sub[:, 3].sum() / ws), 3)}
    res["per_eval_screen_us"] = {"loop": round(float(sub[:, 4].sum() / ne), 3),
                                 "fixup": round(float(sub[:, 5].sum() / ne), 3)}
    top = dur >= np.percentile(dur, 99)
    res["top1pct"] = {"waves": int(top.sum()), "us_mean": float(dur[top].mean()),
                      **{n: round(float(evf[top, j].mean()), 2) for j, n in enumerate(ev_names)},
                      **{"t_" + n: round(float(phf[top, j].mean()), 2) for j, n in enumerate(ph_names)},
                      **{n: round(float(ev2[top, j].mean()), 2) for j, n in enumerate(e2n)},
                      **{n: round(float(sub[top, j].mean()), 2) for j, n in enumerate(sub_names)}}
    print(json.dumps(res))
    if args.json:
        np.savez_compressed(args.json.replace(".json", ".npz"), start=start, end=end, evals=ev)
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
