#!/usr/bin/env python3
"""What would sharing hull evaluations among the 4 waves of a workgroup buy?
(CPU analysis of a per-wave timeline, tools/wave_times.py --json X.json ->
X.npz with each wave-iteration's start/end.)

A pass workgroup holds its CU slot until its slowest wave ends. Per logical
block (4 consecutive waves): today its duration is max(wave), with perfect
sharing it would be sum(wave)/4 (bounded below by the longest single hull
evaluation of its heaviest wave, ~10 us). Both are list-scheduled
longest-first on 1,024 workgroup slots (256 CUs x 4) — the kernel's
cost-ordered schedule — and the predicted spans printed.

    python tools/coop_estimate.py profiles/r03/wt_1m.npz [--slots 1024]
"""
import argparse
import heapq
import json

import numpy as np


def lpt(durs, slots):
    h = [0.0] * slots
    for d in sorted(durs, reverse=True):
        t = heapq.heappop(h)
        heapq.heappush(h, t + d)
    return max(h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--slots", type=int, default=1024)
    ap.add_argument("--min-eval-us", type=float, default=10.0)
    ap.add_argument("--waves-per-block", type=int, default=4)
    ap.add_argument("--strided", action="store_true",
                    help="block b owns chunks b, b+B, b+2B, ... (B blocks) instead of W consecutive chunks")
    a = ap.parse_args()
    z = np.load(a.npz)
    dur = z["end"] - z["start"]
    evals = z["evals"][:, 0]
    W = a.waves_per_block
    nb = len(dur) // W
    d = dur[:nb * W].reshape(nb, W)
    e = evals[:nb * W].reshape(nb, W)
    if a.strided:
        d = dur[:nb * W].reshape(W, nb).T
        e = evals[:nb * W].reshape(W, nb).T
    bmax = d.max(1)
    per_eval = np.where(e.max(1) > 0, bmax / np.maximum(e.max(1), 1), 0)
    floor = np.minimum(bmax, np.maximum(per_eval, a.min_eval_us * (e.max(1) > 0)))
    bshare = np.maximum(d.sum(1) / W, floor)
    out = {"waves": int(len(dur)), "blocks": int(nb), "sum_wave_us": float(dur.sum()),
           "ideal_span_us": float(dur.sum() / (W * a.slots)),
           "lpt_span_today_us": float(lpt(bmax, a.slots)),
           "lpt_span_shared_us": float(lpt(bshare, a.slots)),
           "heaviest_block_today_us": float(bmax.max()), "heaviest_block_shared_us": float(bshare.max()),
           "block_idle_frac_today": float(1 - d.sum() / (W * bmax.sum()))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
