#!/usr/bin/env python3
"""Replay the planned pass's workgroup plans on measured chunk costs (CPU study).

Input: per-chunk one-wave durations dumped by tools/hpart_sweep.py --dump-costs
(fsdf_chunk_costs, 100 MHz ticks). Model: 1,024 workgroup slots (256 CUs x 4),
list scheduling in plan order; a one-wave workgroup lasts as long as its slowest
chunk plus a fixed prologue; a chunk split over p waves lasts cost / speedup(p)
plus the prologue. Durations measured under full load, so the model holds for
full machines; it ignores issue contention when fewer waves run.

    python tools/plan_sim.py gpurun_out/r04e/costs.npz
"""
import heapq
import sys

import numpy as np

SLOTS = 1024
PROLOGUE = 1.5       # us: hull-table load per workgroup
SPEEDUP = {1: 1.0, 2: 1.6, 4: 2.5}


def span(wgs):
    """wgs: list of durations in launch order -> makespan on SLOTS slots."""
    free = [0.0] * SLOTS
    heapq.heapify(free)
    end = 0.0
    for d in wgs:
        t = heapq.heappop(free)
        heapq.heappush(free, t + d)
        end = max(end, t + d)
    return end


def unplanned(c):
    blocks = [max(c[i:i + 4]) + PROLOGUE for i in range(0, len(c), 4)]
    return span(sorted(blocks, reverse=True))  # block-level LPT


def planned(c, f4, f2, slots_waves=4096):
    order = np.argsort(-c, kind="stable")
    nc = len(c)
    n4 = int(min(nc, max(round(f4 * nc), max(0, slots_waves - nc) // 3)))
    n2 = int(min(nc - n4, round(f2 * nc)))
    s = c[order]
    wgs = [s[i] / SPEEDUP[4] + PROLOGUE for i in range(n4)]
    wgs += [max(s[n4 + i:n4 + i + 2]) / SPEEDUP[2] + PROLOGUE for i in range(0, n2, 2)]
    wgs += [max(s[n4 + n2 + i:n4 + n2 + i + 4]) + PROLOGUE for i in range(0, nc - n4 - n2, 4)]
    return span(wgs), n4, n2


def main(path):
    z = np.load(path)
    for key in z.files:
        c = z[key].astype(np.float64) / 100.0  # us
        print(f"{key}: {len(c)} chunks, mean {c.mean():.1f} us, max {c.max():.1f} us, "
              f"sum/4096 slots {c.sum() / 4096:.1f} us")
        print(f"  unplanned (blocks of 4 consecutive, LPT): {unplanned(c):.1f} us")
        for f4, f2 in ((0, 0), (1 / 256, 0), (1 / 128, 1 / 64), (1 / 32, 1 / 16), (1 / 16, 1 / 8)):
            sp, n4, n2 = planned(c, f4, f2)
            print(f"  planned f4={f4:.4f} f2={f2:.4f} (n4 {n4}, n2 {n2}): {sp:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
