#!/usr/bin/env python3
"""A few track! frames of the bench workload (M64, 2^20 points, estimate_state's
default solver: 30 iterations, rate 0.1, max_step 0.5) through fsdf_descend,
device solver loop and host loop, for a rocprofv3 kernel trace of the
iteration's launches (tools/gpu_run.sh step `descend`):

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/descend_probe.py

then `python3 tools/descend_probe.py --trace OUT/.../run_kernel_trace.csv` prints per
kernel the mean duration and, per iteration of the device loop, the span from
one solver step's end to the next (the iteration's device time incl. gaps)."""
import argparse
import csv
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def run(args):
    import torch  # noqa: F401  (the HIP runtime torch loads, before libflashsdf)
    from flash import Models, synthetic
    m = Models.arm_grid() if args.model == "m64" else Models.irb140()
    q_true, q_eval = synthetic.perturbed_configuration(m, 1234)
    pts = synthetic.depth_cloud(m, q_true, args.points, seed=1234 + 17)
    ctx = m.engine(0, 64)
    surf = m.surfaces
    ctx.set_mechanism(m.mechanism, [s.body for s in surf], [s.frame.R for s in surf], [s.frame.t for s in surf])
    for dev_loop in (True, False):
        ctx.set_solver("require" if dev_loop else False)
        ms = []
        for f in range(args.frames):
            t0 = time.perf_counter()
            ctx.set_points(pts)
            x, val, its = ctx.descend(np.asarray(q_eval, np.float64), 30, 0.1, 0.5, 1e-3, None, float(len(pts)))
            ms.append((time.perf_counter() - t0) * 1e3)
        print(f"{'device' if dev_loop else 'host'} loop: frame {statistics.median(ms):.3f} ms, {its} iterations, "
              f"f {val:.9g}", flush=True)


def trace(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by = {}
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:60]
        by.setdefault(name, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"{name:60s} {len(v):6d} x {statistics.mean(v):8.2f} us (median {statistics.median(v):.2f})")
    # (the step: solver_step_kernel, or the reduce + step kernel of FSDF_FUSED_STEP builds)
    steps = [i for i, r in enumerate(rows) if "step_kernel" in r["Kernel_Name"]]
    spans, busy = [], []
    for i0, i1 in zip(steps, steps[1:]):
        a, b = int(rows[i0]["End_Timestamp"]), int(rows[i1]["End_Timestamp"])
        if not 0 < b - a < 1e6:
            continue
        spans.append((b - a) / 1e3)  # one iteration: after a step to the end of the next
        busy.append(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[i0 + 1:i1 + 1]) / 1e3)
    if spans:
        print(f"device loop: iteration span {statistics.median(spans):.2f} us, kernels busy "
              f"{statistics.median(busy):.2f} us, idle {statistics.median([s - b for s, b in zip(spans, busy)]):.2f} us "
              f"(median over {len(spans)})")
    # device loop, per frame (from its solver_init_kernel): the first iterations
    # (the new cloud's unseeded pass, the regroup, the first pass after it)
    # against the steady ones
    inits = [i for i, r in enumerate(rows) if "solver_init_kernel" in r["Kernel_Name"]]
    per = []
    for fi, i0 in enumerate(inits):
        i1 = inits[fi + 1] if fi + 1 < len(inits) else len(rows)
        prev, its = int(rows[i0]["End_Timestamp"]), []
        for k in range(i0 + 1, i1):
            if "step_kernel" in rows[k]["Kernel_Name"]:
                e = int(rows[k]["End_Timestamp"])
                its.append((e - prev) / 1e3)
                prev = e
        if len(its) >= 4:
            per.append(its)
    if per:
        med = lambda j: statistics.median(p[j] for p in per)  # noqa: E731
        steady = statistics.median(x for p in per for x in p[2:])
        print(f"device loop per frame: iteration 1 {med(0):.1f} us, iteration 2 {med(1):.1f} us, then "
              f"{steady:.1f} us (median over {len(per)} frames)")
    # host loop: the iterations' pose -> pass -> reduce triplets (pose_kernel_args) and the gap before each pose
    poses = [i for i, r in enumerate(rows) if "pose_kernel_args" in r["Kernel_Name"]]
    gaps = [(int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])) / 1e3 for i in poses if i > 0]
    gaps = [g for g in gaps if 0 <= g < 1000]
    if gaps:
        print(f"host loop: idle before each iteration's pose kernel {statistics.median(gaps):.2f} us median")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="m64", choices=("m64", "irb140"))
    p.add_argument("--points", type=int, default=1 << 20)
    p.add_argument("--frames", type=int, default=5)
    p.add_argument("--trace", default=None)
    a = p.parse_args()
    if a.trace:
        trace(a.trace)
    else:
        run(a)
