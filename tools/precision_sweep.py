#!/usr/bin/env python3
"""BASELINE config 5's fp32-vs-fp64 tolerance sweep (run on the GPU box).

Scene: irb_and_squishable (7 IRB140 hulls + the squishable RBF skin + the
table box, 63 states; examples/irb_and_squishable.ipynb cells 3-6) with a
random deformation of the squishable's surface points; 2^20 points as SURVEY.md
§8d defines C5: the reference's recorded cloud (squishable_unsquished_xyzrgb.txt,
25,571 points, fixture tests/golden/squishable_unsquished.npz) tiled and
jittered to half the points, generator G on the scene's hulls for the rest
(flash.synthetic.c5_cloud). For each context precision the GPU pass is
compared with the fp64 CPU oracle on the same posed scene:

  max / p99 |Δd*|, k* mismatch rate (and max |Δd*| at the mismatches: a flip
  is harmless only at a near-tie), max |Δ∇d*| where k* agrees,
  relative error of the cost and of ∂c/∂x (63 states, host chain rule);
  and the fp32 context bit for bit against the oracle's fp32 instantiation on
  a sample (`f32_exact_sample`).

    python tools/precision_sweep.py [--points N] [--json out.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "point-cloud-signed-distance_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)


REAL_CLOUD = os.path.join(ROOT, "tests", "golden", "squishable_unsquished.npz")


def scene(n, seed=31):
    import flash  # noqa: F401
    from flash import Models, synthetic
    m, x = Models.irb_and_squishable()
    nq = m.mechanism.num_positions
    r = np.random.Generator(np.random.PCG64(seed))
    x = x.copy()
    x[nq:] = 0.02 * (r.random(len(x) - nq) - 0.5)  # deformed squishable
    real = np.load(REAL_CLOUD)["xyz"]
    return m, x, synthetic.c5_cloud(m, x, n, real, seed=seed + 1)


def sweep(n, seed=31, exact_sample=1 << 17):
    import flash  # noqa: F401
    import oracle
    from flash import rbf as host_rbf
    from flash.core import surface_poses
    from flash.gradientdescent import CostFunctor
    m, x, pts = scene(n, seed)
    nq = m.mechanism.num_positions
    q = m.mechanism.normalize(x[:nq])
    poses = surface_poses(m, q)
    rows = host_rbf.rows(host_rbf.solve(m, q, x[nq:]))
    om = oracle.OracleModel.from_manipulator(m)
    od, ok, og = om.skin(poses, pts, rbf_rows=rows, culled=True)
    oacc = om.cost_accum(poses, pts, rbf_rows=rows)
    out = {"scene": "irb_and_squishable (7 hulls + squishable RBF + table), deformed; reference cloud tiled + G",
           "points": len(pts),
           "states": len(x), "oracle_cost": float(oacc[0])}
    ref_grad = None
    for prec in (64, 32):
        cf = CostFunctor(m, pts, precision=prec)
        c, g = cf.value_and_gradient(x)
        k, d, gr = cf.per_point(x)
        if prec == 64:
            ref_grad = g
        dd = np.abs(d - od)
        mis = k != ok
        agree = ~mis
        ang = np.abs(gr[agree] - og[agree]).max() if agree.any() else 0.0
        row = {"precision": prec, "max_abs_dd": float(dd.max()), "p99_abs_dd": float(np.quantile(dd, 0.99)),
               "kstar_mismatch": int(mis.sum()), "kstar_mismatch_frac": float(mis.mean()),
               "max_abs_dgrad_where_kstar_agrees": float(ang),
               "cost_rel_err": float(abs(c - oacc[0] - 10 * np.dot(x[nq:], x[nq:])) / oacc[0]),
               "dcdx_rel_err_vs_f64": float(np.linalg.norm(g - ref_grad) / np.linalg.norm(ref_grad))}
        if mis.any():
            # a flip is harmless only at a near-tie: |Δd*| there bounds the gap
            row["max_abs_dd_at_mismatch"] = float(dd[mis].max())
        if prec == 32 and exact_sample:
            # the fp32 context against the oracle's fp32 instantiation, bit for bit
            idx = np.sort(np.random.Generator(np.random.PCG64(seed + 7)).choice(len(pts), min(exact_sample, len(pts)),
                                                                                 replace=False))
            fd, fk, fg = om.skin(poses, pts[idx], rbf_rows=rows, precision=32)
            row["f32_exact_sample"] = {"points": int(len(idx)), "kstar_equal": bool(np.array_equal(k[idx], fk)),
                                       "d_equal": bool(np.array_equal(d[idx], fd)),
                                       "grad_equal": bool(np.array_equal(gr[idx], fg))}
        out[f"f{prec}"] = row
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=1 << 20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    res = sweep(a.points)
    print(json.dumps(res, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
