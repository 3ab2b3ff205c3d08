#!/usr/bin/env python3
"""Bit-for-bit agreement of A/B pass-kernel builds (GPU box): per-point k*, d*,
∇d* and the accumulator of every library against the first one, on the M64
bench cloud (shuffled + device sort). The first library is the validated
build; the parity suite (tests/, -m gpu) then pins the chosen one.

    python tools/ab_check.py ab/base.so ab/new.so [--points N]
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud-signed-distance_amd"))


def run_one(lib, n, out):
    import flash
    from flash import Models, synthetic, _lib
    m = Models.arm_grid()
    qt, qe = synthetic.perturbed_configuration(m, 1234)
    pts = synthetic.depth_cloud(m, qt, n, seed=1234 + 17, order="shuffled")
    ctx = _lib.Context(device=0, sort_points=True)
    ctx.set_model([(s.hull.vertices, s.hull.faces, s.hull.planes) for s in m.surfaces])
    ctx.set_points(pts)
    cost, acc, (k, d, g) = ctx.eval(flash.hull_poses(m, qe), per_point=True)
    np.savez(out, k=k, d=d, g=g, acc=acc)


def main():
    args = sys.argv[1:]
    n = 1 << 20
    if "--points" in args:
        i = args.index("--points")
        n = int(args[i + 1])
        del args[i:i + 2]
    if len(args) == 3 and args[0] == "--child":
        run_one(args[1], n, args[2])
        return 0
    outs = []
    for j, lib in enumerate(args):
        out = f"/tmp/ab_check_{j}.npz"
        env = dict(os.environ, FLASHSDF_LIB=os.path.abspath(lib))
        subprocess.run([sys.executable, __file__, "--child", lib, out, "--points", str(n)], env=env, check=True,
                       timeout=300)
        outs.append(np.load(out))
    ref = outs[0]
    ok = True
    for lib, o in zip(args[1:], outs[1:]):
        same = all(np.array_equal(ref[x], o[x]) for x in ("k", "d", "g"))
        accrel = float(np.max(np.abs(ref["acc"] - o["acc"]) / (np.abs(ref["acc"]) + 1e-30)))
        nk = int(np.sum(ref["k"] != o["k"]))
        nd = int(np.sum(ref["d"] != o["d"]))
        dd = float(np.max(np.abs(ref["d"] - o["d"]))) if nd else 0.0
        ng = int(np.sum(np.any(ref["g"] != o["g"], axis=1)))
        print(f"{os.path.basename(lib)}: per-point bit-exact={same} (k* mismatches {nk}, d {nd} max|dd| {dd:.3e}, "
              f"grad {ng}), accum max rel {accrel:.2e}")
        if nd:
            i = np.nonzero(ref["d"] != o["d"])[0][:5]
            print("   first:", i.tolist(), ref["d"][i].tolist(), o["d"][i].tolist(), ref["k"][i].tolist(), o["k"][i].tolist())
        ok &= same and accrel < 1e-9
    print("AB_CHECK", "OK" if ok else "FAIL")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
