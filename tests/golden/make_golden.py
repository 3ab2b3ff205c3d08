"""Generate the golden vectors under tests/golden/ from the CPU oracle.

The reference (Julia 0.5 + un-vendored SpatialFields / EnhancedGJK /
RigidBodyDynamics / ForwardDiff) cannot run here, and its own tests hold no
vectors for the convex-hull path, so these fixtures are the
oracle's outputs on seeded inputs. They freeze the oracle (tests/test_oracle.py
re-derives them bit for bit) and are the target of the GPU parity tests.

    python tests/golden/make_golden.py

Files (npz, float64 / int32):
  c1_irb140.npz    BASELINE config 1: IRB140 (7 hulls, 6 DOF), 1,000 raster-order
                   points, q_true seed 11 / q_eval seed 12.
  m64_2k.npz       the metric model M64 (64 hulls, 48 DOF), 2,048 shuffled points.
  table_quat.npz   the floating table box (QuaternionFloating, un-normalized q), 512 points.
  c3_beanbag.npz   BASELINE config 3's model: deformable beanbag RBF (25 states), 1,000 points.
  c5_scene.npz     BASELINE config 5's scene: irb_and_squishable (9 surfaces, 63 states), 2,000 points.
Each holds: points, q, poses, d, kstar, grad, accum, and dcdq_fd (central
finite differences of the oracle cost through flash.mechanism FK, step 1e-6).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "point-cloud-signed-distance_amd"), os.path.join(ROOT, "oracle")]

import flash  # noqa: E402
from flash import Models, synthetic  # noqa: E402
import oracle as O  # noqa: E402


def fd_gradient(manip, om, q, pts, h=1e-6):
    g = np.zeros_like(q)
    for i in range(len(q)):
        qp, qm = q.copy(), q.copy()
        qp[i] += h
        qm[i] -= h
        cp = om.cost_accum(flash.hull_poses(manip, manip.mechanism.normalize(qp)), pts)[0]
        cm = om.cost_accum(flash.hull_poses(manip, manip.mechanism.normalize(qm)), pts)[0]
        g[i] = (cp - cm) / (2 * h)
    return g


def make(name, manip, q, pts, fd=True):
    om = O.OracleModel.from_manipulator(manip)
    poses = flash.hull_poses(manip, manip.mechanism.normalize(q))
    d, k, g = om.skin(poses, pts, threads=1)
    acc = om.cost_accum(poses, pts)
    out = dict(points=pts, q=q, poses=poses, d=d, kstar=k, grad=g, accum=acc)
    if fd:
        out["dcdq_fd"] = fd_gradient(manip, om, q, pts)
    np.savez_compressed(os.path.join(HERE, name), **out)
    print(name, len(pts), "pts, cost", acc[0], "inside", (d < 0).mean())


def main():
    irb = Models.irb140()
    q_true, q_eval = synthetic.perturbed_configuration(irb, 11)
    make("c1_irb140.npz", irb, q_eval, synthetic.depth_cloud(irb, q_true, 1000, seed=12, order="raster"))

    m64 = Models.arm_grid()
    q_true, q_eval = synthetic.perturbed_configuration(m64, 21)
    make("m64_2k.npz", m64, q_eval, synthetic.depth_cloud(m64, q_true, 2048, seed=22, order="shuffled"), fd=False)

    tab = Models.table()
    rng = np.random.Generator(np.random.PCG64(31))
    q = np.concatenate([rng.normal(size=4) * 0.7, [0.4, 0.0, 0.6]])  # un-normalized quaternion
    pts = np.array([0.4, 0.0, 0.6]) + rng.uniform(-0.45, 0.45, size=(512, 3))
    make("table_quat.npz", tab, q, pts)

    # RBF configs: BASELINE 3 (beanbag, deformed, 25 states) and 5 (the
    # irb_and_squishable scene, 63 states), small clouds
    from flash import rbf as host_rbf
    from flash.gradientdescent import gradient_from_accum
    for fname, (m, x0), npts, seed in (("c3_beanbag.npz", (Models.beanbag(), None), 1000, 41),
                                       ("c5_scene.npz", Models.irb_and_squishable(), 2000, 51)):
        r = np.random.Generator(np.random.PCG64(seed))
        nq = m.mechanism.num_positions
        x = np.zeros(flash.num_states(m)) if x0 is None else x0.copy()
        if x0 is None:
            x[:nq] = m.mechanism.zero_configuration()
            x[4:7] = 2 * r.random(3) ** 3          # examples/deformable_manipulator.ipynb:225
        x[nq:] = 0.5 * (r.random(len(x) - nq) - 0.5) * (0.1 if x0 is not None else 1.0)
        q = m.mechanism.normalize(x[:nq])
        solves = host_rbf.solve(m, q, x[nq:])
        rows = host_rbf.rows(solves)
        poses = flash.core.surface_poses(m, q)
        om = O.OracleModel.from_manipulator(m)
        centre = np.concatenate([s.centres for s in solves]).mean(0)
        pts = centre + r.normal(scale=0.35, size=(npts, 3))
        d, k, g = om.skin(poses, pts, threads=1, rbf_rows=rows)
        acc = om.cost_accum(poses, pts, rbf_rows=rows)
        np.savez_compressed(os.path.join(HERE, fname), points=pts, x=x, poses=poses, rbf_rows=rows, d=d, kstar=k,
                            grad=g, accum=acc, dcdx=gradient_from_accum(m, x, acc, solves, 10))
        print(fname, npts, "pts, cost", acc[0], "k* hist", np.bincount(k))


if __name__ == "__main__":
    main()
