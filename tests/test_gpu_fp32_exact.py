"""GPU: fp32 contexts bit for bit against the fp32 oracle.

The kernel's fp32 instantiation (hull_sdf<float>, rbf_field<float>, the
fp32 rows pose_body<float> writes) is restated operation for operation by
oracle/skin_impl.h compiled with R = float (oracle_skin_f32), so k*, d* and
∇d* of an fp32 context are compared EXACTLY — not within a tolerance — on the
IRB140 / M64 / quaternion-table goldens, the RBF scenes of BASELINE configs 3
and 5 (beanbag, irb_and_squishable), culled and brute force, the edge-case
points, and a sample of the full-size 2^20-point M64 cloud. (fp32 against the
fp64 oracle stays a tolerance check: test_gpu_parity.py::test_fp32_within_
tolerance, test_gpu_rbf.py::test_c5_precision_sweep_vs_oracle.)
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, rng

pytestmark = pytest.mark.gpu


def _manip(name):
    from flash import Models
    return {"c1_irb140": Models.irb140, "m64_2k": Models.arm_grid, "table_quat": Models.table,
            "c3_beanbag": Models.beanbag, "c5_scene": lambda: Models.irb_and_squishable()[0]}[name]()


def _ctx(m, cull=True, sort_points=False):
    from flash import _lib
    from flash.core import ConvexGeometry
    c = _lib.Context(device=0, precision=32, cull=cull, sort_points=sort_points)
    c.set_surfaces([("hull", (s.hull.vertices, s.hull.faces, s.hull.planes)) if isinstance(s, ConvexGeometry)
                    else ("rbf", len(s.surface_points) + len(s.skeleton_points)) for s in m.surfaces])
    return c


def _exact(got, want):
    (k, d, g), (od, ok, og) = got, want
    assert np.array_equal(k, ok), f"k* differs at {np.nonzero(k != ok)[0][:10]}"
    assert np.array_equal(d, od), f"max |Δd| = {np.abs(d - od).max()}"
    assert np.array_equal(g, og), f"max |Δg| = {np.abs(g - og).max()}"


@pytest.mark.parametrize("name", ["c1_irb140", "m64_2k", "table_quat", "c3_beanbag", "c5_scene"])
@pytest.mark.parametrize("cull", [True, False])
def test_fp32_golden_points_bit_exact(name, cull, oracle_mod):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    m = _manip(name)
    rows = z["rbf_rows"] if "rbf_rows" in z.files else None
    c = _ctx(m, cull=cull)
    c.set_points(z["points"])
    if rows is not None:
        c.set_rbf_params(rows)
    cost, acc, (k, d, g) = c.eval(z["poses"], per_point=True)
    om = oracle_mod.OracleModel.from_manipulator(m)
    want = om.skin(z["poses"], z["points"], rbf_rows=rows, precision=32)
    _exact((k, d, g), want)
    # the cost is Σ d² of the fp32 values (summed in fp64 by the kernel)
    assert cost == pytest.approx(np.dot(want[0], want[0]), rel=1e-6)
    c.close()


@pytest.mark.parametrize("order", ["raster", "shuffled"])
def test_fp32_m64_cloud_bit_exact(m64, oracle_mod, order):
    """65,573 M64 points (all 64 hulls in play), culled and brute force, with
    and without the resident Hilbert sort."""
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 401)
    pts = synthetic.depth_cloud(m64, qt, 65536 + 37, seed=402, order=order)
    poses = flash.hull_poses(m64, qe)
    want = oracle_mod.OracleModel.from_manipulator(m64).skin(poses, pts, precision=32)
    for cull, sort_points in ((True, False), (False, False), (True, True)):
        c = _ctx(m64, cull=cull, sort_points=sort_points)
        c.set_points(pts)
        _, _, got = c.eval(poses, per_point=True)
        _exact(got, want)
        c.close()


def test_fp32_edge_points_bit_exact(irb, oracle_mod):
    """Points on hull vertices, at hull centroids (deep inside), far field at
    1e3 m, duplicates; ragged sizes around wave boundaries."""
    import flash
    poses = flash.hull_poses(irb, np.zeros(6))
    verts = np.concatenate([s.hull.vertices @ p[:9].reshape(3, 3).T + p[9:] for s, p in zip(irb.surfaces, poses)])
    cents = np.stack([(s.hull.vertices @ p[:9].reshape(3, 3).T + p[9:]).mean(0) for s, p in zip(irb.surfaces, poses)])
    far = rng(5).normal(size=(50, 3)) * 1e3
    special = np.concatenate([verts, cents, far, verts[:10]])
    om = oracle_mod.OracleModel.from_manipulator(irb)
    c = _ctx(irb)
    for n in (1, 63, 65, 257, len(special)):
        pts = special[:n]
        c.set_points(pts)
        _, _, got = c.eval(poses, per_point=True)
        _exact(got, om.skin(poses, pts, precision=32))
    c.close()


def test_fp32_full_size_sample_bit_exact(m64, oracle_mod):
    """BASELINE config size (2^20 M64 points) in fp32: culled == brute force
    bit for bit over the whole cloud, and both == the fp32 oracle on a
    131,072-point sample (per-point results do not depend on the other points
    of a wave: the culling is exact-safe)."""
    import flash
    from flash import synthetic
    qt, qe = synthetic.perturbed_configuration(m64, 201)
    pts = synthetic.depth_cloud(m64, qt, 1 << 20, seed=202)
    poses = flash.hull_poses(m64, qe)
    out = {}
    for cull in (True, False):
        c = _ctx(m64, cull=cull)
        c.set_points(pts)
        out[cull] = c.eval(poses, per_point=True)[2]
        c.close()
    for a, b in zip(out[True], out[False]):
        assert np.array_equal(a, b)
    idx = np.sort(rng(9).choice(len(pts), 1 << 17, replace=False))
    want = oracle_mod.OracleModel.from_manipulator(m64).skin(poses, pts[idx], precision=32)
    _exact(tuple(x[idx] for x in out[True]), want)
