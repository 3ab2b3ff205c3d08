"""DepthSensors (src/depthsensors.jl) and DepthData (src/depthdata.jl)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, REFERENCE


def test_kinect_rays_geometry():
    from flash.depthsensors import Kinect
    s = Kinect(41, 41)
    assert s.rays.shape == (41, 41, 3)
    assert np.allclose(np.linalg.norm(s.rays, axis=-1), 1.0)
    assert np.allclose(s.rays[20, 20], [0, 0, 1])  # centre pixel (cx = cy = 21)
    # x spans ±tan(vfov)·20/21 before normalization (names swapped as in :20-24)
    r = s.rays[20, 0]
    assert r[0] / r[2] == pytest.approx(-np.tan(0.4682) * 20 / 21)
    r = s.rays[0, 20]
    assert r[1] / r[2] == pytest.approx(-np.tan(0.5449) * 20 / 21)


def _box_scene():
    from flash import Models
    import flash
    tab = Models.table()
    q = tab.mechanism.zero_configuration()
    q[4:7] = [0.0, 0.0, 0.0]
    return tab, flash.hull_poses(tab, q)


def test_oracle_raycast_box_top(oracle_mod):
    """Rays from above onto the table box top (z = 0.05): depth = (1 - 0.05)/cos θ."""
    tab, poses = _box_scene()
    om = oracle_mod.OracleModel.from_manipulator(tab)
    origin = np.array([0.0, 0.0, 1.0])
    ang = np.linspace(-0.2, 0.2, 21)
    rays = np.stack([np.sin(ang), np.zeros_like(ang), -np.cos(ang)], 1)
    d = om.raycast(poses, origin, rays)
    assert np.abs(d - 0.95 / np.cos(ang)).max() < 2e-5
    # the secant march follows the ray's LINE: pointing away from the box it
    # converges behind the origin (depth -0.95), as doRaycast does; sideways it misses
    back, miss = om.raycast(poses, origin, np.array([[0.0, 0.0, 1.0], [1.0, 0.0, 0.0]]))
    assert back == pytest.approx(-0.95, abs=2e-5)
    assert np.isnan(miss)


def test_read_point_cloud_fixture():
    from flash.depthdata import read_point_cloud, subsample
    pc = read_point_cloud(os.path.join(GOLDEN, "squishable_unsquished_head.txt"))
    assert len(pc) == 400
    assert np.allclose(pc.camera_origin, [1.38246, 0.768824, 1.48581])
    assert np.allclose(pc.positions[0], [0.414323, -0.0773639, 0.959196])
    assert np.allclose(pc.colors[0], [0.207843, 0.207843, 0.219608])
    assert repr(pc).startswith("PointCloud with origin: [1.38246, 0.768824, 1.48581] containing 400 points")
    assert len(subsample(pc.positions, 200)) == 2


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference data absent (GPU box)")
def test_read_reference_clouds():
    from flash.depthdata import read_point_cloud
    base = os.path.join(REFERENCE, "examples/data")
    assert len(read_point_cloud(os.path.join(base, "squishable_unsquished_xyzrgb.txt"))) == 25571
    assert len(read_point_cloud(os.path.join(base, "squishable_squished_xyzrgb.txt"))) == 25164
    with pytest.raises(ValueError):  # xyz-only: the reference indexes columns 4-6 and fails too
        read_point_cloud(os.path.join(base, "box_on_table_points.txt"))


def test_kinect_to_pointcloud_interleave():
    """convert_kinect_log_data.py:16-24: even samples are xyz, odd samples rgb,
    n_points = num // 2; then the notebook's [1:200:end] subsampling."""
    from flash.depthdata import kinect_to_pointcloud, pointcloud_positions
    rng = np.random.default_rng(3)
    num = 1001  # odd: the reference writes ceil(num/2) points but n_points = num // 2 (kept as is)
    x, y, z = rng.random((3, num)).astype(np.float32)
    msg = kinect_to_pointcloud(x, y, z, num, utime=42)
    assert msg["utime"] == 42 and msg["n_channels"] == 3 and msg["channel_names"] == ["r", "g", "b"]
    assert msg["n_points"] == num // 2 and len(msg["points"]) == (num + 1) // 2
    assert np.array_equal(msg["points"][3], [x[6], y[6], z[6]])
    assert np.array_equal(msg["channels"][:, 3], [x[7], y[7], z[7]])
    assert msg["channels"].shape == (3, num // 2)
    pos = pointcloud_positions(msg)
    assert pos.dtype == np.float64 and np.array_equal(pos[1], msg["points"][200].astype(np.float64))
