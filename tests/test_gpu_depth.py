"""GPU raycaster (fsdf_raycast) vs the oracle's doRaycast restatement."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def test_raycast_irb140_parity(irb, oracle_mod):
    """examples/irb140.ipynb cells 4 and 8: Kinect(41, 41) at (0, 1.5, 0.5),
    AngleAxis(pi/2, 1, 0, 0); depths bit-identical to the oracle."""
    import flash
    from flash.depthsensors import Kinect, raycast_depths, raycast_points, rays_in_world
    from flash.geometry import Transform, angle_axis
    sensor = Kinect(41, 41)
    tf = Transform(angle_axis(np.pi / 2, [1, 0, 0]), np.array([0.0, 1.5, 0.5]))
    state = flash.ManipulatorState(irb)
    sk = flash.skin(state)
    d = raycast_depths(sk, sensor, tf)
    rw = rays_in_world(sensor, tf)
    rw = rw / np.linalg.norm(rw, axis=-1, keepdims=True)
    od = oracle_mod.OracleModel.from_manipulator(irb).raycast(flash.hull_poses(irb, state.q), tf.t, rw.reshape(-1, 3))
    assert np.array_equal(np.isnan(d.ravel()), np.isnan(od))
    assert np.array_equal(d.ravel()[~np.isnan(od)], od[~np.isnan(od)])
    pts = raycast_points(sk, sensor, tf)
    assert len(pts) == (~np.isnan(od)).sum() > 50
    # hits lie on the skin
    assert np.abs(sk(pts)).max() < 1e-2


def test_raycast_rbf_and_cost_at_truth(oracle_mod):
    """Raycast the deformable beanbag, then the tracking cost of those points
    at the true state is ~0 (the points are on the skin)."""
    import flash
    from flash import Models
    from flash.depthsensors import Kinect, raycast
    from flash.geometry import Transform, angle_axis
    from flash.gradientdescent import CostFunctor
    m = Models.beanbag()
    st = flash.ManipulatorState(m)
    st.deformation_data[:] = 0.1 * np.sin(np.arange(18))
    tf = Transform(angle_axis(np.pi, [1, 0, 0]), np.array([0.0, 0.0, 4.0]))
    pts = raycast(st, Kinect(32, 32), tf)
    assert len(pts) > 100
    x = np.concatenate([st.q, st.deformation_data])
    c = CostFunctor(m, pts)(x) - 10 * np.dot(st.deformation_data, st.deformation_data)
    d = flash.skin(st)(pts)
    # doRaycast keeps a hit when |SDF| <= 1000·EPS = 1e-2 (src/depthsensors.jl:76)
    assert np.abs(d).max() <= 1e-2 * (1 + 1e-6)
    assert np.median(np.abs(d)) < 1e-5
    assert c == pytest.approx(np.dot(d, d), rel=1e-9, abs=1e-18)
