"""The reference's notebook-held numbers on the RBF + raycast + cost path
(examples/manipulator.ipynb), CPU oracle side. The GPU side is in
tests/test_gpu_rbf.py::test_manipulator_notebook_on_gpu.

Setup (cells 2 and 6): two_link_arm(false); Kinect(41, 41); camera
Translation(0,0,4) ∘ AngleAxis(π, x̂); sensed points = raycast at the true
state [π, 1.3]; the callback's undivided cost (src/tracking.jl:19) printed at
x = [6.66999, 0.0956194] → 9.71891410210385 (:5512) and at
x = [3.14754, 1.28436] → 1.3643120087735436e-4 (:14179).

Measured verdict on the formulation (tools/rbf_formulation_search.py,
profiles/rbf_formulation_search_r02.txt): the implemented s = f/|∇f| over the
r³ + affine interpolant satisfies the reference KAT (test/runtests.jl:17) but
gives 4.44× and 2.0× these costs; none of 55 candidate formulations (4 radial
kernels × 3 polynomial tails × 5 normalizations, each re-raycast) satisfies
all three numbers. The ratios are pinned below as a documented divergence and
the reference values are an expected failure (strict xfail: a formulation
that matches them would flip it)."""
import json
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN

PINS = json.load(open(os.path.join(GOLDEN, "notebook_pins.json")))["manipulator"]
# measured on this repo's formulation (CPU oracle == GPU); a change means the
# RBF semantics moved and DESIGN.md §2 must be revisited
MEASURED_RATIO = (4.436, 1.995)
MEASURED_HITS = 58


def camera():
    from flash.geometry import Transform, angle_axis
    th, ax = PINS["camera"]["angle_axis"][0], PINS["camera"]["angle_axis"][1:]
    return Transform(angle_axis(th, ax), np.asarray(PINS["camera"]["translation"], np.float64))


def _oracle_rows(m, q):
    import flash
    from flash import rbf as host_rbf
    q = m.mechanism.normalize(np.asarray(q, np.float64))
    return flash.core.surface_poses(m, q), host_rbf.rows(host_rbf.solve(m, q, np.zeros(0)))


def oracle_notebook(oracle_mod):
    """(sensed points, [cost at each pin]) with the C oracle."""
    from flash import Models
    from flash.depthsensors import Kinect, rays_in_world
    m = Models.two_link_arm(False)
    om = oracle_mod.OracleModel.from_manipulator(m)
    sensor = Kinect(PINS["sensor"]["rows"], PINS["sensor"]["cols"])
    tf = camera()
    rw = rays_in_world(sensor, tf)
    rw = rw / np.linalg.norm(rw, axis=-1, keepdims=True)
    poses, rows = _oracle_rows(m, PINS["x_true"])
    depth = om.raycast(poses, tf.t, rw.reshape(-1, 3), rbf_rows=rows).reshape(sensor.rays.shape[:2])
    hit = ~np.isnan(depth)
    pts = tf.apply(depth[hit][:, None] * sensor.rays[hit])
    costs = []
    for pin in PINS["pins"]:
        p, r = _oracle_rows(m, pin["x"])
        costs.append(float(om.cost_accum(p, pts, rbf_rows=r)[0]))
    return pts, costs


def test_notebook_setup_and_measured_divergence(oracle_mod):
    pts, costs = oracle_notebook(oracle_mod)
    assert len(pts) == MEASURED_HITS
    # the camera looks down from z = 4 onto the tube's upper half (radius ~0.14, RBF bulge)
    assert np.all((pts[:, 2] > 0) & (pts[:, 2] < 0.2))
    for pin, c, ratio in zip(PINS["pins"], costs, MEASURED_RATIO):
        assert c / pin["cost"] == pytest.approx(ratio, rel=2e-3), (pin["x"], c)


@pytest.mark.xfail(strict=True, reason="RBF formulation divergence: f/|grad f| over r^3+affine gives 4.44x / 2.0x "
                                       "the notebook costs (DESIGN.md §2; tools/rbf_formulation_search.py)")
def test_notebook_costs_match_reference(oracle_mod):
    _, costs = oracle_notebook(oracle_mod)
    for pin, c in zip(PINS["pins"], costs):
        assert c == pytest.approx(pin["cost"], rel=pin["rtol"])


def test_pin_rounding_sensitivity(oracle_mod):
    """The notebook prints x to 6 significant digits; moving x by that rounding
    changes the cost by far less than the measured divergence, so the ratios
    are real (tolerances of the xfail check: 1e-4 and 2e-3)."""
    from flash import Models
    pts, costs = oracle_notebook(oracle_mod)
    m = Models.two_link_arm(False)
    om = oracle_mod.OracleModel.from_manipulator(m)
    for pin, c in zip(PINS["pins"], costs):
        x = np.asarray(pin["x"])
        ulp6 = 0.5 * 10.0 ** (np.floor(np.log10(np.abs(x))) - 5)
        for sgn in ([1, 1], [1, -1], [-1, 1], [-1, -1]):
            p, r = _oracle_rows(m, x + np.asarray(sgn) * ulp6)
            c2 = om.cost_accum(p, pts, rbf_rows=r)[0]
            assert abs(c2 / c - 1) < pin["rtol"], (pin["x"], c, c2)


def test_camera_is_the_notebooks():
    tf = camera()
    assert np.allclose(tf.R, np.diag([1.0, -1.0, -1.0]), atol=1e-15)
    assert math.isclose(tf.R[2, 1], math.sin(math.pi))
    assert np.array_equal(tf.t, [0.0, 0.0, 4.0])
