"""GPU twin of tests/test_manipulator_traces.py: the notebook's per-trial
traces (examples/manipulator.ipynb cells 9, 10, 14) against the PRODUCT path's
landscape — flash.gradientdescent.CostFunctor over the sensed cloud on cuda:0
(fsdf_value_and_gradient: FK, RBF weight solve, pass, adjoint, chain rule) —
instead of the C oracle's.

* the cost at every start-circle point of the 200 trials equals the oracle
  landscape's to 1e-9 (sums differ in order only), so the start-point PIT and
  its KS distances are the ones pinned on the CPU side (0.32 / 0.31: the
  measured divergence);
* the gradient at the trials' start points equals the oracle chain rule's;
* a NaiveSolver trial run on the product path (the notebook's step rule:
  rate·∇c on the undivided cost, component-wise clip) follows the oracle
  landscape's (err, cost) trajectory (to 1e-6 over the first 10 steps; the
  iteration amplifies rounding later) into the same basin.
"""
import math

import numpy as np
import pytest

import test_manipulator_traces as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu_landscape(oracle_mod):
    import test_notebook_pins as P
    from flash import Models
    from flash.gradientdescent import CostFunctor
    pts, _ = P.oracle_notebook(oracle_mod)  # the sensed cloud (raycast at x_true; GPU raycast ≡ oracle, test_gpu_rbf)
    cf = CostFunctor(Models.two_link_arm(False), pts)

    def cost(x):
        return float(cf.value_and_gradient(np.asarray(x, np.float64))[0])

    def value_and_gradient(x):
        c, g = cf.value_and_gradient(np.asarray(x, np.float64))
        return float(c), np.asarray(g)
    return cost, value_and_gradient


def test_start_circle_costs_equal_oracle(gpu_landscape, oracle_mod):
    cost_cpu, _, _ = T.oracle_landscape(oracle_mod)
    cost_gpu, _ = gpu_landscape
    th = np.linspace(0.0, 2 * math.pi, 36, endpoint=False)
    dirs = np.stack([np.cos(th), np.sin(th)], -1)
    for kind in ("far", "close"):
        for t in T.TR[kind]["trials"][::5]:
            for d in dirs[::3]:
                x = T.X_TRUE + t["err"][0] * d
                a, b = cost_gpu(x), cost_cpu(x)
                assert a == pytest.approx(b, rel=1e-9, abs=1e-15), (kind, x)


def test_pit_ks_on_product_path(gpu_landscape):
    """The landscape test (a) with the product path's costs: the KS distances
    are the measured divergence pinned on the CPU side."""
    cost, _ = gpu_landscape
    for kind in ("far", "close"):
        u = T._pit(cost, kind)
        assert T.ks_uniform(u) == pytest.approx(T.MEASURED_KS[kind], abs=0.03), kind
        assert np.median(u) < 0.4, kind


def test_start_gradients_equal_oracle(gpu_landscape, oracle_mod):
    _, vg_cpu, _ = T.oracle_landscape(oracle_mod)
    _, vg_gpu = gpu_landscape
    for kind in ("far", "close"):
        for t in T.TR[kind]["trials"][::10]:
            x = T.X_TRUE + t["err"][0] * np.array([0.6, 0.8])
            (ca, ga), (cb, gb) = vg_gpu(x), vg_cpu(x)
            assert ca == pytest.approx(cb, rel=1e-9)
            assert np.allclose(ga, gb, rtol=1e-7, atol=1e-12 * max(1.0, abs(cb)))


@pytest.mark.parametrize("kind", ["far", "close"])
def test_trial_trajectory_equals_oracle(gpu_landscape, oracle_mod, kind):
    _, vg_cpu, _ = T.oracle_landscape(oracle_mod)
    _, vg_gpu = gpu_landscape
    kw = {k: T.TR[kind]["solver"][k] for k in ("rate", "max_step", "iteration_limit")}
    t = T.TR[kind]["trials"][3]
    x0 = T.X_TRUE + t["err"][0] * np.array([math.cos(1.0), math.sin(1.0)])
    e_g, c_g = T.run_notebook_trial(vg_gpu, x0, kw)
    e_c, c_c = T.run_notebook_trial(vg_cpu, x0, kw)
    # the iteration map amplifies the 1e-13 summation-order differences of the
    # two landscapes (a 30-step descent through far-field local minima): the
    # first 10 steps agree to 1e-6, the trajectory ends in the same basin
    assert len(e_g) == len(e_c)
    assert np.allclose(e_g[:10], e_c[:10], rtol=1e-6, atol=1e-9)
    assert np.allclose(c_g[:10], c_c[:10], rtol=1e-6, atol=1e-12)
    assert abs(e_g[-1] - e_c[-1]) < 1e-2 and c_g[-1] == pytest.approx(c_c[-1], rel=1e-2)
