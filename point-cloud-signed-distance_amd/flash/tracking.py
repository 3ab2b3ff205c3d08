"""module Flash.Tracking (src/tracking.jl) — `track!`.

estimate_state(manipulator, sensed_points, x_estimated; callback, solver)
(src/tracking.jl:8-27): wraps the cost as c/N with a callback(x, c) on every
evaluation (:16-21), hands it to a gradient-descent solver warm-started at
x_estimated (:23-26), and returns the solution.

The solver lives in the un-vendored SimpleGradientDescent.jl @0fcc1f95
(REQUIRE.dev:24). `NaiveSolver` below restates its published interface
(rate, max_step, iteration_limit, gradient_convergence_tolerance,
precondition_divisors — kwargs used at examples/irb140.ipynb cell 9 and
examples/squishable.ipynb) with a plain clipped gradient step; trajectory
parity with the Julia solver is UNPINNED (no reference test covers it).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .core import Manipulator, num_states
from .gradientdescent import CostFunctor


@dataclass
class NaiveSolver:
    num_vars: int
    rate: float = 0.1
    max_step: float = 0.5
    iteration_limit: int = 30
    gradient_convergence_tolerance: float = 0.0
    precondition_divisors: np.ndarray | None = None

    def optimize(self, value_and_gradient, x0):
        x = np.array(x0, np.float64, copy=True)
        div = np.ones(self.num_vars) if self.precondition_divisors is None else np.asarray(self.precondition_divisors)
        f = None
        for _ in range(self.iteration_limit):
            f, g = value_and_gradient(x)
            if np.linalg.norm(g) < self.gradient_convergence_tolerance:
                break
            step = np.clip(-self.rate * g / div, -self.max_step, self.max_step)
            x = x + step
        return x, f


def estimate_state(manipulator: Manipulator, sensed_points, x_estimated, callback=None, solver=None,
                   device: int = 0, precision: int = 64):
    """Tracking.estimate_state (src/tracking.jl:8-27). Returns the solution x.

    The default callback accepts (x, c): the reference's default `x -> ()` is
    called with two arguments (src/tracking.jl:9 vs :19) and would throw."""
    pts = np.asarray(sensed_points, np.float64).reshape(-1, 3)
    n = max(len(pts), 1)
    solver = solver or NaiveSolver(num_states(manipulator), rate=0.1, max_step=0.5, iteration_limit=30)
    cost = CostFunctor(manipulator, pts, device=device, precision=precision)

    def wrapped(x):
        c, g = cost.value_and_gradient(x)
        if callback is not None:
            callback(x, c)
        return c / n, g / n

    x, _ = solver.optimize(wrapped, np.asarray(x_estimated, np.float64))
    return x
