"""module Flash.Tracking (src/tracking.jl) — `track!`.

estimate_state(manipulator, sensed_points, x_estimated; callback, solver)
(src/tracking.jl:8-27): wraps the cost as c/N with a callback(x, c) on every
evaluation (:16-21), hands it to a gradient-descent solver warm-started at
x_estimated (:23-26), and returns the solution.

The frame loop around it is the notebooks' (examples/irb_and_squishable.ipynb
cells 11-12): for every KINECT_POINTS_REDUCED message, sensed_points =
msg.points[1:200:end] and gradient_descent!(state, model, sensed_points) runs
estimate_state from the current state with NaiveSolver(num_states; rate=0.5,
max_step=0.1, iteration_limit=1) and writes the solution back into the state
(unflatten!) — the warm start carried from frame to frame. `track` restates
that loop; `Tracker` is its resident form (one device context and CostFunctor
for the whole sequence, the cloud swapped per frame).

The solver lives in the un-vendored SimpleGradientDescent.jl @0fcc1f95
(REQUIRE.dev:24). `NaiveSolver` below restates its interface (num_vars, rate,
max_step, iteration_limit, gradient_convergence_tolerance,
precondition_divisors — the kwargs examples/irb140.ipynb cell 9 and
examples/squishable.ipynb cell 9 pass). Its update rule is pinned by the
reference notebook's own per-trial traces (examples/manipulator.ipynb cells
9/10/14, fixture tests/golden/manipulator_traces.json,
tests/test_manipulator_traces.py): the step is −rate·∇f (κ = rate measured
within 2 % from single trajectories at two rates), clipped component-wise at
max_step (the far set's largest |Δerr| per step is max_step·√2), one
objective evaluation per iteration, and a positive default convergence
tolerance (trials stop early; 1e-3 estimated from where they stop). Trajectory
parity on the RBF scene itself is not reached: the landscape diverges
(DESIGN.md §2).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np

from .core import Manipulator, ManipulatorState, num_states
from .gradientdescent import CostFunctor, flatten, unflatten


@dataclass
class NaiveSolver:
    """NaiveSolver(num_vars; rate, max_step, iteration_limit,
    gradient_convergence_tolerance, precondition_divisors): per iteration
    g ← ∇f(x) ./ precondition_divisors; stop when ‖g‖ < tolerance; else
    x ← x + clamp(−rate·g, ±max_step) (component-wise). Rule and default
    tolerance per the notebook traces (module docstring)."""
    num_vars: int
    rate: float = 0.1
    max_step: float = 0.5
    iteration_limit: int = 30
    gradient_convergence_tolerance: float = 1e-3
    precondition_divisors: np.ndarray | None = None
    iterations: int = field(default=0, init=False)  # of the last optimize

    def optimize(self, value_and_gradient, x0):
        x = np.array(x0, np.float64, copy=True)
        div = np.ones(self.num_vars) if self.precondition_divisors is None else np.broadcast_to(
            np.asarray(self.precondition_divisors, np.float64), x.shape)
        f = None
        self.iterations = 0
        for _ in range(self.iteration_limit):
            f, g = value_and_gradient(x)
            self.iterations += 1
            g = g / div
            if np.linalg.norm(g) < self.gradient_convergence_tolerance:
                break
            x = x + np.clip(-self.rate * g, -self.max_step, self.max_step)
        return x, f


def _default_solver(manipulator):
    # src/tracking.jl:10-13
    return NaiveSolver(num_states(manipulator), rate=0.1, max_step=0.5, iteration_limit=30)


def _optimize(cost: CostFunctor, n_points: int, x_estimated, callback, solver):
    """wrapped_cost (src/tracking.jl:16-21) over a CostFunctor, then optimize!.
    Without a callback, a NaiveSolver runs natively (fsdf_descend: the same
    arithmetic, no Python round trip per iteration)."""
    n = max(n_points, 1)
    if callback is None and type(solver) is NaiveSolver and cost._native:
        x0 = np.asarray(x_estimated, np.float64)
        div = solver.precondition_divisors
        if div is not None:  # NaiveSolver broadcasts the divisors; fsdf_descend takes one per entry
            div = np.broadcast_to(np.asarray(div, np.float64), x0.shape).copy()
        x, _, its = cost.descend(x0, solver.iteration_limit, solver.rate, solver.max_step,
                                 solver.gradient_convergence_tolerance, div, n)
        solver.iterations = its
        return x

    def wrapped(x):
        c, g = cost.value_and_gradient(x)
        if callback is not None:
            callback(x, c)
        return c / n, g / n

    x, _ = solver.optimize(wrapped, np.asarray(x_estimated, np.float64))
    return x


def estimate_state(manipulator: Manipulator, sensed_points, x_estimated, callback=None, solver=None,
                   device: int = 0, precision: int = 64):
    """Tracking.estimate_state (src/tracking.jl:8-27). Returns the solution x.

    The default callback accepts (x, c): the reference's default `x -> ()` is
    called with two arguments (src/tracking.jl:9 vs :19) and would throw."""
    pts = np.asarray(sensed_points, np.float64).reshape(-1, 3)
    solver = solver or _default_solver(manipulator)
    cost = CostFunctor(manipulator, pts, device=device, precision=precision)
    return _optimize(cost, len(pts), x_estimated, callback, solver)


def notebook_frame_solver(manipulator):
    """gradient_descent!'s solver (examples/irb_and_squishable.ipynb cell 11)."""
    return NaiveSolver(num_states(manipulator), rate=0.5, max_step=0.1, iteration_limit=1)


class Tracker:
    """The frame loop with everything resident: one CostFunctor (device model,
    context, ManipulatorState) for the whole sequence; per frame the cloud is
    swapped (one upload + device sort) and estimate_state runs warm-started
    from the previous frame's solution. Timings per frame and per solver
    iteration are recorded (host FK + pass + chain rule, end to end)."""

    def __init__(self, manipulator: Manipulator, state: ManipulatorState | None = None, solver=None,
                 device: int = 0, precision: int = 64):
        self.manipulator = manipulator
        self.state = state if state is not None else ManipulatorState(manipulator)
        self.solver = solver or notebook_frame_solver(manipulator)
        self.cost = CostFunctor(manipulator, np.zeros((0, 3)), device=device, precision=precision)
        self.frame_ms: list[float] = []
        self.set_points_ms: list[float] = []
        self.iterations: list[int] = []

    def step(self, sensed_points, callback=None, next_points=None) -> np.ndarray:
        """gradient_descent!(state, model, sensed_points): one frame.
        next_points (optional): the next frame's cloud, whose upload then runs
        under this frame's solver iterations (CostFunctor.prefetch_sensed_points)."""
        pts = np.asarray(sensed_points, np.float64).reshape(-1, 3)
        t0 = time.perf_counter()
        self.cost.set_sensed_points(sensed_points)  # (the object itself: a prefetched frame is matched by identity)
        if next_points is not None:
            self.cost.prefetch_sensed_points(next_points)
        t1 = time.perf_counter()
        x = _optimize(self.cost, len(pts), flatten(self.state), callback, self.solver)
        unflatten(self.state, x)
        t2 = time.perf_counter()
        self.set_points_ms.append((t1 - t0) * 1e3)
        self.frame_ms.append((t2 - t0) * 1e3)
        self.iterations.append(getattr(self.solver, "iterations", 0))
        return x

    def iteration_ms(self) -> float:
        """Mean end-to-end milliseconds per solver iteration (excluding the cloud swap)."""
        its = sum(self.iterations)
        return (sum(self.frame_ms) - sum(self.set_points_ms)) / its if its else float("nan")


def track(manipulator: Manipulator, frames, state: ManipulatorState | None = None, solver=None, callback=None,
          device: int = 0, precision: int = 64):
    """for event in log: gradient_descent!(state, model, sensed_points)
    (examples/irb_and_squishable.ipynb cells 11-12). `frames` yields sensed
    clouds ([n,3]); returns (the per-frame solutions [F, n_states], the Tracker)."""
    tr = Tracker(manipulator, state, solver, device, precision)
    xs = []
    it = iter(frames)
    cur = next(it, None)
    while cur is not None:
        nxt = next(it, None)  # (its upload overlaps this frame's iterations)
        xs.append(tr.step(cur, callback, next_points=nxt))
        cur = nxt
    return np.array(xs), tr
