"""module Flash.GradientDescent (src/gradientdescent.jl).

  default_deformation_cost_weight = 10          :7
  flatten(state) / unflatten!(state, x)         :9-17
  normalize!(mechanism_state)                   :19-26
  cost(state, sensed_points, weight)            :28-39
  CostFunctor(manipulator, sensed_points)(x)    :41-57
In the reference the gradient of CostFunctor comes from ForwardDiff (Dual{9}
chunk passes, ⌈n/9⌉ full point passes per gradient, examples/irb_and_squishable
.ipynb:482). Here ONE GPU residual pass returns the cost and the per-hull
wrenches, and `value_and_gradient` chains them analytically to ∂c/∂x.
"""
from __future__ import annotations

import numpy as np

from .core import ConvexGeometry, InterpolatingGeometry, Manipulator, ManipulatorState, prepare_pass

default_deformation_cost_weight = 10


def flatten(state: ManipulatorState) -> np.ndarray:
    """vcat(q, deformation_data) (src/gradientdescent.jl:9-11)."""
    return np.concatenate([state.q, state.deformation_data])


def unflatten(state: ManipulatorState, x) -> None:
    """unflatten!(state, x) (src/gradientdescent.jl:13-17)."""
    x = np.asarray(x, np.float64)
    nq = state.manipulator.mechanism.num_positions
    state.q[:] = x[:nq]
    state.deformation_data[:] = x[nq:]


def normalize(state: ManipulatorState) -> None:
    """normalize!(state.mechanism_state) in place (src/gradientdescent.jl:19-26)."""
    state.q[:] = state.manipulator.mechanism.normalize(state.q)


def _regularizer(state: ManipulatorState, weight) -> float:
    return float(weight) * float(np.dot(state.deformation_data, state.deformation_data))


def cost(state: ManipulatorState, sensed_points, deformation_cost_weight=default_deformation_cost_weight,
         device: int = 0, precision: int = 64) -> float:
    """Σ_p skin(p)^2 + w·Σ‖δ‖² (src/gradientdescent.jl:28-39); normalizes q in place first."""
    normalize(state)
    m = state.manipulator
    ctx = m.engine(device, precision)
    pts = np.asarray(sensed_points, np.float64).reshape(-1, 3)
    d = np.zeros(0)
    if len(pts):
        poses, _ = prepare_pass(ctx, m, state.q, state.deformation_data)
        d, _, _ = ctx.skin(poses, pts)
    return float(np.dot(d, d)) + _regularizer(state, deformation_cost_weight)


def gradient_from_accum(manip: Manipulator, x: np.ndarray, accum: np.ndarray, solves, weight) -> np.ndarray:
    """∂c/∂x from one pass's accumulator: hull wrenches (slot = surface index)
    plus the RBF adjoint block, contracted with the joint motion subspaces;
    ∂c/∂δ from the RBF block plus the regularizer 2wδ."""
    mech = manip.mechanism
    nq = mech.num_positions
    S = len(manip.surfaces)
    sb = getattr(manip, "_surface_body", None)
    if sb is None or len(sb) != S:
        sb = np.array([s.body if isinstance(s, ConvexGeometry) else -1 for s in manip.surfaces], np.int32)
        manip._surface_body = sb
    gd = 2.0 * weight * np.asarray(x[nq:], np.float64)
    body_w = None
    if solves:
        from . import rbf
        w_rbf, g_rbf = rbf.chain(manip, mech.normalize(x[:nq]), solves, accum[1 + 6 * S:], manip.num_deformations())
        body_w = w_rbf
        gd = gd + g_rbf
    # the gradient is taken at the caller's (un-normalized) x: the chain rule
    # includes the normalization projection (src/gradientdescent.jl:30)
    gq = mech.config_gradient(np.asarray(x[:nq], np.float64), body_w, sb, np.asarray(accum[1:1 + 6 * S]))
    return np.concatenate([gq, gd])


def native_capable(manipulator: Manipulator) -> bool:
    """Scenes fsdf_value_and_gradient handles: convex hulls and RBF skins."""
    return all(isinstance(s, (ConvexGeometry, InterpolatingGeometry)) for s in manipulator.surfaces)


def register_native(manipulator: Manipulator, ctx, weight) -> None:
    """Declare the mechanism, surface bodies/frames, RBF centres and
    deformations to the context (fsdf_set_mechanism, fsdf_set_rbf_centres,
    fsdf_set_deformations) for its native iterations."""
    m = manipulator
    surf = m.surfaces
    hull = [isinstance(s, ConvexGeometry) for s in surf]
    eye, zero = np.eye(3), np.zeros(3)
    ctx.set_mechanism(m.mechanism, [s.body if h else -1 for s, h in zip(surf, hull)],
                      [s.frame.R if h else eye for s, h in zip(surf, hull)],
                      [s.frame.t if h else zero for s, h in zip(surf, hull)])
    row0 = 0  # deformation rows in surface order (flash/rbf.py solve)
    for k, s in enumerate(surf):
        nd = s.num_deformations()
        if isinstance(s, InterpolatingGeometry):
            rows = np.arange(row0, row0 + nd, dtype=np.int32) if nd else None
            ctx.set_rbf_centres(k, s.surface_points, s.skeleton_points, rows)
        row0 += nd
    ctx.set_deformations(m.num_deformations(), weight)
    ctx._mechanism_of = (m, weight)


class CostFunctor:
    """CostFunctor(manipulator, sensed_points) (src/gradientdescent.jl:41-57).

    The sensed cloud is uploaded once (the reference keeps it by reference for
    every evaluation); each call ships only the hull poses."""

    def __init__(self, manipulator: Manipulator, sensed_points, device: int = 0, precision: int = 64,
                 deformation_cost_weight=default_deformation_cost_weight):
        self.manipulator = manipulator
        self.sensed_points = np.ascontiguousarray(sensed_points, np.float64).reshape(-1, 3)
        self.weight = deformation_cost_weight
        self.state = ManipulatorState(manipulator)
        self.ctx = manipulator.engine(device, precision)
        # a private context would be needed to keep two functors resident at once
        self.ctx.set_points(self.sensed_points)
        self._resident = id(self)
        manipulator._resident_cloud = self._resident
        # the whole iteration (FK, RBF weight solve, pass, chain rule,
        # regularizer) in one native call (fsdf_value_and_gradient)
        self._native = native_capable(manipulator)
        if self._native and getattr(self.ctx, "_mechanism_of", None) != (manipulator, self.weight):
            self._register_native()

    def _register_native(self):
        register_native(self.manipulator, self.ctx, self.weight)

    def set_sensed_points(self, sensed_points):
        """Swap the resident cloud (a new frame): one upload + device sort; the
        functor, its state and the device model are kept. The array given to
        prefetch_sensed_points last is made resident from its device copy."""
        pre, src = getattr(self, "_prefetched", None), getattr(self, "_prefetched_src", None)
        self._prefetched = self._prefetched_src = None
        if pre is not None and sensed_points is src:  # (the object prefetched: its device copy)
            self.sensed_points = pre
            self.ctx.set_points_prefetched()
        else:
            self.sensed_points = np.ascontiguousarray(sensed_points, np.float64).reshape(-1, 3)
            self.ctx.set_points(self.sensed_points)
        self.manipulator._resident_cloud = self._resident

    def prefetch_sensed_points(self, sensed_points):
        """Start the NEXT frame's upload now (fsdf_prefetch_points: a copy on a
        stream of the context's own, running under the current frame's passes —
        fully when the array is page-locked); set_sensed_points(that array)
        then skips the host-to-device copy. The array must not change until then."""
        self._prefetched = np.ascontiguousarray(sensed_points, np.float64).reshape(-1, 3)
        self._prefetched_src = sensed_points
        self.ctx.prefetch_points(self._prefetched)

    def regroup(self):
        """Once per frame, after its first evaluation: regroup the resident
        cloud by each point's nearest surface in that pass (fsdf_regroup_points;
        hull-only scenes). Later evaluations give the same per-point results and
        sums to rounding, faster on large clouds."""
        self._ensure_resident()
        self.ctx.regroup_points()

    def _ensure_resident(self):
        if getattr(self.manipulator, "_resident_cloud", None) != self._resident:
            self.ctx.set_points(self.sensed_points)
            self.manipulator._resident_cloud = self._resident

    def _pass(self, x, per_point=False):
        unflatten(self.state, x)
        normalize(self.state)
        self._ensure_resident()
        poses, self._solves = prepare_pass(self.ctx, self.manipulator, self.state.q, self.state.deformation_data)
        c, accum, extras = self.ctx.eval(poses, per_point)
        return c + _regularizer(self.state, self.weight), accum, extras

    def __call__(self, x) -> float:
        return self._pass(x)[0]

    def value_and_gradient(self, x):
        """(c(x), ∂c/∂x) from one residual pass."""
        x = np.asarray(x, np.float64)
        if self._native:
            self._ensure_resident()
            if getattr(self.ctx, "_mechanism_of", None) != (self.manipulator, self.weight):
                self._register_native()  # another functor of this engine registered its own
            return self.ctx.value_and_gradient(x)
        c, accum, _ = self._pass(x)
        return c, gradient_from_accum(self.manipulator, x, accum, self._solves, self.weight)

    def descend(self, x, iteration_limit, rate, max_step, tolerance=0.0, divisors=None, n_points=1.0):
        """The NaiveSolver loop over value_and_gradient in one native call
        (fsdf_descend); native-capable scenes only. Returns (x, f, iterations)."""
        if not self._native:
            raise NotImplementedError("descend: scene is not native-capable")
        self._ensure_resident()
        if getattr(self.ctx, "_mechanism_of", None) != (self.manipulator, self.weight):
            self._register_native()
        return self.ctx.descend(x, iteration_limit, rate, max_step, tolerance, divisors, n_points)

    def per_point(self, x):
        """(d*, k*, ∇d*) for every sensed point at configuration x."""
        return self._pass(x, per_point=True)[2]
