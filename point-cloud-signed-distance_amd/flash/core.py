"""Core geometry and state types + the scene signed-distance closure.

Mirrors module Flash (src/Flash.jl):
  BodyGeometry / ConvexGeometry / Rigid- & DeformableInterpolatingSkin  :30-48
  Manipulator (mechanism + surfaces)                                    :62-67
  ManipulatorState (configuration + deformation views)                  :71-125
  num_deformations / num_states                                         :79-90
  surfaces(state), skin(state)                                          :261-268
The closure `skin(state)` evaluates every point on the GPU through
libflashsdf (one launch per batch of points), never on the CPU.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .geometry import ConvexHull, Transform
from .mechanism import Mechanism


class BodyGeometry:
    """abstract BodyGeometry (src/Flash.jl:30)."""

    def num_deformations(self) -> int:
        return 0


class ConvexGeometry(BodyGeometry):
    """ConvexGeometry{GeomType}(geometry, frame) (src/Flash.jl:45-48).

    `hull` is expressed in the geometry frame; `frame` is that frame's fixed
    transform relative to body `body` (the URDF visual origin, src/models.jl:154-164)."""

    def __init__(self, hull: ConvexHull, body: int, frame: Transform | None = None, name: str = ""):
        self.hull = hull
        self.body = body
        self.frame = frame or Transform.identity()
        self.name = name

    def __repr__(self):
        return f"ConvexGeometry({self.name or 'hull'}, {len(self.hull.vertices)} vertices, body={self.body})"


class InterpolatingGeometry(BodyGeometry):
    """abstract InterpolatingGeometry (src/Flash.jl:33): RBF skins over surface
    points (value 0) and skeleton points (value −1), src/Flash.jl:207-213."""

    def __init__(self, surface_points, skeleton_points):
        # lists of (body index, xyz in body frame)
        self.surface_points = [(int(b), np.asarray(p, np.float64)) for b, p in surface_points]
        self.skeleton_points = [(int(b), np.asarray(p, np.float64)) for b, p in skeleton_points]


class RigidInterpolatingSkin(InterpolatingGeometry):
    """src/Flash.jl:40-43."""


class DeformableInterpolatingSkin(InterpolatingGeometry):
    """src/Flash.jl:35-38: every surface point carries a 3-vector deformation."""

    def num_deformations(self) -> int:
        return len(self.surface_points)


class Manipulator:
    """Manipulator{T}(mechanism, surfaces) (src/Flash.jl:62-65)."""

    def __init__(self, mechanism: Mechanism, surfaces: list[BodyGeometry]):
        self.mechanism = mechanism
        self.surfaces = list(surfaces)
        self._engines: dict = {}

    def __repr__(self):
        return (f"Manipulator with {self.mechanism.num_bodies} links and {len(self.surfaces)} surfaces")

    def num_deformations(self) -> int:
        return sum(s.num_deformations() for s in self.surfaces)

    def convex_surfaces(self) -> list[ConvexGeometry]:
        return [s for s in self.surfaces if isinstance(s, ConvexGeometry)]

    def engine(self, device: int = 0, precision: int = 64, cull: bool = True,
               sort_points: bool = True, slot: int = 0) -> "_lib.Context":
        """The native context holding this model on `device` (created once).
        sort_points: the resident cloud is Hilbert-ordered on the device once per
        frame (set_points); outputs still come back in caller order. slot: further
        independent contexts of the same model (each its own cloud copy, stream
        and buffers — passes over independent states in flight together)."""
        key = (device, precision, cull, sort_points, slot)
        ctx = self._engines.get(key)
        if ctx is None:
            ctx = _lib.Context(device=device, precision=precision, cull=cull, sort_points=sort_points)
            spec = []
            for s in self.surfaces:
                if isinstance(s, ConvexGeometry):
                    spec.append(("hull", (s.hull.vertices, s.hull.faces, s.hull.planes)))
                else:
                    spec.append(("rbf", len(s.surface_points) + len(s.skeleton_points)))
            ctx.set_surfaces(spec)
            self._engines[key] = ctx
        return ctx

    def has_rbf(self) -> bool:
        return any(isinstance(s, InterpolatingGeometry) for s in self.surfaces)

    def invalidate(self):
        """Drop device contexts and the surface caches (after editing surfaces /
        merging; the caches key on the surface list's identity and length)."""
        for ctx in self._engines.values():
            ctx.close()
        self._engines.clear()
        for attr in ("_frame_cache", "_surface_plan", "_surface_body"):
            if hasattr(self, attr):
                delattr(self, attr)


def num_deformations(x) -> int:
    return x.num_deformations()


def num_states(manip: Manipulator) -> int:
    """num_positions + 3·#deformable points (src/Flash.jl:90)."""
    return manip.mechanism.num_positions + 3 * manip.num_deformations()


@dataclass
class ManipulatorState:
    """ManipulatorState (src/Flash.jl:71-125). `q` is the RBD configuration,
    `deformation_data` the flat δ vector; `deformations[i]` are (n,3) views,
    one per surface, in surface order (src/Flash.jl:97-104)."""
    manipulator: Manipulator
    q: np.ndarray = None
    deformation_data: np.ndarray = None
    deformations: list = field(default_factory=list)

    def __post_init__(self):
        m = self.manipulator
        if self.q is None:
            self.q = m.mechanism.zero_configuration()
        if self.deformation_data is None:
            self.deformation_data = np.zeros(3 * m.num_deformations())
        self.deformations = []
        off = 0
        for s in m.surfaces:
            nd = s.num_deformations()
            self.deformations.append(self.deformation_data[off:off + 3 * nd].reshape(nd, 3))
            off += 3 * nd

    def set_configuration(self, q):
        self.q[:] = q


def _posed(manip: Manipulator, q: np.ndarray, surfaces) -> np.ndarray:
    """[n,12] T_world_body · T_body_geometry for the given convex surfaces (batched)."""
    if not surfaces:
        return np.zeros((0, 12))
    R, t, _, _ = manip.mechanism.body_transform_arrays(q)
    # surface lists only grow during model construction (Models.merge!): the
    # list object and its length identify its contents
    key = (id(surfaces), len(surfaces))
    cache = getattr(manip, "_frame_cache", None)
    if cache is None or cache[0] != key:
        cache = (key, np.array([s.body for s in surfaces]), np.stack([s.frame.R for s in surfaces]),
                 np.stack([s.frame.t for s in surfaces])[:, :, None])
        manip._frame_cache = cache
    _, b, FR, Ft = cache
    out = np.empty((len(surfaces), 12))
    out[:, :9] = (R[b] @ FR).reshape(-1, 9)
    out[:, 9:] = (R[b] @ Ft)[:, :, 0] + t[b]
    return out


def _surface_plan(manip: Manipulator):
    """(key, convex surface indices, the convex surfaces (a list kept for the
    pose cache), all surfaces convex) — rebuilt when the surface list changes."""
    surf = manip.surfaces
    plan = getattr(manip, "_surface_plan", None)
    if plan is None or plan[0] != (id(surf), len(surf)):
        idx = [i for i, s in enumerate(surf) if isinstance(s, ConvexGeometry)]
        plan = ((id(surf), len(surf)), idx, [surf[i] for i in idx], len(idx) == len(surf))
        manip._surface_plan = plan
    return plan


def hull_poses(manip: Manipulator, q: np.ndarray) -> np.ndarray:
    """[K,12] world poses of the convex surfaces: transform_to_root(state, frame)
    (src/Flash.jl:248) = T_world_body · T_body_geometry."""
    return _posed(manip, q, _surface_plan(manip)[2])


_IDENTITY12 = np.concatenate([np.eye(3).ravel(), np.zeros(3)])


def surface_poses(manip: Manipulator, q: np.ndarray) -> np.ndarray:
    """[S,12] one pose per surface in surface order (identity for RBF skins,
    whose centres travel separately)."""
    surf = manip.surfaces
    _, idx, convex, all_convex = _surface_plan(manip)
    posed = _posed(manip, q, convex)
    if all_convex:
        return posed
    out = np.tile(_IDENTITY12, (len(surf), 1))
    out[idx] = posed
    return out


def prepare_pass(ctx, manip: Manipulator, q_normalized: np.ndarray, deformation_data: np.ndarray):
    """Poses for every surface; uploads the RBF rows when the scene has skins.
    Returns (poses, rbf solves or [])."""
    solves = []
    if manip.has_rbf():
        from . import rbf
        solves = rbf.solve(manip, q_normalized, deformation_data)
        ctx.set_rbf_params(rbf.rows(solves))
    return surface_poses(manip, q_normalized), solves


class SceneSkin:
    """The closure returned by skin(state): x -> minimum(s(x) for s in surfaces)
    (src/Flash.jl:265-268). Accepts one point (returns a float) or an (n,3)
    batch (returns an array). `.evaluate` also returns k* and ∇d*."""

    def __init__(self, state: ManipulatorState, device: int = 0, precision: int = 64):
        self.state = state
        self.ctx = state.manipulator.engine(device, precision)
        self.q = state.manipulator.mechanism.normalize(state.q)
        self.deformation_data = state.deformation_data.copy()

    def evaluate(self, x):
        pts = np.asarray(x, np.float64).reshape(-1, 3)
        poses, _ = prepare_pass(self.ctx, self.state.manipulator, self.q, self.deformation_data)
        return self.ctx.skin(poses, pts)

    def __call__(self, x):
        x = np.asarray(x, np.float64)
        d, _, _ = self.evaluate(x)
        return float(d[0]) if x.ndim == 1 else d

    def raycast(self, origin, rays):
        """Depth along each unit world ray (src/depthsensors.jl:56-97) on the GPU."""
        poses, _ = prepare_pass(self.ctx, self.state.manipulator, self.q, self.deformation_data)
        return self.ctx.raycast(poses, origin, rays)


def surfaces(state: ManipulatorState) -> list:
    """surfaces(state) (src/Flash.jl:261-263): one posed evaluator per surface."""
    poses = hull_poses(state.manipulator, state.manipulator.mechanism.normalize(state.q))
    return [(s, Transform(p[:9].reshape(3, 3), p[9:])) for s, p in zip(state.manipulator.convex_surfaces(), poses)]


def skin(state: ManipulatorState, device: int = 0, precision: int = 64) -> SceneSkin:
    """Flash.skin(state) (src/Flash.jl:265-268)."""
    return SceneSkin(state, device, precision)
