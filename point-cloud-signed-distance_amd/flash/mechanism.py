"""Kinematic tree, forward kinematics and the DOF chain rule (host side).

Restates the subset of RigidBodyDynamics.jl 0.0.2 the hot path touches
(un-vendored, REQUIRE.dev:18):
  * Mechanism(world) / attach!(mech, parent, joint, joint_to_parent, body,
    body_to_joint)                 src/models.jl:25-39,76-83,103-110
  * joint types Revolute(axis), QuaternionFloating, Fixed
  * q layout: joints in attach order; QuaternionFloating q = [w x y z tx ty tz]
    (SURVEY.md Appendix A); default configuration = identity quaternion
  * transform_to_root(state, frame)  src/Flash.jl:147,248
  * normalize!(state) of quaternion blocks   src/gradientdescent.jl:19-26
The reference gets ∂cost/∂q from ForwardDiff (⌈n/9⌉ chunk passes over every
point). Here it is analytic: the residual pass returns, per hull, the wrench
(F, M) = (Σ 2d∇d, Σ 2d p×∇d) and `config_gradient` contracts the subtree
wrenches with each joint's world motion subspace: ∂c/∂q_i = −(ω_i·M + v_i·F).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .geometry import Transform, angle_axis, quat_to_matrix


@dataclass
class Joint:
    name: str
    kind: str  # "fixed" | "revolute" | "quaternion_floating"
    axis: np.ndarray = field(default_factory=lambda: np.array([0.0, 0.0, 1.0]))
    lower: float = -np.inf
    upper: float = np.inf

    @property
    def nq(self) -> int:
        return {"fixed": 0, "revolute": 1, "quaternion_floating": 7}[self.kind]

    def transform(self, q: np.ndarray) -> Transform:
        """frameAfter -> frameBefore."""
        if self.kind == "fixed":
            return Transform.identity()
        if self.kind == "revolute":
            return Transform(angle_axis(q[0], self.axis), np.zeros(3))
        quat = q[:4] / np.linalg.norm(q[:4])
        return Transform(quat_to_matrix(quat), np.asarray(q[4:7], np.float64).copy())


def Revolute(axis, name="joint", lower=-np.inf, upper=np.inf) -> Joint:
    a = np.asarray(axis, np.float64)
    return Joint(name, "revolute", a / np.linalg.norm(a), lower, upper)


def QuaternionFloating(name="floating") -> Joint:
    return Joint(name, "quaternion_floating")


def Fixed(name="fixed") -> Joint:
    return Joint(name, "fixed")


@dataclass
class _Edge:
    joint: Joint
    parent: int
    joint_to_parent: Transform
    body_to_joint: Transform
    q_offset: int = 0


class Mechanism:
    """Rooted tree of bodies; body 0 is the world."""

    def __init__(self, root_name: str = "world"):
        self.body_names = [root_name]
        self.edges: list[_Edge | None] = [None]
        self._nq = 0

    # -- construction -------------------------------------------------------
    def body_index(self, name: str) -> int:
        return self.body_names.index(name)

    def attach(self, parent: str | int, joint: Joint, joint_to_parent: Transform | None, body_name: str,
               body_to_joint: Transform | None = None) -> int:
        p = parent if isinstance(parent, int) else self.body_index(parent)
        if body_name in self.body_names:
            raise ValueError(f"body {body_name!r} already in mechanism")
        e = _Edge(joint, p, joint_to_parent or Transform.identity(), body_to_joint or Transform.identity(), self._nq)
        self._nq += joint.nq
        self.body_names.append(body_name)
        self.edges.append(e)
        return len(self.body_names) - 1

    def attach_mechanism(self, other: "Mechanism", parent: int = 0) -> dict[int, int]:
        """Graft `other` (its world becomes `parent`); returns body index map.
        Mirrors RigidBodyDynamics.attach!(mech, root, mech2) (src/models.jl:174)."""
        remap = {0: parent}
        for b in range(1, other.num_bodies):
            e = other.edges[b]
            remap[b] = self.attach(remap[e.parent], e.joint, e.joint_to_parent, other.body_names[b], e.body_to_joint)
        return remap

    def change_joint_type(self, body: str | int, joint: Joint):
        """change_joint_type! (examples/irb_and_squishable.ipynb cell 4); re-lays out q."""
        b = body if isinstance(body, int) else self.body_index(body)
        self.edges[b].joint = joint
        off = 0
        for e in self.edges[1:]:
            e.q_offset = off
            off += e.joint.nq
        self._nq = off

    # -- queries --------------------------------------------------------------
    @property
    def num_bodies(self) -> int:
        return len(self.body_names)

    @property
    def num_positions(self) -> int:
        return self._nq

    def joints(self):
        return [e.joint for e in self.edges[1:]]

    def q_range(self, body: int) -> slice:
        e = self.edges[body]
        return slice(e.q_offset, e.q_offset + e.joint.nq)

    def zero_configuration(self) -> np.ndarray:
        q = np.zeros(self._nq)
        for e in self.edges[1:]:
            if e.joint.kind == "quaternion_floating":
                q[e.q_offset] = 1.0
        return q

    def normalize(self, q: np.ndarray) -> np.ndarray:
        """normalize! of every QuaternionFloating block (src/gradientdescent.jl:19-26)."""
        q = np.array(q, np.float64, copy=True)
        for e in self.edges[1:]:
            if e.joint.kind == "quaternion_floating":
                s = slice(e.q_offset, e.q_offset + 4)
                q[s] = q[s] / np.linalg.norm(q[s])
        return q

    # -- kinematics -----------------------------------------------------------
    def body_transforms(self, q: np.ndarray) -> list[Transform]:
        """transform_to_root of every body frame."""
        T = [Transform.identity()] * self.num_bodies
        for b in range(1, self.num_bodies):
            e = self.edges[b]
            qj = q[e.q_offset:e.q_offset + e.joint.nq]
            T[b] = T[e.parent] @ e.joint_to_parent @ e.joint.transform(qj) @ e.body_to_joint
        return T

    def config_gradient(self, q: np.ndarray, body_wrench: np.ndarray) -> np.ndarray:
        """∂c/∂q from per-body wrenches body_wrench[b] = (F, M about the world origin).

        For a world twist (ω, v) of a body, δc = −(ω·M + v·F) (include/flashsdf.h).
        Quaternion blocks include the normalization projection (I − q̂q̂ᵀ)/|q| that
        ForwardDiff sees through normalize! (src/gradientdescent.jl:30)."""
        nb = self.num_bodies
        sub = np.array(body_wrench, np.float64, copy=True).reshape(nb, 6)
        for b in range(nb - 1, 0, -1):  # children appear after parents
            sub[self.edges[b].parent] += sub[b]
        T = self.body_transforms(q)
        g = np.zeros(self._nq)
        for b in range(1, nb):
            e = self.edges[b]
            if e.joint.nq == 0:
                continue
            F, M = sub[b, :3], sub[b, 3:]
            before = T[e.parent] @ e.joint_to_parent
            if e.joint.kind == "revolute":
                w = before.R @ e.joint.axis
                o = before.t
                v = np.cross(o, w)
                g[e.q_offset] = -(w @ M + v @ F)
            else:
                qq = q[e.q_offset:e.q_offset + 7]
                nrm = np.linalg.norm(qq[:4])
                qh = qq[:4] / nrm
                W, X, Y, Z = qh
                E = np.array([[-X, W, -Z, Y], [-Y, Z, W, -X], [-Z, -Y, X, W]])
                o = before.R @ qq[4:7] + before.t  # world origin of frameAfter
                for j in range(4):
                    w = before.R @ (2.0 * E[:, j])
                    v = np.cross(o, w)
                    g[e.q_offset + j] = -(w @ M + v @ F) / nrm
                for j in range(3):
                    v = before.R[:, j]
                    g[e.q_offset + 4 + j] = -(v @ F)
        return g
