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
        self._version = getattr(self, "_version", 0) + 1
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
        self._version = getattr(self, "_version", 0) + 1
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
        P = self._kinematic_plan()
        for o in P["quat_qoff"]:
            q[o:o + 4] = q[o:o + 4] / np.linalg.norm(q[o:o + 4])
        return q

    # -- kinematics -----------------------------------------------------------
    def _kinematic_plan(self):
        """Arrays of the tree grouped by depth, rebuilt when the tree changes:
        every level's bodies are posed with one batch of stacked 3x3 products
        (a Python loop over bodies cost ~20 us per body — 1.3 ms for M64's 64
        bodies, 6x the GPU pass it feeds)."""
        key = (self.num_bodies, getattr(self, "_version", 0))
        plan = getattr(self, "_plan", None)
        if plan is not None and plan["key"] == key:
            return plan
        nb = self.num_bodies
        depth = np.zeros(nb, np.int64)
        for b in range(1, nb):
            depth[b] = depth[self.edges[b].parent] + 1
        E = [None] + self.edges[1:]
        parent = np.array([0] + [e.parent for e in self.edges[1:]], np.int64)
        AR = np.stack([np.eye(3)] + [e.joint_to_parent.R for e in E[1:]])
        At = np.stack([np.zeros(3)] + [e.joint_to_parent.t for e in E[1:]])[:, :, None]
        BR = np.stack([np.eye(3)] + [e.body_to_joint.R for e in E[1:]])
        Bt = np.stack([np.zeros(3)] + [e.body_to_joint.t for e in E[1:]])[:, :, None]
        kind = np.array([-1] + [{"fixed": 0, "revolute": 1, "quaternion_floating": 2}[e.joint.kind] for e in E[1:]])
        axis = np.stack([np.zeros(3)] + [e.joint.axis / np.linalg.norm(e.joint.axis) for e in E[1:]])
        qoff = np.array([0] + [e.q_offset for e in E[1:]], np.int64)
        levels = [np.nonzero(depth == d)[0] for d in range(1, int(depth.max()) + 1)] if nb > 1 else []
        rev = np.nonzero(kind == 1)[0]
        a = axis[rev]
        Kax = np.zeros((len(rev), 3, 3))
        Kax[:, 0, 1], Kax[:, 0, 2] = -a[:, 2], a[:, 1]
        Kax[:, 1, 0], Kax[:, 1, 2] = a[:, 2], -a[:, 0]
        Kax[:, 2, 0], Kax[:, 2, 1] = -a[:, 1], a[:, 0]
        quat = np.nonzero(kind == 2)[0]
        plan = dict(key=key, parent=parent, AR=AR, At=At, BR=BR, Bt=Bt, kind=kind, axis=axis, qoff=qoff,
                    levels=levels, rev=rev, Kax=Kax, KK=Kax @ Kax, quat=quat,
                    quat_qoff=[int(qoff[i]) for i in quat])
        # contiguous copies for the native fsdf_tree_transforms (kept alive by the plan)
        c = lambda a, dt=np.float64: np.ascontiguousarray(a, dt)  # noqa: E731
        nat = (c(parent, np.int32), c(np.maximum(kind, 0), np.int32), c(qoff, np.int32), c(axis),
               c(AR.reshape(nb, 9)), c(At.reshape(nb, 3)), c(BR.reshape(nb, 9)), c(Bt.reshape(nb, 3)))
        plan["native"] = nat
        plan["native_ptrs"] = [a.ctypes.data for a in nat]
        self._plan = plan
        return plan

    def body_transform_arrays(self, q: np.ndarray):
        """transform_to_root of every body frame as arrays: R [nb,3,3], t [nb,3],
        plus the joint frames before the joint motion (T_parent · joint_to_parent),
        Rb [nb,3,3], tb [nb,3] (the chain rule's motion subspaces live there).
        Computed natively (fsdf_tree_transforms, csrc/kinematics.cpp: one loop over
        the bodies, ~20x faster than the numpy levels below for M64)."""
        P = self._kinematic_plan()
        q = np.ascontiguousarray(q, np.float64)
        last = getattr(self, "_fk_last", None)  # the pass and its chain rule share one q
        if last is not None and last[0] is P and np.array_equal(last[1], q):
            return last[2]
        from . import _lib
        nb = self.num_bodies
        R = np.empty((nb, 3, 3))
        t = np.empty((nb, 3))
        Rb = np.empty((nb, 3, 3))
        tb = np.empty((nb, 3))
        st = _lib.load().fsdf_tree_transforms(nb, *P["native_ptrs"], q.ctypes.data, R.ctypes.data, t.ctypes.data,
                                              Rb.ctypes.data, tb.ctypes.data)
        if st != _lib.FSDF_OK:
            raise _lib.FlashNativeError(st, "fsdf_tree_transforms: bad tree or configuration")
        out = (R, t, Rb, tb)
        for a in out:
            a.flags.writeable = False
        self._fk_last = (P, q.copy(), out, (Rb.ctypes.data, tb.ctypes.data))
        return out

    def body_transform_arrays_numpy(self, q: np.ndarray):
        """The same transforms in numpy (test reference for the native path):
        every body's local transform joint_to_parent · joint(q) · body_to_joint is
        formed in one batch, then composed down the tree one depth level at a time."""
        P = self._kinematic_plan()
        q = np.asarray(q, np.float64)
        nb = self.num_bodies
        JR = np.broadcast_to(np.eye(3), (nb, 3, 3)).copy()
        Jt = np.zeros((nb, 3, 1))
        rev = P["rev"]
        if len(rev):
            a = P["axis"][rev]
            ang = q[P["qoff"][rev]]
            K = P["Kax"]
            JR[rev] = np.eye(3) + np.sin(ang)[:, None, None] * K + (1 - np.cos(ang))[:, None, None] * P["KK"]
        for i in P["quat"]:
            o = P["qoff"][i]
            qq = q[o:o + 7]
            JR[i] = quat_to_matrix(qq[:4] / np.linalg.norm(qq[:4]))
            Jt[i, :, 0] = qq[4:7]
        AJ = P["AR"] @ JR
        LR = AJ @ P["BR"]
        Lt = AJ @ P["Bt"] + (P["AR"] @ Jt + P["At"])
        R = np.empty((nb, 3, 3))
        t = np.empty((nb, 3, 1))
        R[0] = np.eye(3)
        t[0] = 0.0
        for lv in P["levels"]:
            pr = P["parent"][lv]
            R[lv] = R[pr] @ LR[lv]
            t[lv] = R[pr] @ Lt[lv] + t[pr]
        pr = P["parent"]
        Rb = R[pr] @ P["AR"]
        tb = R[pr] @ P["At"] + t[pr]
        Rb[0] = np.eye(3)
        tb[0] = 0.0
        return R, t[:, :, 0], Rb, tb[:, :, 0]

    def body_transforms(self, q: np.ndarray) -> list[Transform]:
        """transform_to_root of every body frame."""
        R, t, _, _ = self.body_transform_arrays(q)
        return [Transform(R[b], t[b]) for b in range(self.num_bodies)]

    def config_gradient(self, q: np.ndarray, body_wrench: np.ndarray | None = None, surface_body=None,
                        surface_wrench=None) -> np.ndarray:
        """∂c/∂q from wrenches (F, M about the world origin): per body
        (body_wrench [nb, 6]) and/or per surface (surface_wrench [S, 6] on body
        surface_body[k], -1 = none) — natively (fsdf_config_gradient,
        csrc/kinematics.cpp; config_gradient_numpy is the test reference).

        For a world twist (ω, v) of a body, δc = −(ω·M + v·F) (include/flashsdf.h).
        Quaternion blocks include the normalization projection (I − q̂q̂ᵀ)/|q| that
        ForwardDiff sees through normalize! (src/gradientdescent.jl:30)."""
        from . import _lib
        P = self._kinematic_plan()
        q = np.ascontiguousarray(q, np.float64)
        self.body_transform_arrays(q)
        rb_ptr, tb_ptr = self._fk_last[3]
        nb = self.num_bodies
        bw = None if body_wrench is None else np.ascontiguousarray(body_wrench, np.float64).reshape(nb, 6)
        ns = 0 if surface_body is None else len(surface_body)
        sb = None if ns == 0 else np.ascontiguousarray(surface_body, np.int32)
        sw = None if ns == 0 else np.ascontiguousarray(surface_wrench, np.float64).reshape(ns, 6)
        if "cg_work" not in P:
            P["cg_work"] = np.empty(6 * nb)
            P["cg_work_ptr"] = P["cg_work"].ctypes.data
        g = np.zeros(self._nq)
        nat = P["native_ptrs"]
        ptr = lambda a: None if a is None else a.ctypes.data  # noqa: E731
        st = _lib.load().fsdf_config_gradient(nb, nat[0], nat[1], nat[2], nat[3], rb_ptr, tb_ptr, q.ctypes.data, ns,
                                              ptr(sb), ptr(sw), ptr(bw), P["cg_work_ptr"], g.ctypes.data)
        if st != _lib.FSDF_OK:
            raise _lib.FlashNativeError(st, "fsdf_config_gradient: bad tree, configuration or surface bodies")
        return g

    def config_gradient_numpy(self, q: np.ndarray, body_wrench: np.ndarray) -> np.ndarray:
        """The chain rule of config_gradient in numpy (test reference)."""
        nb = self.num_bodies
        P = self._kinematic_plan()
        sub = np.array(body_wrench, np.float64, copy=True).reshape(nb, 6)
        for lv in reversed(P["levels"]):  # children (deeper levels) into parents
            np.add.at(sub, P["parent"][lv], sub[lv])
        _, _, Rb, tb = self.body_transform_arrays(q)
        g = np.zeros(self._nq)
        rev = np.nonzero(P["kind"] == 1)[0]
        if len(rev):
            w = np.einsum("nij,nj->ni", Rb[rev], P["axis"][rev])
            v = np.cross(tb[rev], w)
            F, M = sub[rev, :3], sub[rev, 3:]
            g[P["qoff"][rev]] = -(np.einsum("ni,ni->n", w, M) + np.einsum("ni,ni->n", v, F))
        for b in np.nonzero(P["kind"] == 2)[0]:
            e = self.edges[b]
            F, M = sub[b, :3], sub[b, 3:]
            qq = q[e.q_offset:e.q_offset + 7]
            nrm = np.linalg.norm(qq[:4])
            qh = qq[:4] / nrm
            W, X, Y, Z = qh
            E = np.array([[-X, W, -Z, Y], [-Y, Z, W, -X], [-Z, -Y, X, W]])
            o = Rb[b] @ qq[4:7] + tb[b]  # world origin of frameAfter
            for j in range(4):
                w = Rb[b] @ (2.0 * E[:, j])
                v = np.cross(o, w)
                g[e.q_offset + j] = -(w @ M + v @ F) / nrm
            for j in range(3):
                v = Rb[b][:, j]
                g[e.q_offset + 4 + j] = -(v @ F)
        return g
