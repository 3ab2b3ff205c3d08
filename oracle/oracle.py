"""Python face of the CPU oracle (liboracle.so) — TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
as the checker / timed CPU baseline; never by the product package `flash`.

Contents
  * OracleModel.from_manipulator: the concatenated local model (same layout the
    C-ABI builds in fsdf_set_model), from a flash.Manipulator's convex surfaces.
  * pose / skin / cost_accum: ctypes calls into flash_oracle.c (the bit-exact
    restatement of src/Flash.jl:233-268 + src/gradientdescent.jl:28-39).
  * numpy_hull_sdf: an INDEPENDENT formulation of the polytope SDF (vertex /
    edge / face-interior candidates, no shared code or operation order), used to
    pin the C restatement at 1e-12.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_int32, c_int64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
FX = 24

_lib = None


def build():
    import subprocess
    subprocess.run(["make", "-C", HERE], check=True, stdout=subprocess.DEVNULL)


class Posed(ctypes.Structure):
    _fields_ = [("K", c_int32), ("face_off", c_void_p), ("vert_off", c_void_p), ("nbr", c_void_p),
                ("planes_w", c_void_p), ("facex_w", c_void_p), ("verts_w", c_void_p), ("hscale", c_void_p),
                ("S", c_int32), ("surf_index", c_void_p), ("rbf_row_off", c_void_p), ("rbf_acc_off", c_void_p),
                ("rbf_rows", c_void_p), ("faces", c_void_p)]


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        lib.oracle_pose_model.argtypes = [c_int32, c_int32, c_int32] + [c_void_p] * 11
        lib.oracle_hull_sdf.argtypes = [ctypes.POINTER(Posed), c_int32, c_void_p, c_void_p, c_void_p]
        lib.oracle_skin.argtypes = [ctypes.POINTER(Posed), c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int32]
        lib.oracle_skin_culled.argtypes = [ctypes.POINTER(Posed), c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                           c_int32]
        lib.oracle_skin_culled.restype = c_int32
        lib.oracle_cost_accum.argtypes = [ctypes.POINTER(Posed), c_void_p, c_int64, c_void_p]
        lib.oracle_rbf_skin.argtypes = [c_void_p, c_int32, c_void_p, c_void_p, c_void_p]
        lib.oracle_raycast.argtypes = [ctypes.POINTER(Posed), c_void_p, c_void_p, c_int64, c_void_p, c_int32]
        lib.oracle_max_threads.restype = c_int32
        # fp32 instantiation (skin_impl.h with R = float): fp32 contexts bit for bit
        lib.oracle_pose_model_f32.argtypes = [c_int32, c_int32, c_int32] + [c_void_p] * 11
        lib.oracle_hull_sdf_f32.argtypes = [ctypes.POINTER(Posed), c_int32, c_void_p, c_void_p, c_void_p]
        lib.oracle_skin_f32.argtypes = [ctypes.POINTER(Posed), c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                        c_int32]
        lib.oracle_rbf_skin_f32.argtypes = [c_void_p, c_int32, c_void_p, c_void_p, c_void_p]
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else c_void_p(a.ctypes.data)


def face_neighbours(faces, fbase):
    """Face across edge i (v_i -> v_{i+1}) of every face (global ids), like fsdf_set_model."""
    owner = {}
    for f, (a, b, c) in enumerate(faces):
        for e, (u, v) in enumerate(((a, b), (b, c), (c, a))):
            owner[(int(u), int(v))] = f
    nb = np.empty((len(faces), 3), np.int32)
    for f, (a, b, c) in enumerate(faces):
        for e, (u, v) in enumerate(((a, b), (b, c), (c, a))):
            nb[f, e] = fbase + owner.get((int(v), int(u)), f)
    return nb


class OracleModel:
    def __init__(self, hulls, surfaces=None):
        """hulls: list of (vertices, faces, planes) in local frames; surfaces:
        optional scene order [("hull", h) | ("rbf", n_centres)] (default: hulls only)."""
        if surfaces is None:
            surfaces = [("hull", i) for i in range(len(hulls))]
        V, Fc, P, FH, VH, NB, off, voff = [], [], [], [], [], [], [0], [0]
        vbase = 0
        for k, (v, f, p) in enumerate(hulls):
            V.append(np.asarray(v, np.float64))
            Fc.append(np.asarray(f, np.int32) + vbase)
            P.append(np.asarray(p, np.float64))
            FH.append(np.full(len(f), k, np.int32))
            VH.append(np.full(len(v), k, np.int32))
            NB.append(face_neighbours(np.asarray(f), off[-1]))
            off.append(off[-1] + len(f))
            voff.append(voff[-1] + len(v))
            vbase += len(v)
        self.K = len(hulls)
        cat = lambda xs, dt: np.ascontiguousarray(np.concatenate(xs) if xs else np.zeros((0,), dt))  # noqa: E731
        self.verts_l = cat(V, np.float64).reshape(-1, 3)
        self.faces = cat(Fc, np.int32).reshape(-1, 3)
        self.planes_l = cat(P, np.float64).reshape(-1, 4)
        self.face_hull = cat(FH, np.int32)
        self.vert_hull = cat(VH, np.int32)
        self.nbr = cat(NB, np.int32).reshape(-1, 3)
        self.face_off = np.asarray(off, np.int32)
        self.vert_off = np.asarray(voff, np.int32)
        self.F = len(self.face_hull)
        self.V = len(self.vert_hull)
        self.hulls = hulls
        # surface table
        self.S = len(surfaces)
        si, rows, acc, hk, self.hull_surface = [], [0], [0], 0, []
        for k, (kind, spec) in enumerate(surfaces):
            if kind == "hull":
                si.append(hk)
                self.hull_surface.append(k)
                hk += 1
            else:
                si.append(-(len(rows) - 1) - 1)
                rows.append(rows[-1] + int(spec) + 1)
                acc.append(acc[-1] + 4 * int(spec) + 4)
        self.surf_index = np.asarray(si, np.int32)
        self.rbf_row_off = np.asarray(rows, np.int32)
        self.rbf_acc_off = np.asarray(acc, np.int32)
        self.accum_len = 1 + 6 * self.S + int(self.rbf_acc_off[-1])

    @staticmethod
    def from_manipulator(manip):
        from flash.core import ConvexGeometry
        hulls, surfaces = [], []
        for s in manip.surfaces:
            if isinstance(s, ConvexGeometry):
                surfaces.append(("hull", len(hulls)))
                hulls.append((s.hull.vertices, s.hull.faces, s.hull.planes))
            else:
                surfaces.append(("rbf", len(s.surface_points) + len(s.skeleton_points)))
        return OracleModel(hulls, surfaces)

    def pose(self, poses, rbf_rows=None, precision: int = 64):
        """World-frame model arrays for `poses` ([S,12], one per surface).
        precision=32: the rows an fp32 context works on (computed in fp64 from
        the fp64 poses, rounded once to fp32, edge records formed in fp32)."""
        if precision not in (32, 64):
            raise ValueError("precision is 32 or 64")
        rt = np.float64 if precision == 64 else np.float32
        poses = np.ascontiguousarray(poses, np.float64).reshape(self.S, 12)
        hp = np.ascontiguousarray(poses[self.hull_surface]) if self.K else np.zeros((1, 12))
        pw = np.empty((max(self.F, 1), 4), rt)
        fx = np.empty((max(self.F, 1), FX), rt)
        vw = np.empty((max(self.V, 1), 4), rt)
        hs = np.empty(max(self.K, 1), rt)
        fn = load().oracle_pose_model if precision == 64 else load().oracle_pose_model_f32
        fn(self.F, self.V, self.K, _p(self.verts_l), _p(self.faces), _p(self.planes_l),
           _p(self.face_hull), _p(self.vert_hull), _p(self.vert_off), _p(hp), _p(pw),
           _p(fx), _p(vw), _p(hs))
        rr = np.ascontiguousarray(rbf_rows if rbf_rows is not None else np.zeros((1, 4)), rt)
        arrays = (pw, fx, vw, hs, rr)
        st = Posed(self.K, self.face_off.ctypes.data, self.vert_off.ctypes.data, self.nbr.ctypes.data,
                   pw.ctypes.data, fx.ctypes.data, vw.ctypes.data, hs.ctypes.data, self.S,
                   self.surf_index.ctypes.data, self.rbf_row_off.ctypes.data, self.rbf_acc_off.ctypes.data,
                   rr.ctypes.data, self.faces.ctypes.data)
        return st, arrays

    def skin(self, poses, pts, threads: int = 0, rbf_rows=None, culled: bool = False, precision: int = 64):
        """Per-point (d*, k*, ∇d*). culled=True visits the hulls by a bounding-sphere
        lower bound and stops early (same results bit for bit; the CPU baseline's
        culled leg). precision=32 restates an fp32 context (points and RBF rows
        rounded to fp32 as fsdf_set_points / fsdf_set_rbf_params do; results
        returned as float64 holding fp32 values, like the C-ABI's outputs)."""
        if precision == 32:
            if culled:
                raise ValueError("the culled leg is fp64 only")
            p32 = np.ascontiguousarray(np.asarray(pts, np.float64).reshape(-1, 3).astype(np.float32))
            st, _keep = self.pose(poses, rbf_rows, precision=32)
            n = len(p32)
            d = np.empty(n, np.float32)
            k = np.empty(n, np.int32)
            g = np.empty((n, 3), np.float32)
            load().oracle_skin_f32(ctypes.byref(st), _p(p32), n, _p(d), _p(k), _p(g), threads)
            return d.astype(np.float64), k, g.astype(np.float64)
        pts = np.ascontiguousarray(pts, np.float64).reshape(-1, 3)
        st, _keep = self.pose(poses, rbf_rows)
        n = len(pts)
        d = np.empty(n)
        k = np.empty(n, np.int32)
        g = np.empty((n, 3))
        if culled:
            if load().oracle_skin_culled(ctypes.byref(st), _p(pts), n, _p(d), _p(k), _p(g), threads) != 0:
                raise ValueError("oracle_skin_culled: more than 1024 surfaces")
        else:
            load().oracle_skin(ctypes.byref(st), _p(pts), n, _p(d), _p(k), _p(g), threads)
        return d, k, g

    def cost_accum(self, poses, pts, rbf_rows=None):
        pts = np.ascontiguousarray(pts, np.float64).reshape(-1, 3)
        st, _keep = self.pose(poses, rbf_rows)
        acc = np.empty(self.accum_len)
        load().oracle_cost_accum(ctypes.byref(st), _p(pts), len(pts), _p(acc))
        return acc

    def raycast(self, poses, origin, rays, threads: int = 0, rbf_rows=None):
        """doRaycast per ray (src/depthsensors.jl:56-81) -> depth [n] (NaN = miss)."""
        st, _keep = self.pose(poses, rbf_rows)
        o = np.ascontiguousarray(origin, np.float64).reshape(3)
        r = np.ascontiguousarray(rays, np.float64).reshape(-1, 3)
        depth = np.empty(len(r))
        load().oracle_raycast(ctypes.byref(st), _p(o), _p(r), len(r), _p(depth), threads)
        return depth

    def world_hull(self, poses, k):
        """(world vertices, faces, world planes) of hull k, plain numpy."""
        P = np.asarray(poses, np.float64).reshape(self.K, 12)[k]
        R, t = P[:9].reshape(3, 3), P[9:]
        v, f, p = self.hulls[k]
        n = p[:, :3] @ R.T
        return v @ R.T + t, f, np.concatenate([n, (p[:, 3] + n @ t)[:, None]], axis=1)


def max_threads() -> int:
    return int(load().oracle_max_threads())


# ---------------------------------------------------------------------------
# Independent numpy formulation (no shared code with flash_oracle.c)
# ---------------------------------------------------------------------------
def _seg_dist2(p, a, b):
    ab = b - a
    t = np.clip(((p[:, None, :] - a[None]) * ab[None]).sum(-1) / (ab * ab).sum(-1)[None], 0.0, 1.0)
    q = a[None] + t[..., None] * ab[None]
    return ((p[:, None, :] - q) ** 2).sum(-1)


def numpy_hull_sdf(verts, faces, planes, pts):
    """Signed distance to conv(verts): inside max plane value; outside the min
    over {vertices, edges, face interiors whose projection falls inside}."""
    pts = np.asarray(pts, np.float64).reshape(-1, 3)
    h = pts @ planes[:, :3].T - planes[:, 3][None]
    hmax = h.max(1)
    out = hmax > 0
    d = hmax.copy()
    if out.any():
        p = pts[out]
        best = ((p[:, None, :] - verts[None]) ** 2).sum(-1).min(1)
        edges = np.concatenate([faces[:, [0, 1]], faces[:, [1, 2]], faces[:, [2, 0]]])
        edges = np.unique(np.sort(edges, 1), axis=0)
        best = np.minimum(best, _seg_dist2(p, verts[edges[:, 0]], verts[edges[:, 1]]).min(1))
        a, b, c = verts[faces[:, 0]], verts[faces[:, 1]], verts[faces[:, 2]]
        n = planes[:, :3]
        hp = h[out]
        proj = p[:, None, :] - hp[..., None] * n[None]
        def side(u, v):
            return (np.cross(v - u, proj - u[None]) * n[None]).sum(-1) >= -1e-15
        inside_face = side(a, b) & side(b, c) & side(c, a) & (hp > 0)
        face_d2 = np.where(inside_face, hp ** 2, np.inf).min(1)
        best = np.minimum(best, face_d2)
        d[out] = np.sqrt(best)
    return d


def numpy_scene_sdf(om, poses, pts, chunk=4096):
    """Independent scene minimum over the hulls (numpy_hull_sdf per hull), with
    its own exact-safe pruning so that large samples stay cheap: c_k = vertex
    centroid (inside conv(V_k), so d_k(p) <= |p − c_k|), r_k = max vertex
    distance (d_k(p) >= |p − c_k| − r_k); hull k is evaluated for p only if
    |p − c_k| − r_k <= min_j |p − c_j| + margin. Returns (d*, per-point minimum
    set as a boolean matrix [n, K] of hulls within 1e-12 of d*)."""
    pts = np.asarray(pts, np.float64).reshape(-1, 3)
    world = [om.world_hull(poses, k) for k in range(om.K)]
    cen = np.stack([v.mean(0) for v, _, _ in world])
    rad = np.array([np.sqrt(((v - c) ** 2).sum(1).max()) for (v, _, _), c in zip(world, cen)])
    n = len(pts)
    per = np.full((n, om.K), np.inf)
    for s in range(0, n, chunk):
        p = pts[s:s + chunk]
        dc = np.sqrt(((p[:, None, :] - cen[None]) ** 2).sum(-1))
        ub = dc.min(1)
        cand = dc - rad[None] <= ub[:, None] + 1e-9 * (1 + np.abs(p).sum(1))[:, None]
        for k in range(om.K):
            idx = np.nonzero(cand[:, k])[0]
            if len(idx):
                per[s + idx, k] = numpy_hull_sdf(*world[k], p[idx])
    d = per.min(1)
    return d, per <= d[:, None] + 1e-12
