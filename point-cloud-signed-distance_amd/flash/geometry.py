"""Rigid transforms, mesh ingest and convex hulls (host side).

Restates the pieces of CoordinateTransformations / Rotations / MeshIO /
EnhancedGJK.NeighborMesh that the reference's hot path consumes:
  * URDF rpy -> rotation  (R = Rz(yaw) Ry(pitch) Rx(roll), RigidBodyDynamics'
    parse_urdf convention used by src/models.jl:167);
  * binary STL -> float64 vertex set (MeshIO 0.0.6, src/models.jl:152,168);
  * conv(vertices) planes via the native hull builder (fsdf_convex_hull).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np

from . import _lib


@dataclass
class Transform:
    """x_out = R x_in + t (a Transform3D from frame_in to frame_out)."""
    R: np.ndarray
    t: np.ndarray

    @staticmethod
    def identity() -> "Transform":
        return Transform(np.eye(3), np.zeros(3))

    @staticmethod
    def from_xyz_rpy(xyz, rpy) -> "Transform":
        return Transform(rpy_to_matrix(*rpy), np.asarray(xyz, np.float64).copy())

    def __matmul__(self, other: "Transform") -> "Transform":
        return Transform(self.R @ other.R, self.R @ other.t + self.t)

    def apply(self, x: np.ndarray) -> np.ndarray:
        return x @ self.R.T + self.t

    def inverse(self) -> "Transform":
        return Transform(self.R.T, -(self.R.T @ self.t))

    def as_pose12(self) -> np.ndarray:
        return np.concatenate([self.R.reshape(9), self.t])


def rot_x(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]], np.float64)


def rot_y(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]], np.float64)


def rot_z(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]], np.float64)


def rpy_to_matrix(roll, pitch, yaw) -> np.ndarray:
    return rot_z(yaw) @ rot_y(pitch) @ rot_x(roll)


def angle_axis(angle: float, axis) -> np.ndarray:
    """Rodrigues rotation (Rotations.AngleAxis / RBD Revolute joint transform)."""
    a = np.asarray(axis, np.float64)
    a = a / np.linalg.norm(a)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(angle) * K + (1 - np.cos(angle)) * (K @ K)


def quat_to_matrix(q) -> np.ndarray:
    """Rotation of a unit quaternion [w, x, y, z] (x_parent = R x_child)."""
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ], np.float64)


def read_stl_vertices(path: str) -> np.ndarray:
    """Unique vertices of a binary (or ASCII) STL as float64, first-occurrence order."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) >= 84:
        ntri = struct.unpack("<I", data[80:84])[0]
        if 84 + 50 * ntri == len(data):
            rec = np.frombuffer(data[84:], dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
            v = rec["v"].reshape(-1, 3).astype(np.float64)
            return unique_rows(v)
    verts = []
    for line in data.decode(errors="replace").splitlines():
        parts = line.strip().split()
        if len(parts) == 4 and parts[0] == "vertex":
            verts.append([float(p) for p in parts[1:]])
    if not verts:
        raise ValueError(f"{path}: not an STL file")
    return unique_rows(np.asarray(verts, np.float64))


def unique_rows(v: np.ndarray) -> np.ndarray:
    _, idx = np.unique(v, axis=0, return_index=True)
    return v[np.sort(idx)]


@dataclass
class ConvexHull:
    """conv(vertices) as outward CCW triangles with unit planes (n, d): n·x <= d inside."""
    vertices: np.ndarray
    faces: np.ndarray
    planes: np.ndarray

    @staticmethod
    def from_points(points) -> "ConvexHull":
        v, f, p = _lib.convex_hull(np.asarray(points, np.float64))
        return ConvexHull(v, f, p)

    def transformed(self, T: Transform) -> "ConvexHull":
        """The same hull expressed in another frame (rebuilt from moved vertices)."""
        return ConvexHull.from_points(T.apply(self.vertices))

    @property
    def centroid(self) -> np.ndarray:
        return self.vertices.mean(axis=0)
