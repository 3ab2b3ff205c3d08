"""module Flash.DepthData (src/depthdata.jl) — point-cloud ingest.

read_point_cloud(file) (:19-30): line 1 is the camera origin "x, y, z"; every
following line is "x, y, z, r, g, b" (comma separated, readdlm). Returns a
PointCloud (camera_origin, positions [n,3], colors [n,3]). As in the
reference, rows without colour columns are an error (:27 indexes columns 4-6;
box_on_table_points.txt is xyz-only and fails there too). LCMGL rendering
(:32-46) is out of scope.
"""
from __future__ import annotations

import io
import os
from dataclasses import dataclass

import numpy as np


@dataclass
class PointCloud:
    camera_origin: np.ndarray
    positions: np.ndarray  # [n,3] float64
    colors: np.ndarray     # [n,3] float64 (RGB in [0,1])

    def __repr__(self):
        o = ", ".join(repr(float(v)) for v in self.camera_origin)
        return f"PointCloud with origin: [{o}] containing {len(self.positions)} points"

    def __len__(self):
        return len(self.positions)


def read_point_cloud(file) -> PointCloud:
    """Path or text file object -> PointCloud."""
    if isinstance(file, (str, os.PathLike)):
        with open(file) as f:
            return read_point_cloud(f)
    origin_line = file.readline()
    origin = np.array([float(c) for c in origin_line.split(",")[:3]], np.float64)
    rest = file.read()
    data = np.loadtxt(io.StringIO(rest), delimiter=",", dtype=np.float64, ndmin=2) if rest.strip() else np.zeros((0, 6))
    if data.shape[1] < 6:
        raise ValueError(f"read_point_cloud: rows have {data.shape[1]} columns, expected x,y,z,r,g,b")
    return PointCloud(origin, np.ascontiguousarray(data[:, :3]), np.ascontiguousarray(data[:, 3:6]))


def subsample(points: np.ndarray, step: int = 200) -> np.ndarray:
    """msg[:points][1:200:end] (examples/irb_and_squishable.ipynb cell 12)."""
    return np.ascontiguousarray(np.asarray(points)[::step])


def kinect_to_pointcloud(x, y, z, num: int | None = None, utime: int = 0) -> dict:
    """The message conversion of convert_kinect_log_data.py:11-31 on arrays.

    A kinect.pointcloud_t (KINECT_POINTS_REDUCED) interleaves positions and
    colours in its x/y/z arrays: even indices are xyz, odd indices rgb. The
    bot_core.pointcloud_t it becomes holds n_points = num // 2 points
    (x[i], y[i], z[i]) for even i, and n_channels = 3 channels "r", "g", "b"
    whose values are x[i], y[i], z[i] for odd i. Returns that message as a dict
    (utime, n_points, points [n,3] f32, n_channels, channel_names, channels
    [3,n] f32). LCM wire encoding is out of scope: the lcmtypes are not part of
    the reference."""
    x, y, z = (np.asarray(v, np.float32) for v in (x, y, z))
    num = len(x) if num is None else int(num)
    pts = np.stack([x[0:num:2], y[0:num:2], z[0:num:2]], axis=1)
    chans = np.stack([v[1:num:2] for v in (x, y, z)])
    return {"utime": int(utime), "n_points": num // 2, "points": np.ascontiguousarray(pts), "n_channels": 3,
            "channel_names": ["r", "g", "b"], "channels": np.ascontiguousarray(chans)}


def pointcloud_positions(msg: dict, step: int = 200) -> np.ndarray:
    """[n,3] float64 positions of a bot_core.pointcloud_t dict, subsampled as
    msg[:points][1:200:end] (examples/irb_and_squishable.ipynb cell 12)."""
    return subsample(np.asarray(msg["points"], np.float64), step)
