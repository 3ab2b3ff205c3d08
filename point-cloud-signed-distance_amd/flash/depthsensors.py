"""module Flash.DepthSensors (src/depthsensors.jl) — synthetic depth on the GPU.

  generateKinectRays(rows, cols, vfov, hfov)   :10-30  (camera-frame unit rays)
  Kinect(rows, cols, vfov, hfov)               :54
  rays_in_world(sensor, tform)                 :83-86
  raycast_depths(surface, sensor, tform)       :88-97  (doRaycast per ray, :56-81)
  raycast_points(surface, sensor, tform)       :99-113 (row-major, NaN rays dropped)
  raycast(state, sensor, tform)                :115-118
The per-ray secant march runs in raycast_kernel (fsdf_raycast), one lane per
ray, on the same scene SDF as the residual pass. LCMGL drawing (:36-52,
:120-135) is out of scope.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .core import ManipulatorState, SceneSkin, skin
from .geometry import Transform


def generate_kinect_rays(rows: int, cols: int, vertical_fov: float = 0.4682, horizontal_fov: float = 0.5449):
    """[rows, cols, 3] unit rays. As in the reference, x uses tan(vertical_fov)/cx
    and y tan(horizontal_fov)/cy (the names are swapped there; kept)."""
    cx, cy = (cols + 1) / 2.0, (rows + 1) / 2.0
    tv, th = np.tan(vertical_fov), np.tan(horizontal_fov)
    v, u = np.meshgrid(np.arange(1, rows + 1), np.arange(1, cols + 1), indexing="ij")
    r = np.stack([(u - cx) * tv / cx, (v - cy) * th / cy, np.ones_like(u, dtype=np.float64)], axis=-1)
    return r / np.linalg.norm(r, axis=-1, keepdims=True)


@dataclass
class DepthSensor:
    rays: np.ndarray  # [rows, cols, 3], camera frame


def Kinect(rows: int, cols: int, vertical_fov: float = 0.4682, horizontal_fov: float = 0.5449) -> DepthSensor:
    return DepthSensor(generate_kinect_rays(rows, cols, vertical_fov, horizontal_fov))


def rays_in_world(sensor: DepthSensor, tform: Transform) -> np.ndarray:
    return sensor.rays @ tform.R.T


def raycast_depths(surface: SceneSkin, sensor: DepthSensor, tform: Transform) -> np.ndarray:
    """[rows, cols] depths (NaN = miss)."""
    rw = rays_in_world(sensor, tform)
    rw = rw / np.linalg.norm(rw, axis=-1, keepdims=True)  # normalize(rays[i]) (:93)
    d = surface.raycast(tform.t, rw.reshape(-1, 3))
    return d.reshape(sensor.rays.shape[:2])


def raycast_points(surface: SceneSkin, sensor: DepthSensor, tform: Transform) -> np.ndarray:
    """World points of every hit, row-major (:99-113)."""
    d = raycast_depths(surface, sensor, tform)
    hit = ~np.isnan(d)
    r = sensor.rays / np.linalg.norm(sensor.rays, axis=-1, keepdims=True)
    return tform.apply(d[hit][:, None] * r[hit])


def raycast(state: ManipulatorState, sensor: DepthSensor, tform: Transform, device: int = 0) -> np.ndarray:
    return raycast_points(skin(state, device), sensor, tform)
