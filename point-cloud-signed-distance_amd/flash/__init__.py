"""flash — MI355X-native residual pass of Flash.jl (host package).

Module layout mirrors `module Flash` (src/Flash.jl): core types and
`skin(state)` here, submodules `Models`, `GradientDescent`, `Tracking`.
The compute path is libflashsdf.so (HIP, gfx950) through ctypes; there is no
CPU fallback.
"""
from .core import (BodyGeometry, ConvexGeometry, DeformableInterpolatingSkin, InterpolatingGeometry,
                   Manipulator, ManipulatorState, RigidInterpolatingSkin, SceneSkin, hull_poses,
                   num_deformations, num_states, skin, surfaces)
from . import models as Models  # noqa: N812
from ._lib import FlashNativeError

__all__ = ["BodyGeometry", "ConvexGeometry", "DeformableInterpolatingSkin", "InterpolatingGeometry",
           "Manipulator", "ManipulatorState", "RigidInterpolatingSkin", "SceneSkin", "hull_poses",
           "num_deformations", "num_states", "skin", "surfaces", "Models", "FlashNativeError"]


def __getattr__(name):
    # GradientDescent / Tracking import lazily (they pull in the solver)
    if name == "GradientDescent":
        from . import gradientdescent
        return gradientdescent
    if name == "Tracking":
        from . import tracking
        return tracking
    if name == "DepthSensors":
        from . import depthsensors
        return depthsensors
    if name == "DepthData":
        from . import depthdata
        return depthdata
    raise AttributeError(name)
