"""Independent forward kinematics for the IRB140 fixture — TEST INFRASTRUCTURE ONLY.

Restates RigidBodyDynamics' URDF kinematics (transform_to_root, src/Flash.jl:248;
parse_urdf, src/models.jl:167) with 4x4 homogeneous matrices and
scipy.spatial.transform.Rotation, sharing no code with flash.mechanism:
  T_child = T_parent · H(origin xyz, rpy) · H(AngleAxis(q, axis))
  hull pose = T_link · H(visual origin)
Used to pin the product's FK (tests/test_kinematics.py).
"""
from __future__ import annotations

import numpy as np
from scipy.spatial.transform import Rotation


def H(xyz=(0, 0, 0), R=None):
    M = np.eye(4)
    if R is not None:
        M[:3, :3] = R
    M[:3, 3] = xyz
    return M


def H_rpy(xyz, rpy):
    # URDF fixed-axis roll-pitch-yaw: R = Rz(y) Ry(p) Rx(r) == extrinsic 'xyz'
    return H(xyz, Rotation.from_euler("xyz", rpy).as_matrix())


def irb140_hull_poses(fixture: dict, q, base=None, ati=False):
    """World 4x4 pose of every visual hull, in the URDF link order (+ATI)."""
    desc = fixture["urdf"]
    T = {}
    links = [ln["name"] for ln in desc["links"]]
    children = {j["child"] for j in desc["joints"]}
    root = [n for n in links if n not in children][0]
    T[root] = np.eye(4) if base is None else base
    qi = 0
    joints = list(desc["joints"])
    while joints:
        for j in list(joints):
            if j["parent"] in T:
                M = T[j["parent"]] @ H_rpy(j["xyz"], j["rpy"])
                if j["type"] == "revolute":
                    ax = np.asarray(j["axis"], float)
                    ax = ax / np.linalg.norm(ax)
                    M = M @ H((0, 0, 0), Rotation.from_rotvec(q[qi] * ax).as_matrix())
                    qi += 1
                T[j["child"]] = M
                joints.remove(j)
    poses = []
    for ln in desc["links"]:
        for v in ln["visuals"]:
            poses.append(T[ln["name"]] @ H_rpy(v["xyz"], v["rpy"]))
    if ati:
        a = fixture["ati"]
        poses.append(T[a["parent"]] @ H_rpy(a["xyz"], a["rpy"]) @ H_rpy(a["visual_xyz"], a["visual_rpy"]))
    return poses
