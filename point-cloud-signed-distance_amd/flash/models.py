"""Model factories — module Flash.Models (src/models.jl).

  two_link_arm(deformable)   src/models.jl:19-71   (RBF skin; 46 centres, 2 DOF)
  beanbag()                  src/models.jl:73-98   (deformable RBF; 25 DOF)
  squishable()               src/models.jl:100-136 (deformable RBF; 43 DOF)
  load_urdf(file; package_path)  src/models.jl:154-171 (convex hulls of URDF visuals)
  merge(m1, m2)              src/models.jl:173-177 (merge!)
plus the scene pieces the notebooks build inline:
  table()                    examples/irb_and_squishable.ipynb cell 3 (8-vertex box)
  irb140(ati)                the IRB140 convex-hull robot from the committed
                             model fixture (flash/data/irb140.json, extracted
                             from examples/data/IRB140 by tools/extract_irb140.py)
  arm_grid(...)              M64, the metric's 64-primitive model:
                             8 IRB140 arms (7 link hulls + ATI sensor hull) on a
                             2x4 grid at 1.2 m pitch, 48 revolute DOF.
"""
from __future__ import annotations

import json
import math
import os

import numpy as np

from .core import (ConvexGeometry, DeformableInterpolatingSkin, Manipulator, RigidInterpolatingSkin)
from .geometry import ConvexHull, Transform, read_stl_vertices
from .mechanism import Fixed, Mechanism, QuaternionFloating, Revolute
from . import urdf as _urdf

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def two_link_arm(deformable: bool = False) -> Manipulator:
    """src/models.jl:19-71 (`deformable` is ignored there too)."""
    link_length, radius = 1.0, 0.1
    mech = Mechanism("world")
    parent = 0
    surface, skeleton = [], []
    for i in (1, 2):
        j2p = Transform(np.eye(3), np.array([link_length, 0.0, 0.0])) if i > 1 else None
        body = mech.attach(parent, Revolute([0, 0, 1], f"joint{i}"), j2p, f"body{i}")
        parent = body
        for x in np.linspace(0.3 * link_length, 0.7 * link_length, 3):
            for y in (-radius, radius):
                for z in (-radius, radius):
                    surface.append((body, [x, y, z]))
            for z in (-math.sqrt(2) * radius, math.sqrt(2) * radius):
                surface.append((body, [x, 0.0, z]))
        if i == 1:
            for z in (-math.sqrt(2) * radius, math.sqrt(2) * radius):
                surface.append((body, [link_length, 0.0, z]))
            surface.append((body, [0.0, 0.0, 0.0]))
        else:
            surface.append((body, [link_length, 0.0, 0.0]))
        for x in np.linspace(0.2 * link_length, 0.8 * link_length, 3):
            skeleton.append((body, [x, 0.0, 0.0]))
    return Manipulator(mech, [RigidInterpolatingSkin(surface, skeleton)])


def beanbag() -> Manipulator:
    """src/models.jl:73-98."""
    mech = Mechanism("world")
    body = mech.attach(0, QuaternionFloating("joint1"), None, "body1")
    surface = []
    for axis in range(3):
        for s in (-1.0, 1.0):
            x = [0.0, 0.0, 0.0]
            x[axis] = s
            surface.append((body, x))
    return Manipulator(mech, [DeformableInterpolatingSkin(surface, [(body, [0.0, 0.0, 0.0])])])


def squishable() -> Manipulator:
    """src/models.jl:100-136 (tan(π/4) kept as computed, not replaced by 1)."""
    mech = Mechanism("world")
    body = mech.attach(0, QuaternionFloating("joint1"), None, "squishable_body")
    radii = [0.44 / 2, 0.40 / 2, 0.30 / 2]
    surface = []
    for axis in (1, 2, 3):
        for i_sign in (-1, 1):
            for j_sign in (-1, 1):
                theta = math.pi / 4
                x = [0.0, 0.0, 0.0]
                i = axis % 3 + 1
                j = i % 3 + 1
                a = radii[i - 1] * 1.25
                b = radii[j - 1] * 1.25
                t2 = math.tan(theta) ** 2
                x[i - 1] = i_sign * math.sqrt(a ** 2 * b ** 2 / (a ** 2 * t2 + b ** 2))
                x[j - 1] = j_sign * math.sqrt(b ** 2 * (1 - b ** 2 / (a ** 2 * t2 + b ** 2)))
                surface.append((body, x))
    return Manipulator(mech, [DeformableInterpolatingSkin(surface, [(body, [0.0, 0.0, 0.0])])])


def box_hull(half_extents) -> ConvexHull:
    hx, hy, hz = half_extents
    pts = [[x, y, z] for z in (-hz, hz) for x in (-hx, hx) for y in (-hy, hy)]
    return ConvexHull.from_points(np.array(pts, np.float64))


def table(width: float = 0.25, thickness: float = 0.05) -> Manipulator:
    """The floating table box of examples/irb_and_squishable.ipynb (cell 3)."""
    mech = Mechanism("world")
    body = mech.attach(0, QuaternionFloating("joint1"), None, "table_body")
    return Manipulator(mech, [ConvexGeometry(box_hull((width, width, thickness)), body, name="table")])


def merge(m1: Manipulator, m2: Manipulator) -> Manipulator:
    """merge!(manip1, manip2) (src/models.jl:173-177): graft m2 under m1's root."""
    remap = m1.mechanism.attach_mechanism(m2.mechanism, 0)
    for s in m2.surfaces:
        if isinstance(s, ConvexGeometry):
            m1.surfaces.append(ConvexGeometry(s.hull, remap[s.body], s.frame, s.name))
        else:
            t = type(s)
            m1.surfaces.append(t([(remap[b], p) for b, p in s.surface_points],
                                 [(remap[b], p) for b, p in s.skeleton_points]))
    m1.invalidate()
    return m1


# ---------------------------------------------------------------------------
# URDF robots
# ---------------------------------------------------------------------------
def _build_from_urdf(desc: dict, mesh_vertices, suffix: str = "", base: Transform | None = None,
                     mech: Mechanism | None = None, surfaces: list | None = None):
    """Mechanism + ConvexGeometry per link visual. The root link is attached to
    the world by a Fixed joint at `base` (RigidBodyDynamics.parse_urdf)."""
    mech = mech or Mechanism("world")
    surfaces = [] if surfaces is None else surfaces
    root = _urdf.root_link(desc)
    links = {ln["name"]: ln for ln in desc["links"]}
    body_of = {root: mech.attach(0, Fixed(f"{root}_to_world{suffix}"), base, root + suffix)}
    pending = list(desc["joints"])
    while pending:
        progressed = False
        for j in list(pending):
            if j["parent"] in body_of:
                kind = j["type"]
                if kind in ("revolute", "continuous"):
                    jt = Revolute(j["axis"], j["name"] + suffix,
                                  j["lower"] if j["lower"] is not None else -np.inf,
                                  j["upper"] if j["upper"] is not None else np.inf)
                elif kind == "fixed":
                    jt = Fixed(j["name"] + suffix)
                elif kind == "floating":
                    jt = QuaternionFloating(j["name"] + suffix)
                else:
                    raise NotImplementedError(f"URDF joint type {kind!r}")
                body_of[j["child"]] = mech.attach(body_of[j["parent"]], jt, Transform.from_xyz_rpy(j["xyz"], j["rpy"]),
                                                  j["child"] + suffix)
                pending.remove(j)
                progressed = True
        if not progressed:
            raise ValueError("URDF joints do not form a tree rooted at " + root)
    for name, body in body_of.items():
        for vis in links[name]["visuals"]:
            frame = Transform.from_xyz_rpy(vis["xyz"], vis["rpy"])
            if "mesh" in vis:
                verts = np.asarray(mesh_vertices(vis["mesh"]), np.float64) * np.asarray(vis.get("scale", [1, 1, 1]))
                hull = ConvexHull.from_points(verts)
            else:
                hull = box_hull(np.asarray(vis["box"]) / 2)
            surfaces.append(ConvexGeometry(hull, body, frame, name + suffix))
    return mech, surfaces, body_of


def load_urdf(filename: str, package_path=()) -> Manipulator:
    """load_urdf(filename; package_path) (src/models.jl:166-171)."""
    desc = _urdf.parse_urdf(filename)
    cache = {}

    def mesh_vertices(uri):
        if uri not in cache:
            cache[uri] = read_stl_vertices(_urdf.resolve_mesh(uri, filename, package_path))
        return cache[uri]

    mech, surfaces, _ = _build_from_urdf(desc, mesh_vertices)
    return Manipulator(mech, surfaces)


def _irb140_fixture(path: str | None = None) -> dict:
    with open(path or os.path.join(DATA_DIR, "irb140.json")) as f:
        return json.load(f)


def _add_irb140(mech, surfaces, fx, suffix, base: Transform | None, ati: bool):
    meshes = fx["meshes"]
    mech, surfaces, body_of = _build_from_urdf(fx["urdf"], lambda uri: meshes[os.path.basename(uri)], suffix, base,
                                               mech, surfaces)
    if ati:
        a = fx["ati"]
        body = mech.attach(body_of[a["parent"]], Fixed("ati_joint" + suffix),
                           Transform.from_xyz_rpy(a["xyz"], a["rpy"]), "ATI_sensor" + suffix)
        hull = ConvexHull.from_points(np.asarray(meshes[a["mesh"]], np.float64))
        surfaces.append(ConvexGeometry(hull, body, Transform.from_xyz_rpy(a["visual_xyz"], a["visual_rpy"]),
                                       "ATI_sensor" + suffix))
    return mech, surfaces


def irb140(ati: bool = False, fixture: str | None = None) -> Manipulator:
    """The IRB140 convex-hull arm (examples/data/IRB140/urdf/irb_140_convhull.urdf):
    7 link hulls, 6 revolute DOF; `ati` adds the ATI sensor hull fixed to link_6
    (ati_joint of irb_140_robotiq_ati.urdf)."""
    fx = _irb140_fixture(fixture)
    mech, surfaces = _add_irb140(Mechanism("world"), [], fx, "", None, ati)
    return Manipulator(mech, surfaces)


def arm_grid(rows: int = 2, cols: int = 4, pitch: float = 1.2, ati: bool = True,
             fixture: str | None = None) -> Manipulator:
    """M64: rows x cols IRB140 arms at `pitch` metres, each with
    7 link hulls + the ATI hull = 8 hulls/arm; 2x4 -> 64 hulls, 48 DOF."""
    fx = _irb140_fixture(fixture)
    mech, surfaces = Mechanism("world"), []
    for r in range(rows):
        for c in range(cols):
            base = Transform(np.eye(3), np.array([c * pitch, r * pitch, 0.0]))
            mech, surfaces = _add_irb140(mech, surfaces, fx, f"_a{r * cols + c}", base, ati)
    return Manipulator(mech, surfaces)


def joint_limits(manip: Manipulator):
    lo = np.full(manip.mechanism.num_positions, -np.inf)
    hi = np.full(manip.mechanism.num_positions, np.inf)
    for b in range(1, manip.mechanism.num_bodies):
        e = manip.mechanism.edges[b]
        if e.joint.kind == "revolute":
            lo[e.q_offset], hi[e.q_offset] = e.joint.lower, e.joint.upper
    return lo, hi


def irb_and_squishable():
    """The multi-body scene of examples/irb_and_squishable.ipynb (cells 3-6):
    IRB140 with its base joint made QuaternionFloating (cell 4), merged with
    squishable() and the table box; surfaces = 7 hulls + squishable RBF + table
    (9), 63 states. Returns (manipulator, x0) with the notebook's placements
    (cell 6): IRB t = (0, 0, 0.75), squishable t = (0.55, 0.45, 0.8),
    table t = (0.4, 0, 0.6)."""
    from .core import num_states
    m = irb140()
    m.mechanism.change_joint_type(1, QuaternionFloating("base_link_floating"))
    merge(m, squishable())
    merge(m, table())
    x0 = np.zeros(num_states(m))
    x0[:m.mechanism.num_positions] = m.mechanism.zero_configuration()
    for name, t in (("base_link", (0.0, 0.0, 0.75)), ("squishable_body", (0.55, 0.45, 0.8)),
                    ("table_body", (0.4, 0.0, 0.6))):
        rng = m.mechanism.q_range(m.mechanism.body_index(name))
        x0[rng.start + 4: rng.start + 7] = t
    return m, x0
