"""URDF subset parser (links, visuals, joints) — host side of Models.load_urdf.

Restates what RigidBodyDynamics.parse_urdf + RigidBodyTreeInspector.parse_urdf_visuals
(src/models.jl:166-171) extract for the convex-hull model: joint origin
(xyz, rpy), axis, type and limits; each link's visual origin and mesh. Mesh URIs
`package://PKG/rest` are resolved against `package_path` and then against the
URDF file's own ancestors named PKG.
"""
from __future__ import annotations

import os
import xml.etree.ElementTree as ET


def _floats(s, n, default):
    if s is None:
        return list(default)
    v = [float(x) for x in s.split()]
    if len(v) != n:
        raise ValueError(f"expected {n} numbers, got {s!r}")
    return v


def _origin(el):
    o = el.find("origin") if el is not None else None
    if o is None:
        return [0.0, 0.0, 0.0], [0.0, 0.0, 0.0]
    return _floats(o.get("xyz"), 3, (0, 0, 0)), _floats(o.get("rpy"), 3, (0, 0, 0))


def parse_urdf_string(text: str) -> dict:
    root = ET.fromstring(text)
    links = []
    for ln in root.findall("link"):
        visuals = []
        for vis in ln.findall("visual"):
            xyz, rpy = _origin(vis)
            geom = vis.find("geometry")
            entry = {"xyz": xyz, "rpy": rpy}
            mesh = geom.find("mesh") if geom is not None else None
            box = geom.find("box") if geom is not None else None
            if mesh is not None:
                entry["mesh"] = mesh.get("filename")
                entry["scale"] = _floats(mesh.get("scale"), 3, (1, 1, 1))
            elif box is not None:
                entry["box"] = _floats(box.get("size"), 3, (0, 0, 0))
            else:
                continue
            visuals.append(entry)
        links.append({"name": ln.get("name"), "visuals": visuals})
    joints = []
    for j in root.findall("joint"):
        xyz, rpy = _origin(j)
        lim = j.find("limit")
        ax = j.find("axis")
        joints.append({
            "name": j.get("name"), "type": j.get("type"),
            "parent": j.find("parent").get("link"), "child": j.find("child").get("link"),
            "xyz": xyz, "rpy": rpy,
            "axis": _floats(ax.get("xyz") if ax is not None else None, 3, (1, 0, 0)),
            "lower": float(lim.get("lower")) if lim is not None and lim.get("lower") else None,
            "upper": float(lim.get("upper")) if lim is not None and lim.get("upper") else None,
        })
    return {"name": root.get("name"), "links": links, "joints": joints}


def parse_urdf(path: str) -> dict:
    with open(path) as f:
        d = parse_urdf_string(f.read())
    d["path"] = os.path.abspath(path)
    return d


def resolve_mesh(uri: str, urdf_path: str | None, package_path=()) -> str:
    if uri.startswith("package://"):
        pkg, _, rest = uri[len("package://"):].partition("/")
        cands = [os.path.join(p, pkg, rest) for p in package_path]
        if urdf_path:
            d = os.path.dirname(os.path.abspath(urdf_path))
            while d and d != os.path.dirname(d):
                if os.path.basename(d) == pkg:
                    cands.append(os.path.join(d, rest))
                d = os.path.dirname(d)
        for c in cands:
            if os.path.exists(c):
                return c
        raise FileNotFoundError(f"cannot resolve {uri} (searched {cands})")
    if urdf_path and not os.path.isabs(uri):
        return os.path.join(os.path.dirname(urdf_path), uri)
    return uri


def root_link(d: dict) -> str:
    children = {j["child"] for j in d["joints"]}
    roots = [ln["name"] for ln in d["links"] if ln["name"] not in children]
    if len(roots) != 1:
        raise ValueError(f"URDF must have exactly one root link, found {roots}")
    return roots[0]
