"""Extract the IRB140 convex-hull model fixture from the reference's data files.

Reads (container only; /root/reference never reaches the GPU box):
  examples/data/IRB140/urdf/irb_140_convhull.urdf      joints, link visual origins
  examples/data/IRB140/urdf/irb_140_robotiq_ati.urdf   ati_joint (ATI sensor on link_6)
  examples/data/IRB140/urdf/ATI_sensor.urdf            ATI visual origin
  examples/data/IRB140/urdf/meshes/*_chull.stl         hull vertex sets
and writes point-cloud-signed-distance_amd/flash/data/irb140.json: the parsed
URDF description plus each mesh's unique float64 vertices (float32 STL values,
widened exactly). Data only — no reference source is copied.

    python tools/extract_irb140.py [/root/reference]
"""
import json
import os
import sys
import xml.etree.ElementTree as ET

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "point-cloud-signed-distance_amd"))

from flash import urdf as U  # noqa: E402
from flash.geometry import read_stl_vertices  # noqa: E402


def main(ref="/root/reference"):
    base = os.path.join(ref, "examples/data/IRB140/urdf")
    desc = U.parse_urdf(os.path.join(base, "irb_140_convhull.urdf"))
    desc.pop("path", None)
    meshes = {}
    for ln in desc["links"]:
        for v in ln["visuals"]:
            name = os.path.basename(v["mesh"])
            meshes[name] = read_stl_vertices(os.path.join(base, "meshes", name)).tolist()
    # ATI sensor: joint from the robotiq_ati variant, visual origin from ATI_sensor.urdf
    ati_j = [j for j in U.parse_urdf(os.path.join(base, "irb_140_robotiq_ati.urdf"))["joints"]
             if j["name"] == "ati_joint"][0]
    ati_v = U.parse_urdf(os.path.join(base, "ATI_sensor.urdf"))["links"][0]["visuals"][0]
    meshes["ATI_sensor_chull.stl"] = read_stl_vertices(os.path.join(base, "meshes", "ATI_sensor_chull.stl")).tolist()
    out = {
        "source": "examples/data/IRB140/urdf (irb_140_convhull.urdf, irb_140_robotiq_ati.urdf:1312-1316, "
                  "ATI_sensor.urdf, meshes/*_chull.stl)",
        "urdf": desc,
        "ati": {"parent": ati_j["parent"], "xyz": ati_j["xyz"], "rpy": ati_j["rpy"],
                "visual_xyz": ati_v["xyz"], "visual_rpy": ati_v["rpy"], "mesh": "ATI_sensor_chull.stl"},
        "meshes": meshes,
    }
    dst = os.path.join(HERE, "..", "point-cloud-signed-distance_amd", "flash", "data", "irb140.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.normpath(dst), {k: len(v) for k, v in meshes.items()})


if __name__ == "__main__":
    main(*sys.argv[1:])
