"""Read the reference notebooks' printed contour-mesh sizes into
tests/golden/contour_pins.json (the fixture tests/test_contour_pins.py and
tests/test_gpu_contour_pins.py check against).

Each notebook cell that calls DrakeVisualizer.contour_mesh (directly, or via
Flash.draw -> src/Flash.jl:316-323) prints
`HomogenousMesh(vertices: Vx..., faces: Fx...)`; the line numbers are those
of the .ipynb JSON files.

    python tests/golden/make_contour_pins.py [/root/reference]
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = {  # name: (notebook, printed-at line)
    "irb140": ("examples/irb140.ipynb", 299),
    "irb_and_squishable": ("examples/irb_and_squishable.ipynb", 318),
    "squishable": ("examples/squishable.ipynb", 230),
}


def main(ref="/root/reference"):
    path = os.path.join(HERE, "contour_pins.json")
    fx = json.load(open(path))
    for name, (nb, line) in SOURCES.items():
        text = open(os.path.join(ref, nb)).read().splitlines()[line - 1]
        m = re.search(r"vertices: (\d+)x.*faces: (\d+)x", text)
        V, F = int(m.group(1)), int(m.group(2))
        pin = fx["pins"][name]
        assert pin["printed_at"] == f"{nb}:{line}"
        pin["vertices"], pin["faces"] = V, F
        print(name, V, F)
    with open(path, "w") as f:
        json.dump(fx, f, indent=2)
        f.write("\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
