"""Copy the head of the reference's recorded Kinect cloud as a test fixture.

examples/data/squishable_unsquished_xyzrgb.txt (25,571 points + origin line) is
data the reference's notebooks read (examples/squishable.ipynb); the first 400
points are kept under tests/golden/ so the ingest and the GPU raycast/cost tests
run where /root/reference is absent; the whole cloud's positions go to
squishable_unsquished.npz (`xyz` [25,571 x 3] f64 as parsed, `origin` the
camera line) for BASELINE config 5 (the real cloud tiled and
jittered to 2^20 points, flash.synthetic.c5_cloud).

    python tests/golden/make_pointcloud_fixture.py [/root/reference]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main(ref="/root/reference"):
    src = os.path.join(ref, "examples/data/squishable_unsquished_xyzrgb.txt")
    with open(src) as f:
        lines = [next(f) for _ in range(401)]
    with open(os.path.join(HERE, "squishable_unsquished_head.txt"), "w") as f:
        f.writelines(lines)
    print("wrote", len(lines) - 1, "points")
    import numpy as np
    rows = [[float(v) for v in l.split(",")] for l in open(src) if l.strip()]
    origin = np.array(rows[0], np.float64)
    xyz = np.array([r[:3] for r in rows[1:]], np.float64)
    np.savez_compressed(os.path.join(HERE, "squishable_unsquished.npz"), xyz=xyz, origin=origin)
    print("wrote", len(xyz), "positions")


if __name__ == "__main__":
    main(*sys.argv[1:])
