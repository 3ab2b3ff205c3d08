"""Copy the head of the reference's recorded Kinect cloud as a test fixture.

examples/data/squishable_unsquished_xyzrgb.txt (25,571 points + origin line) is
data the reference's notebooks read (examples/squishable.ipynb); the first 400
points are kept under tests/golden/ so the ingest and the GPU raycast/cost tests
run where /root/reference is absent.

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


if __name__ == "__main__":
    main(*sys.argv[1:])
