"""The C-ABI boundary: library loads, exports every declared symbol, fails
loudly without a device, and the host hull builder matches qhull."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REFERENCE, ROOT, rng

HEADER = os.path.join(ROOT, "include", "flashsdf.h")


def header_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(fsdf_\w+)\s*\(", text, re.M)))


def test_library_exports_every_header_symbol():
    from flash import _lib
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (fsdf_\w+)", out))
    assert set(names) <= exported
    # the ctypes prototypes cover exactly the header
    assert sorted(_lib.SYMBOLS) == names


def test_library_targets_gfx950():
    from flash import _lib
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", _lib.LIB_PATH],
                         capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in out.stdout + out.stderr


def _has_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


def test_no_cpu_fallback_without_device():
    if _has_gpu():
        pytest.skip("a GPU is visible")
    from flash import _lib
    with pytest.raises(_lib.FlashNativeError) as e:
        _lib.Context(device=0)
    assert e.value.status == 2  # FSDF_ERR_HIP


def test_compute_entry_points_reject_null_context():
    from flash import _lib
    lib = _lib.load()
    assert lib.fsdf_eval(None, None, None, None, None, None, None) == 1
    assert lib.fsdf_set_points(None, None, 0) == 1
    assert lib.fsdf_destroy(None) == 1
    assert lib.fsdf_last_error(None) == b"null context"


# ---- host hull builder vs qhull -------------------------------------------------
def _check_hull(points):
    from scipy.spatial import ConvexHull as QH
    from flash.geometry import ConvexHull
    h = ConvexHull.from_points(points)
    q = QH(points)
    # same vertex set
    assert len(h.vertices) == len(q.vertices)
    assert np.allclose(np.sort(h.vertices, axis=0), np.sort(points[q.vertices], axis=0))
    # unit outward planes containing every vertex
    n = h.planes[:, :3]
    assert np.allclose(np.linalg.norm(n, axis=1), 1.0)
    assert (points @ n.T - h.planes[:, 3] <= 1e-12 * np.abs(points).max()).all()
    # same volume (divergence theorem over the triangles)
    a, b, c = (h.vertices[h.faces[:, i]] for i in range(3))
    vol = np.einsum("ij,ij->i", a, np.cross(b, c)).sum() / 6.0
    assert vol == pytest.approx(q.volume, rel=1e-12)
    # every face outward: centroid strictly inside
    cen = h.vertices.mean(0)
    assert (cen @ n.T - h.planes[:, 3] < 0).all()
    # closed 2-manifold: every directed edge has its twin
    e = set()
    for f in h.faces:
        for i in range(3):
            e.add((f[i], f[(i + 1) % 3]))
    assert all((b_, a_) in e for a_, b_ in e)
    return h


def test_hull_irb140_meshes_match_qhull():
    from flash.models import _irb140_fixture
    fx = _irb140_fixture()
    for name, v in fx["meshes"].items():
        h = _check_hull(np.asarray(v))
        assert len(h.vertices) == 52 and len(h.faces) == 100, name


@pytest.mark.parametrize("seed", range(5))
def test_hull_random_clouds(seed):
    r = rng(seed)
    pts = r.normal(size=(200, 3)) * [1.0, 0.3, 2.0]
    _check_hull(pts)


def test_hull_box_with_coplanar_points():
    pts = np.array([[x, y, z] for x in (-1, 0, 1) for y in (-1, 0, 1) for z in (-1, 0, 1)], float)
    from flash.geometry import ConvexHull
    h = ConvexHull.from_points(pts)
    assert len(h.vertices) == 8 and len(h.faces) == 12


def test_hull_degenerate_inputs():
    from flash import _lib
    flat = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0], [0.5, 0.5, 0]], float)
    with pytest.raises(_lib.FlashNativeError) as e:
        _lib.convex_hull(flat)
    assert e.value.status == 5
    with pytest.raises(_lib.FlashNativeError):
        _lib.convex_hull(np.zeros((3, 3)))
    with pytest.raises(_lib.FlashNativeError) as e:
        _lib.convex_hull(np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, np.nan]]))
    assert e.value.status == 1


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference checkout absent (GPU box)")
def test_stl_ingest_matches_fixture():
    """read_stl_vertices on the reference STLs reproduces the committed fixture."""
    from flash.geometry import read_stl_vertices
    from flash.models import _irb140_fixture
    fx = _irb140_fixture()
    base = os.path.join(REFERENCE, "examples/data/IRB140/urdf/meshes")
    for name, v in fx["meshes"].items():
        assert np.array_equal(read_stl_vertices(os.path.join(base, name)), np.asarray(v))
