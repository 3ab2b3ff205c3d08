"""The reference's own iso-surface mesh counts (tests/golden/contour_pins.json),
CPU oracle side. GPU side (the scene sampled through the product path):
tests/test_gpu_contour_pins.py. Helper and the restated meshing:
tests/contour_mesh.py.

What each count pins:
* squishable 294 / 584 (examples/squishable.ipynb:230) — REPRODUCED. It
  depends only on the sign of the RBF field on a 9x9x8 grid, i.e. on the
  zero set of SpatialFields' InterpolatingSurface (no normalization moves it)
  and on the grid convention: r^3 with an affine (or constant) tail gives
  294 / 584; r^5, r, r^2 log r and the tail-free r^3 do not, nor does an
  endpoint-exact linspace grid. First reference-held evidence that the
  implemented RBF interpolant is the reference's.
* IRB140 2,226 / 4,460 (examples/irb140.ipynb:299) — NOT reproduced: the exact
  polytope SDF gives 2,242 / 4,480, robust to every grid convention. The
  reference's surface has Euler characteristic V - F/2 = -4 where ours is 2.
  A single node flip CAN change χ (one isolated node in: (14, 24), χ = 2,
  test_mesh_counts_closed_surfaces; a node at a thin junction can open or
  close a tunnel), so χ alone does not tell a shape change from a few flips;
  moving every node within δ of the iso level (δ 1e-4 .. 1e-2) to either side
  keeps χ = 2. EnhancedGJK's hill-climbing NeighborMesh support and
  warm-started simplex (un-vendored @404de6a9) were emulated over three mesh
  loaders (merged STL, STL triangle soup, .obj face indices), two initial
  simplices and two warm-start orders (tools/contour_study.py,
  profiles/r05/contour_study.txt): the merged STL and the .obj give 2,242 /
  4,480 with no node on the other side of the iso level, the soup 276 / 528
  or 202 / 384. No variant gives 2,226 / 4,460; the cause stays open without
  the package.
* C5 4,494 / 8,912 (examples/irb_and_squishable.ipynb:318) — NOT reproduced:
  4,390 / 8,712; the arm's part is the IRB140 mesh above (same relative grid)
  and the rest depends on the RBF skin's normalization near its zero set.
The measured counts are pinned (a change means the SDF moved); the reference
counts are strict xfails."""
import json
import os

import numpy as np
import pytest

import contour_mesh as cm
from conftest import GOLDEN

PINS = json.load(open(os.path.join(GOLDEN, "contour_pins.json")))["pins"]
# measured with this repo's SDF (oracle == GPU path, bit for bit)
MEASURED = {"irb140": (2242, 4480), "irb_and_squishable": (4390, 8712), "squishable": (294, 584)}


def oracle_sdf(oracle_mod, m, x):
    import flash
    from flash import rbf as host_rbf
    nq = m.mechanism.num_positions
    q = m.mechanism.normalize(x[:nq])
    om = oracle_mod.OracleModel.from_manipulator(m)
    poses = flash.core.surface_poses(m, q)
    rows = host_rbf.rows(host_rbf.solve(m, q, x[nq:])) if m.has_rbf() else None
    return lambda pts: om.skin(poses, pts, rbf_rows=rows)[0]


def counts(oracle_mod, name, variant="ceil"):
    m, x, lb, ub, iso, res = cm.pinned_case(name)
    axes = cm.grid_axes(lb, ub, res, variant)
    vals = cm.to_volume(oracle_sdf(oracle_mod, m, x)(cm.grid_points(axes)), axes)
    return cm.mesh_counts(cm.classify(vals, iso))


def test_expected_matches_fixture():
    for name, (V, F) in cm.EXPECTED.items():
        assert (PINS[name]["vertices"], PINS[name]["faces"]) == (V, F)


def test_mesh_counts_closed_surfaces():
    """A voxelised ball and a solid torus: closed meshes, V - F/2 = χ = 2 / 0."""
    g = np.arange(-1.5, 1.5001, 0.1)
    X, Y, Z = np.meshgrid(g, g, g, indexing="ij")
    V, F = cm.mesh_counts(X ** 2 + Y ** 2 + Z ** 2 < 1.0)
    assert V - F // 2 == 2 and F % 2 == 0
    V, F = cm.mesh_counts((np.sqrt(X ** 2 + Y ** 2) - 0.9) ** 2 + Z ** 2 < 0.35 ** 2)
    assert V - F // 2 == 0
    # one node in: its 14 lattice edges (6 axis, 6 face-diagonal, 2 body-diagonal) cross, 24 tetrahedra
    b = np.zeros((3, 3, 3), bool)
    b[1, 1, 1] = True
    assert cm.mesh_counts(b) == (14, 24)


def test_grid_convention():
    """GeometryTypes' SignedDistanceField: n = ceil(rng/res) steps of res from
    the lower bound (the grid may overshoot the upper bound)."""
    ax = cm.grid_axes((-0.5, -0.5, -0.25), (1.0, 0.5, 1.0), 0.05)
    assert [len(a) for a in ax] == [31, 21, 26]
    assert ax[0][1] == 1 * 0.05 + -0.5


def test_squishable_zero_set_matches_reference(oracle_mod):
    assert counts(oracle_mod, "squishable") == cm.EXPECTED["squishable"]


def test_squishable_count_discriminates(oracle_mod):
    """The 294 / 584 pin is informative: other interpolants or an
    endpoint-exact grid give other counts (independent numpy fits)."""
    m, x, lb, ub, iso, res = cm.pinned_case("squishable")
    from flash import rbf as host_rbf
    C = host_rbf.solve(m, m.mechanism.normalize(x[:7]), x[7:])[0].centres
    v = np.concatenate([np.zeros(12), [-1.0]])
    axes = cm.grid_axes(lb, ub, res)
    P = cm.grid_points(axes)

    def fit_count(phi, tail, axes=axes, P=P):
        n = len(C)
        A = phi(np.linalg.norm(C[:, None] - C[None], axis=-1))
        T = np.hstack([np.ones((n, 1)), C]) if tail else np.zeros((n, 0))
        k = T.shape[1]
        u = np.linalg.solve(np.block([[A, T], [T.T, np.zeros((k, k))]]), np.concatenate([v, np.zeros(k)]))
        f = phi(np.linalg.norm(P[:, None] - C[None], axis=-1)) @ u[:n]
        if tail:
            f = f + u[n] + P @ u[n + 1:]
        return cm.mesh_counts(cm.to_volume(f, axes) < 0.0)

    assert fit_count(lambda r: r ** 3, True) == (294, 584)
    for phi, tail in ((lambda r: r ** 3, False), (lambda r: r ** 5, True), (lambda r: r, True),
                      (lambda r: np.where(r > 0, r * r * np.log(np.where(r > 0, r, 1.0)), 0.0), True)):
        assert fit_count(phi, tail) != (294, 584)
    lin = cm.grid_axes(lb, ub, res, "linspace")
    assert fit_count(lambda r: r ** 3, True, lin, cm.grid_points(lin)) != (294, 584)


@pytest.mark.parametrize("name", ["irb140", "irb_and_squishable"])
def test_measured_counts(oracle_mod, name):
    """Robust to the grid convention (every variant gives the same count)."""
    for variant in ("ceil", "round", "floor", "linspace"):
        assert counts(oracle_mod, name, variant) == MEASURED[name]


def test_irb140_part_of_c5(oracle_mod):
    """The C5 region samples the arm (base at z = 0.75) at the same relative
    grid as the IRB140 call: its component of the C5 mesh is the IRB140 mesh."""
    from scipy import ndimage
    m, x, lb, ub, iso, res = cm.pinned_case("irb_and_squishable")
    axes = cm.grid_axes(lb, ub, res)
    P = cm.grid_points(axes)
    d = oracle_sdf(oracle_mod, m, x)(P)
    ins = cm.to_volume(d, axes) < iso
    lab, n = ndimage.label(ins, structure=np.ones((3, 3, 3)))
    parts = sorted(cm.mesh_counts(lab == c) for c in range(1, n + 1))
    assert n == 2 and MEASURED["irb140"] in parts


@pytest.mark.xfail(strict=True, reason="hull SDF = exact polytope distance: 2,242 / 4,480 vs the reference's "
                                       "2,226 / 4,460 (EnhancedGJK support/warm start; DESIGN.md §3)")
def test_irb140_matches_reference(oracle_mod):
    assert counts(oracle_mod, "irb140") == cm.EXPECTED["irb140"]


@pytest.mark.xfail(strict=True, reason="C5: 4,390 / 8,712 vs 4,494 / 8,912 (the IRB140 part and the RBF skin's "
                                       "normalization near its zero set; DESIGN.md §3)")
def test_c5_matches_reference(oracle_mod):
    assert counts(oracle_mod, "irb_and_squishable") == cm.EXPECTED["irb_and_squishable"]
