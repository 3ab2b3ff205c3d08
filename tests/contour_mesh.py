"""Vertex and face counts of the reference's iso-surface meshes (test helper).

Three notebook cells print the size of a `DrakeVisualizer.contour_mesh` of a
Flash SDF (`HomogenousMesh(vertices: V, faces: F)`):

* examples/irb140.ipynb:299 (call :311): IRB140 at q = 0,
  `contour_mesh(skin, [-.5,-.5,-.25], [1,.5,1], 0.01, 0.05)` -> 2,226 / 4,460;
* examples/irb_and_squishable.ipynb:318 (call :336): the C5 scene at cell 6's
  poses, `contour_mesh(skin, [-.5,-.5,.5], [1,.5,2], 0.01, 0.05)` -> 4,494 / 8,912;
* examples/squishable.ipynb:230 (cell 6, `Flash.draw(state)`): the squishable
  RBF surface alone, `contour_mesh(surface, drawing_region(surface)..., 0.0, 0.1)`
  (src/Flash.jl:270-275, 316-323) -> 294 / 584.

The meshing lives in un-vendored packages (DrakeVisualizer, GeometryTypes
@705e5a64, REQUIRE.dev:20). Their published algorithms, restated here:

* `contour_mesh(f, lb, ub, iso, res)` samples `x -> f(x) - iso` on a
  `SignedDistanceField(HyperRectangle(lb, ub - lb), res)` and meshes its zero
  level with `HomogenousMesh(sdf, ...)`.
* `SignedDistanceField(f, bounds, res)`: with rng = maximum(bounds) -
  minimum(bounds) per axis, n = ceil(Int, rng/res), the field holds
  f(i*res + min) for i = 0:n (the grid may overshoot ub by < res).
* `HomogenousMesh(::SignedDistanceField)` is GeometryTypes' marching
  tetrahedra (isosurface.jl): each voxel is cut into six tetrahedra around its
  main diagonal (corners 1-7), a corner is "in" when value < iso, every lattice
  edge whose ends differ gets ONE vertex (keyed by edge, shared between voxels),
  and a tetrahedron with 1 or 3 corners in emits one triangle, with 2 in, two.

Hence V and F depend only on the sign pattern of f - iso on the grid: V = the
crossed edges of the 19-edge lattice (3 axes, the three face diagonals from the
low corner, the body diagonal), F = sum over tetrahedra. `mesh_counts` returns
both; `grid_axes` builds the sample grid for each convention variant, so that a
convention the restatement cannot pin from text (the rounding of n, how the
range is formed, endpoint-exact linspace) is enumerated rather than guessed.
"""
import math

import numpy as np

# voxel corner offsets, GeometryTypes numbering 1..8 (here 0..7)
CORNERS = ((0, 0, 0), (0, 1, 0), (1, 1, 0), (1, 0, 0), (0, 0, 1), (0, 1, 1), (1, 1, 1), (1, 0, 1))
# the six tetrahedra of a voxel, all around the diagonal corner 1 -> corner 7
TETS = ((0, 2, 1, 6), (0, 7, 3, 6), (0, 3, 2, 6), (0, 1, 5, 6), (0, 4, 7, 6), (0, 5, 4, 6))
# the seven lattice edge families: start at a grid node, step by the offset
EDGE_STEPS = ((1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 0), (1, 0, 1), (0, 1, 1), (1, 1, 1))

REGIONS = {
    # name: (lower bound, upper bound, iso level, resolution), as the notebooks call it
    "irb140": ((-0.5, -0.5, -0.25), (1.0, 0.5, 1.0), 0.01, 0.05),
    "irb_and_squishable": ((-0.5, -0.5, 0.5), (1.0, 0.5, 2.0), 0.01, 0.05),
}
EXPECTED = {"irb140": (2226, 4460), "irb_and_squishable": (4494, 8912), "squishable": (294, 584)}


def grid_axes(lb, ub, res, variant="ceil"):
    """Per-axis sample coordinates of the SignedDistanceField.

    variant:
      "ceil"     n = ceil(rng/res), x_i = i*res + min, rng = (lb + (ub-lb)) - lb
                 (the GeometryTypes constructor);
      "round"    as "ceil" with n = round(rng/res);
      "floor"    as "ceil" with n = floor(rng/res);
      "linspace" n = ceil(rng/res), x_i = linspace(lb, ub, n+1) (endpoint-exact).
    """
    axes = []
    for lo, hi in zip(lb, ub):
        lo, hi = float(lo), float(hi)
        width = hi - lo
        rng = (lo + width) - lo
        q = rng / res
        n = {"ceil": math.ceil(q), "round": int(round(q)), "floor": math.floor(q),
             "linspace": math.ceil(q)}[variant]
        if variant == "linspace":
            axes.append(np.linspace(lo, lo + width, n + 1))
        else:
            axes.append(np.arange(n + 1, dtype=np.float64) * res + lo)
    return axes


def grid_points(axes):
    """(n,3) sample points, x fastest (Julia's column-major vol[x,y,z])."""
    z, y, x = np.meshgrid(axes[2], axes[1], axes[0], indexing="ij")
    return np.stack([x.ravel(), y.ravel(), z.ravel()], axis=1)


def to_volume(values, axes):
    """Values in grid_points order -> vol[x, y, z]."""
    return np.asarray(values).reshape(len(axes[2]), len(axes[1]), len(axes[0])).transpose(2, 1, 0)


def mesh_counts(inside):
    """(vertices, faces) of the marching-tetrahedra mesh of a boolean volume
    inside[x, y, z] (True where value < iso)."""
    b = np.asarray(inside, bool)
    nx, ny, nz = b.shape
    verts = 0
    for dx, dy, dz in EDGE_STEPS:
        a = b[:nx - dx, :ny - dy, :nz - dz]
        c = b[dx:, dy:, dz:]
        verts += int(np.count_nonzero(a != c))
    corner = [b[cx:nx - 1 + cx, cy:ny - 1 + cy, cz:nz - 1 + cz].astype(np.int8) for cx, cy, cz in CORNERS]
    faces = 0
    for t in TETS:
        k = corner[t[0]] + corner[t[1]] + corner[t[2]] + corner[t[3]]
        faces += int(np.count_nonzero((k == 1) | (k == 3))) + 2 * int(np.count_nonzero(k == 2))
    return verts, faces


def classify(values, iso, mode="shift"):
    """mode "shift": (f - iso) < 0 (contour_mesh samples f - iso, meshes level 0);
    mode "direct": f < iso."""
    values = np.asarray(values, np.float64)
    return (values - iso) < 0.0 if mode == "shift" else values < iso


def rbf_drawing_region(centres):
    """drawing_region(::InterpolatingSurface) (src/Flash.jl:270-275): the
    centres' bounding box widened by half its widths on every side."""
    c = np.asarray(centres, np.float64)
    lb, ub = c.min(axis=0), c.max(axis=0)
    w = ub - lb
    return lb - 0.5 * w, ub + 0.5 * w


def count_variants(sdf, lb, ub, iso, res, variants=("ceil", "round", "floor", "linspace"),
                   modes=("shift", "direct")):
    """{(variant, mode): (V, F, grid shape)} for an SDF callable on (n,3) arrays."""
    out = {}
    for v in variants:
        axes = grid_axes(lb, ub, res, v)
        vals = to_volume(sdf(grid_points(axes)), axes)
        for mode in modes:
            V, F = mesh_counts(classify(vals, iso, mode))
            out[(v, mode)] = (V, F, tuple(len(a) for a in axes))
    return out


def pinned_case(name):
    """(manipulator, x, lb, ub, iso, res) of a pinned notebook call; x is the
    full state vector [q; δ] (src/Flash.jl:97-104)."""
    from flash import Models
    from flash import rbf as host_rbf
    from flash.core import num_states
    if name == "irb140":
        m = Models.irb140()
        x = m.mechanism.zero_configuration()
    elif name == "irb_and_squishable":
        m, x = Models.irb_and_squishable()
    elif name == "squishable":
        m = Models.squishable()
        x = np.zeros(num_states(m))
        x[:m.mechanism.num_positions] = m.mechanism.zero_configuration()
    else:
        raise KeyError(name)
    if name in REGIONS:
        lb, ub, iso, res = REGIONS[name]
    else:
        nq = m.mechanism.num_positions
        centres = host_rbf.solve(m, m.mechanism.normalize(x[:nq]), x[nq:])[0].centres
        lb, ub = rbf_drawing_region(centres)
        iso, res = 0.0, 0.1
    return m, np.asarray(x, np.float64), lb, ub, iso, res
