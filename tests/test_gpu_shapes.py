"""GPU parity on model shapes the metric model does not exercise: more than 64
and more than 128 surfaces (the 2- and 4-slot accumulator variants), hulls with
fewer faces than one plane batch (tetrahedra), hulls far larger than the IRB140
links (multi-round LDS staging, > 64 KiB of LDS per workgroup), the LDS limit,
and RBF skins with more centres than one staging chunk. All against the C
oracle; fp64 results bit for bit, sums at 1e-9 relative."""
import numpy as np
import pytest

from conftest import rng

pytestmark = pytest.mark.gpu


def _random_hull(r, n, scale=0.05):
    from flash import _lib
    v, f, p = _lib.convex_hull(r.normal(size=(n, 3)) * scale * r.uniform(0.5, 1.5, size=3))
    return v, f, p


def _sphere_hull(n, radius=0.1):
    from flash import _lib
    i = np.arange(n) + 0.5
    phi = np.arccos(1 - 2 * i / n)
    th = np.pi * (1 + 5 ** 0.5) * i
    pts = radius * np.stack([np.cos(th) * np.sin(phi), np.sin(th) * np.sin(phi), np.cos(phi)], 1)
    return _lib.convex_hull(pts)


def _poses(r, K, spread=1.0):
    P = np.zeros((K, 12))
    for k in range(K):
        q = r.normal(size=4)
        q /= np.linalg.norm(q)
        w, x, y, z = q
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                      [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                      [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
        P[k, :9] = R.reshape(-1)
        P[k, 9:] = r.uniform(-spread, spread, size=3)
    return P


def _cloud(r, poses, n, spread=0.15):
    """points around random hull centres (inside, near and far)."""
    c = poses[r.integers(0, len(poses), n), 9:]
    return c + r.normal(size=(n, 3)) * spread


def _parity(hulls, poses, pts, oracle_mod, precision=64, cull=True, sort_points=False):
    from flash import _lib
    om = oracle_mod.OracleModel(hulls)
    od, ok, og = om.skin(poses, pts)
    oacc = om.cost_accum(poses, pts)
    c = _lib.Context(device=0, precision=precision, cull=cull, sort_points=sort_points)
    try:
        c.set_model(hulls)
        c.set_points(pts)
        cost, acc, (k, d, g) = c.eval(poses, per_point=True)
    finally:
        c.close()
    assert np.array_equal(k, ok), np.nonzero(k != ok)[0][:10]
    if precision == 64:
        assert np.array_equal(d, od), np.abs(d - od).max()
        assert np.array_equal(g, og), np.abs(g - og).max()
        assert np.allclose(acc, oacc, rtol=1e-9, atol=1e-9 * max(1.0, np.abs(oacc).max()))
    else:
        assert np.abs(d - od).max() < 2e-5
    return k


@pytest.mark.parametrize("K", [64, 65, 100, 200])
@pytest.mark.parametrize("cull", [True, False])
def test_many_surfaces_slot_variants(K, cull, oracle_mod):
    """K > 64 selects 2 accumulator slots per lane, K > 128 four (up to 256);
    K <= 64 poses ride in the pose kernel's arguments, K = 65 takes the copy."""
    r = rng(700 + K)
    hulls = [_random_hull(r, int(r.integers(8, 40))) for _ in range(K)]
    poses = _poses(r, K, spread=0.6)
    pts = _cloud(r, poses, 6000, spread=0.08)
    k = _parity(hulls, poses, pts, oracle_mod, cull=cull)
    if K > 64:
        assert k.max() >= 64  # slots beyond the first are exercised


def test_tetrahedra_and_boxes(oracle_mod):
    """4-face hulls (fewer faces than one plane batch) next to 12-face boxes."""
    from flash import _lib
    r = rng(711)
    tet = _lib.convex_hull(np.array([[0, 0, 0], [0.1, 0, 0], [0, 0.1, 0], [0, 0, 0.1]], np.float64))
    box = _lib.convex_hull(np.array([[x, y, z] for x in (-.05, .05) for y in (-.03, .03) for z in (-.02, .02)]))
    assert len(tet[1]) == 4 and len(box[1]) == 12
    hulls = [tet, box] * 6
    poses = _poses(r, len(hulls), spread=0.3)
    pts = _cloud(r, poses, 5000, spread=0.06)
    for cull in (True, False):
        _parity(hulls, poses, pts, oracle_mod, cull=cull)


@pytest.mark.parametrize("precision", [64, 32])
def test_large_hulls(precision, oracle_mod):
    """~500-face hulls: the per-wave stage needs several bulk-copy rounds and the
    workgroup more than 64 KiB of LDS (f64: ~140 KiB, one workgroup per CU)."""
    r = rng(712)
    big = _sphere_hull(250)
    assert len(big[1]) >= 490
    hulls = [big, _random_hull(r, 30), big]
    poses = _poses(r, 3, spread=0.25)
    pts = _cloud(r, poses, 4000, spread=0.12)
    _parity(hulls, poses, pts, oracle_mod, precision=precision)


def test_hull_beyond_lds_is_rejected():
    """A hull whose stage cannot fit the 160 KiB a workgroup may declare is an
    argument error at set_model, not a launch failure."""
    from flash import _lib
    huge = _sphere_hull(3000)
    c = _lib.Context(device=0)
    try:
        with pytest.raises(_lib.FlashNativeError) as e:
            c.set_model([huge])
        assert e.value.status == 1 and "LDS" in str(e.value)
        c.set_model([_sphere_hull(40)])  # the context stays usable
        c.set_points(np.zeros((1, 3)))
        cost, acc, _ = c.eval(np.array([[1, 0, 0, 0, 1, 0, 0, 0, 1, 0.5, 0, 0]], np.float64))
        assert cost > 0
    finally:
        c.close()


def test_rbf_skin_with_many_centres(oracle_mod):
    """An RBF skin of 121 centres (rows staged in two chunks of the 64-row stage;
    the adjoint block 4n+4 = 488 of the 512 per-wave accumulators) next to a hull."""
    import rbf as orbf  # oracle/rbf.py (numpy restatement)
    from flash import _lib
    r = rng(713)
    n_s = 120
    i = np.arange(n_s) + 0.5
    phi = np.arccos(1 - 2 * i / n_s)
    th = np.pi * (1 + 5 ** 0.5) * i
    surf = 0.2 * np.stack([np.cos(th) * np.sin(phi), 0.8 * np.sin(th) * np.sin(phi), 0.6 * np.cos(phi)], 1)
    centres = np.vstack([surf, [[0.0, 0.0, 0.0]]])
    values = np.concatenate([np.zeros(n_s), [-1.0]])
    u, _ = orbf.fit(centres, values)
    rows = np.vstack([np.hstack([centres, u[:len(centres), None]]), u[len(centres):][None]])
    hull = _random_hull(r, 20)
    ident = np.eye(3).reshape(-1)
    poses = np.array([np.concatenate([ident, [0.0, 0.0, 0.0]]), np.concatenate([ident, [0.35, 0.0, 0.0]])])
    pts = r.normal(size=(3000, 3)) * 0.25
    om = oracle_mod.OracleModel([hull], [("rbf", len(centres)), ("hull", 0)])
    od, ok, og = om.skin(poses, pts, rbf_rows=rows)
    oacc = om.cost_accum(poses, pts, rbf_rows=rows)
    assert (ok == 0).any() and (ok == 1).any()
    for cull in (True, False):
        c = _lib.Context(device=0, cull=cull)
        try:
            c.set_surfaces([("rbf", len(centres)), ("hull", hull)])
            c.set_rbf_params(rows)
            c.set_points(pts)
            cost, acc, (k, d, g) = c.eval(poses, per_point=True)
        finally:
            c.close()
        assert np.array_equal(k, ok)
        assert np.array_equal(d, od), np.abs(d - od).max()
        assert np.array_equal(g, og), np.abs(g - og).max()
        assert np.allclose(acc, oacc, rtol=1e-9, atol=1e-9 * np.abs(oacc).max())


def test_cone_fallback_paths(oracle_mod):
    """An apex of valence 48 (the descent walk's fan test stops at 32 faces, so
    those lanes take the exhaustive scan) over a coplanar triangulated base (fp32
    screen near-ties across batches -> the full fp64 scan): bit for bit vs the
    oracle, and the kernel counters show both fallbacks ran."""
    from flash import _lib
    from test_oracle import _cone_cloud, _cone_hull
    hull = _cone_hull()
    r = rng(714)
    poses = np.array([[1.0, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0], [1.0, 0, 0, 0, 1, 0, 0, 0, 1, 0.4, 0, 0]])
    pts = np.vstack([_cone_cloud(r, 3000), _cone_cloud(r, 3000) + [0.4, 0, 0]])
    _parity([hull, hull], poses, pts, oracle_mod)
    c = _lib.Context(device=0)
    try:
        c.set_model([hull, hull])
        c.set_points(pts)
        c.kernel_stats(True)
        c.eval(poses)
        st = c.kernel_stats(False)
    finally:
        c.close()
    assert st["full_scan_lanes"] > 0 and st["screen_fallbacks"] > 0 and st["walk_steps"] > 0, st


@pytest.mark.parametrize("precision", [64, 32])
def test_needles_oriented_box_culling(precision, oracle_mod):
    """Thin rods at random orientations, packed so that their bounding spheres
    overlap everywhere: the oriented-box lower bound does the culling. Some
    rods have body frames far from their vertices (box centre offset 3 m in
    the body frame, undone by the pose) and one sits 50 m from the origin:
    the f32 box transform and its margins at large coordinates. Culled and
    sorted results equal the oracle's brute force."""
    from flash import _lib
    r = rng(733)
    K = 24
    hulls, offs = [], []
    for k in range(K):
        off = np.array([3.0, -2.0, 1.0]) if k % 3 == 0 else np.zeros(3)
        ax = r.normal(size=(30, 3)) * np.array([0.2, 0.006, 0.004]) + off
        hulls.append(_lib.convex_hull(ax))
        offs.append(off)
    poses = _poses(r, K, spread=0.12)
    for k in range(K):
        R = poses[k, :9].reshape(3, 3)
        poses[k, 9:] -= R @ offs[k]
    poses[K - 1, 9:] += np.array([50.0, 0.0, 0.0])
    # points along the rods' world axes (surface, inside, near) plus a haze
    n = 8000
    kk = r.integers(0, K, n)
    t = r.uniform(-0.25, 0.25, n)
    axis = poses[kk][:, [0, 3, 6]]
    centre = poses[kk, 9:] + np.einsum("nij,nj->ni", poses[kk, :9].reshape(n, 3, 3), np.asarray(offs)[kk])
    pts = centre + axis * t[:, None] + r.normal(size=(n, 3)) * 0.01
    pts[: n // 8] = r.uniform(-0.3, 0.3, size=(n // 8, 3))
    for sort_points in (False, True):
        k = _parity(hulls, poses, pts, oracle_mod, precision=precision, cull=True, sort_points=sort_points)
    assert len(np.unique(k)) == K
