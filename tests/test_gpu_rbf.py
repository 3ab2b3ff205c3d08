"""GPU: RBF skins (BASELINE configs 3 and 5) against the oracle golden vectors
and the reference KAT, through the C-ABI."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, rng

pytestmark = pytest.mark.gpu


def _scene(name):
    from flash import Models
    if name == "c3_beanbag":
        return Models.beanbag()
    return Models.irb_and_squishable()[0]


def _ctx(m, precision=64, cull=True, sort_points=False):
    from flash import _lib
    from flash.core import ConvexGeometry
    c = _lib.Context(device=0, precision=precision, cull=cull, sort_points=sort_points)
    c.set_surfaces([("hull", (s.hull.vertices, s.hull.faces, s.hull.planes)) if isinstance(s, ConvexGeometry)
                    else ("rbf", len(s.surface_points) + len(s.skeleton_points)) for s in m.surfaces])
    return c


def test_beanbag_kat_on_gpu():
    """test/runtests.jl:17 through Flash.skin(state) on the GPU."""
    import flash
    from flash import Models
    m = Models.beanbag()
    skin = flash.skin(flash.ManipulatorState(m))
    v = skin([100.0, 0.0, 0.0])
    assert v == pytest.approx(99.0, rel=2e-2)


@pytest.mark.parametrize("name", ["c3_beanbag", "c5_scene"])
@pytest.mark.parametrize("cull", [True, False])
def test_rbf_golden_parity(name, cull):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    m = _scene(name)
    c = _ctx(m, cull=cull)
    c.set_points(z["points"])
    c.set_rbf_params(z["rbf_rows"])
    cost, acc, (k, d, g) = c.eval(z["poses"], per_point=True)
    assert np.array_equal(k, z["kstar"])
    assert np.array_equal(d, z["d"]), np.abs(d - z["d"]).max()
    assert np.array_equal(g, z["grad"]), np.abs(g - z["grad"]).max()
    assert np.allclose(acc, z["accum"], rtol=1e-9, atol=1e-9 * np.abs(z["accum"]).max())
    # the chained gradient of the whole state (63 / 25 states)
    from flash import rbf as host_rbf
    from flash.gradientdescent import gradient_from_accum
    x = z["x"]
    nq = m.mechanism.num_positions
    solves = host_rbf.solve(m, m.mechanism.normalize(x[:nq]), x[nq:])
    gx = gradient_from_accum(m, x, acc, solves, 10)
    assert np.allclose(gx, z["dcdx"], rtol=1e-7, atol=1e-7 * np.abs(z["dcdx"]).max())
    c.close()


def test_rbf_fp32_beanbag():
    z = np.load(os.path.join(GOLDEN, "c3_beanbag.npz"))
    c = _ctx(_scene("c3_beanbag"), precision=32)
    c.set_points(z["points"])
    c.set_rbf_params(z["rbf_rows"])
    cost, acc, (k, d, g) = c.eval(z["poses"], per_point=True)
    assert np.abs(d - z["d"]).max() < 1e-4 * max(1.0, np.abs(z["d"]).max())
    assert cost == pytest.approx(z["accum"][0], rel=1e-4)
    c.close()


def test_rbf_requires_params():
    from flash import _lib
    c = _ctx(_scene("c3_beanbag"))
    c.set_points(np.zeros((10, 3)))
    with pytest.raises(_lib.FlashNativeError) as e:
        c.eval(np.zeros((1, 12)))
    assert e.value.status == 3
    c.close()


def test_tracking_deformable_beanbag():
    """estimate_state on the deformable beanbag (examples/deformable_manipulator
    .ipynb): the GPU cost/gradient drive the cost down."""
    import flash
    from flash import Models, rbf as host_rbf
    from flash.tracking import NaiveSolver, estimate_state
    from flash.gradientdescent import CostFunctor
    m = Models.beanbag()
    r = rng(11)
    nq = m.mechanism.num_positions
    x_true = np.zeros(flash.num_states(m))
    x_true[:nq] = m.mechanism.zero_configuration()
    x_true[4:7] = 2 * r.random(3) ** 3
    x_true[nq:] = 0.5 * (r.random(18) - 0.5)
    solves = host_rbf.solve(m, m.mechanism.normalize(x_true[:nq]), x_true[nq:])
    C = solves[0].centres
    # sensed points on the true skin: project random points along the gradient
    skin_true = flash.ManipulatorState(m)
    skin_true.q[:] = x_true[:nq]
    skin_true.deformation_data[:] = x_true[nq:]
    f = flash.skin(skin_true)
    pts = C.mean(0) + r.normal(size=(4000, 3))
    for _ in range(6):
        d, _, g = f.evaluate(pts)
        pts = pts - d[:, None] * g
    x0 = x_true.copy()
    x0[4:7] += 0.1
    cf = CostFunctor(m, pts)
    c0 = cf(x0)
    seen = []
    x = estimate_state(m, pts, x0, callback=lambda x, c: seen.append(c),
                       solver=NaiveSolver(len(x0), rate=0.05, max_step=0.05, iteration_limit=25))
    assert seen[-1] < 0.5 * c0


@pytest.mark.parametrize("precision", [64, 32])
def test_scheduled_passes_rbf_scene(precision):
    """Config 5's scene (hulls + RBF skin + table) in the RBF pass variant, f64
    and f32, sorted cloud: 20 repeated passes (scheduled from the second on,
    the order rebuilt at the 16th) are bit-identical to the first."""
    z = np.load(os.path.join(GOLDEN, "c5_scene.npz"))
    c = _ctx(_scene("c5_scene"), precision=precision, sort_points=True)
    pts = np.concatenate([z["points"]] * 40)  # > one block per wave-iteration round
    c.set_points(pts)
    c.set_rbf_params(z["rbf_rows"])
    first = c.eval(z["poses"], per_point=True)
    for it in range(20):
        cost, acc, pp = c.eval(z["poses"], per_point=True)
        assert cost == first[0] and np.array_equal(acc, first[1]), it
        for a, b in zip(pp, first[2]):
            assert np.array_equal(a, b), it
    if precision == 64:
        n0 = len(z["points"])
        assert np.array_equal(first[2][0][:n0], z["kstar"]) and np.array_equal(first[2][1][:n0], z["d"])
    c.close()


def test_manipulator_notebook_on_gpu(oracle_mod):
    """examples/manipulator.ipynb cells 2/6 through the product path (GPU
    raycast of the true state, GPU CostFunctor at the two printed
    configurations) == the CPU oracle; the divergence from the notebook's
    printed costs is the measured one (tests/test_notebook_pins.py)."""
    import flash
    from flash import Models
    from flash.depthsensors import Kinect, raycast
    from flash.gradientdescent import CostFunctor
    import test_notebook_pins as nb
    m = Models.two_link_arm(False)
    st = flash.ManipulatorState(m)
    st.set_configuration(nb.PINS["x_true"])
    pts = raycast(st, Kinect(nb.PINS["sensor"]["rows"], nb.PINS["sensor"]["cols"]), nb.camera())
    opts, ocosts = nb.oracle_notebook(oracle_mod)
    assert pts.shape == opts.shape == (nb.MEASURED_HITS, 3)
    assert np.allclose(pts, opts, rtol=0, atol=1e-12)
    cf = CostFunctor(m, pts)
    for pin, oc, ratio in zip(nb.PINS["pins"], ocosts, nb.MEASURED_RATIO):
        c = cf(np.asarray(pin["x"]))
        assert c == pytest.approx(oc, rel=1e-9)
        assert c / pin["cost"] == pytest.approx(ratio, rel=2e-3)


def test_async_rbf_rows_not_torn():
    """fsdf_set_rbf_params + fsdf_eval_device queued several times with
    different RBF rows and no host sync in between (ShardedCostFunctor's
    pattern): each pass sees its own rows (the pinned staging slot of a row set
    is reused only after its copy ran). Each accumulator == a synchronous
    fsdf_eval with the same rows, bit for bit."""
    import torch
    z = np.load(os.path.join(GOLDEN, "c5_scene.npz"))
    m = _scene("c5_scene")
    c = _ctx(m)
    c.set_points(np.concatenate([z["points"]] * 8))
    rows0 = z["rbf_rows"]
    variants = []
    for j in range(12):  # > the 8-slot ring
        r = rows0.copy()
        r[:-1, 3] *= 1.0 + 0.01 * j  # scale the weights: a different field per pass
        variants.append(r)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    c.set_stream(stream.cuda_stream)
    accs = [torch.zeros(c.accum_len, dtype=torch.float64, device=dev) for _ in variants]
    for r, a in zip(variants, accs):
        c.set_rbf_params(r)
        c.eval_device(z["poses"], a.data_ptr())
    torch.cuda.synchronize()
    got = [a.cpu().numpy() for a in accs]
    for j, r in enumerate(variants):
        c.set_rbf_params(r)
        _, want, _ = c.eval(z["poses"])
        assert np.array_equal(got[j], want), j
    assert not np.array_equal(got[0], got[-1])
    c.set_stream(None)
    c.close()


def test_c5_precision_sweep_vs_oracle():
    """BASELINE config 5 as SURVEY.md §8d defines it: 2^20 points — the
    reference's recorded squishable cloud (25,571 points) tiled and jittered to
    half of them, generator G on the scene's hulls for the rest — on the
    deformed irb_and_squishable scene (tools/precision_sweep.py), both
    precisions against the fp64 CPU oracle on ALL points. Tolerances: f64
    k*/d* exact (north-star bar: k* exact, 1e-6 rel); f32 bit-exact against
    the fp32 oracle on a 131,072-point sample; f32 vs f64: |Δd*| < 5e-5 m, k*
    flips on < 0.5 % of the points and only at near-ties (|Δd*| < 5e-5
    there), cost within 1e-4 rel, ∂c/∂x within 1e-2 rel of the f64 gradient.
    Reference: examples/irb_and_squishable.ipynb:329-331 (poses),
    src/depthdata.jl:19-30 (the cloud's format)."""
    import sys
    from conftest import ROOT
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import precision_sweep
    r = precision_sweep.sweep(1 << 20)
    assert r["points"] == 1 << 20
    f64, f32 = r["f64"], r["f32"]
    assert f64["max_abs_dd"] == 0.0 and f64["kstar_mismatch"] == 0
    assert f64["cost_rel_err"] < 1e-9
    ex = f32["f32_exact_sample"]
    assert ex["points"] == 1 << 17 and ex["kstar_equal"] and ex["d_equal"] and ex["grad_equal"], ex
    assert f32["max_abs_dd"] < 5e-5
    assert f32["kstar_mismatch_frac"] < 5e-3
    assert f32.get("max_abs_dd_at_mismatch", 0.0) < 5e-5
    assert f32["cost_rel_err"] < 1e-4
    assert f32["dcdx_rel_err_vs_f64"] < 1e-2
