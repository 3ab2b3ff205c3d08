"""The reference notebook's own per-trial (err, cost) traces
(examples/manipulator.ipynb cells 9, 10, 14; fixture made by
tests/golden/make_manipulator_traces.py) against this repo's RBF landscape and
NaiveSolver. CPU side: the landscape is the C oracle's (test infrastructure);
the GPU twin runs the product path (tests/test_gpu_traces.py).

What the traces pin, and how:

* the solver's update rule, independently of the landscape. In a trajectory's
  late linear phase err_{k+1}/err_k = 1 − 2κa with a = cost_k/err_k² read off
  the SAME trajectory, so κ = (1 − ρ)/(2a) is the step per unit gradient. The
  notebook gives κ = 0.0986 (close, rate 0.1) and 0.0508 (far, rate 0.05):
  the step is rate·∇c on the UNDIVIDED cost — the notebook's session predates
  or bypasses src/tracking.jl:20's c/N (κ would be rate/58 ≈ 0.0017). The far
  set's largest per-step |Δerr| is 0.2828 = 0.2·√2 with max_step 0.2: the
  clip is component-wise (a norm clip caps |Δx|, hence |Δerr|, at 0.2). One
  callback per iteration (≤ 30 points per trial, iteration_limit 30).
* the landscape, through the start points: x0 is uniform on the torus (far)
  or the ±0.5 square (close), so given err0 the start lies uniformly on a
  circle and u = P_θ[c ≤ cost0] is Uniform(0,1) under the true landscape.
  This repo's f/|∇f| over r³ + affine gives KS distances 0.32 / 0.31 from
  uniform (5 % critical value 0.136 for 100 trials): REJECTED — the measured
  divergence already seen at the two printed costs (test_notebook_pins.py).
  The notebook's costs sit mostly low in our circle distributions (its cost
  is ~½ ours near the truth, and its far-field local minima — cost 9.68 at
  err 3.05-3.08, 1.09 at err 2.645 — are not ours). None of the 55 candidate
  formulations passes both (tools/rbf_trace_rescore.py,
  profiles/r03/rbf_trace_rescore.txt).
"""
import json
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN

TR = json.load(open(os.path.join(GOLDEN, "manipulator_traces.json")))
X_TRUE = np.array(TR["x_true"])
KS_5PCT_100 = 0.136
# measured on this repo's formulation (oracle == GPU); a change means the RBF
# landscape moved and DESIGN.md §2 must be revisited
MEASURED_KS = {"far": 0.32, "close": 0.31}


def angle_err(x):
    """norm(angle_diff.(x, x_true)) (cell 5: mod(φ2 − φ1 + π, 2π) − π)."""
    d = np.mod(X_TRUE - np.asarray(x) + math.pi, 2 * math.pi) - math.pi
    return float(np.linalg.norm(d))


def kappa_estimates(trials, rate, exact=False):
    """Single-trajectory κ estimates (step = κ·∇c) from the late linear phase.
    The windows keep cost above ~10 plot-resolution steps; `exact` traces (our
    own, unrounded) use the quadratic regime err < 0.1 instead."""
    lo, hi, cmin, emax = (0.8, 0.95, 0.012, 0.3) if rate >= 0.1 else (0.85, 0.99, 0.1, 0.5)
    if exact:
        lo, hi, cmin, emax = 0.5, 0.999, 0.0, 0.1
    out = []
    for e, c in trials:
        e, c = np.asarray(e), np.asarray(c)
        for k in range(3, len(e) - 1):
            if c[k] >= cmin and e[k] < emax and lo < e[k + 1] / e[k] < hi and lo < e[k] / e[k - 1] < hi:
                out.append((1 - e[k + 1] / e[k]) / (2 * c[k] / e[k] ** 2))
    return np.array(out)


def ks_uniform(u):
    u = np.sort(np.asarray(u))
    i = np.arange(1, len(u) + 1)
    return float(max(np.max(i / len(u) - u), np.max(u - (i - 1) / len(u))))


# ---------------------------------------------------------------- the fixture


def test_fixture_structure():
    for kind, n_ok in (("far", 93), ("close", 190 // 2)):
        trials = TR[kind]["trials"]
        assert len(trials) == 100
        assert [t["trial"] for t in trials] == list(range(1, 101))
        lens = [len(t["err"]) for t in trials]
        assert all(1 <= n <= 30 for n in lens) and all(len(t["cost"]) == len(t["err"]) for t in trials)
        assert sum(n == 30 for n in lens) >= n_ok
        assert all(v >= -TR[kind]["resolution"]["err"] for t in trials for v in t["err"])
    # x0 ranges: far starts within the torus (err ≤ π√2), close within ±0.5 (err ≤ 0.5√2)
    assert max(t["err"][0] for t in TR["far"]["trials"]) <= math.pi * math.sqrt(2)
    assert max(t["err"][0] for t in TR["close"]["trials"]) <= 0.5 * math.sqrt(2) + 1e-3


def test_fixture_pixel_round_trip():
    """Every stored value maps back to a 0.01-mm SVG coordinate (the plots
    print two decimals) — the extraction is exact up to the print step."""
    for kind in ("far", "close"):
        for t in TR[kind]["trials"]:
            for key in ("err", "cost"):
                step = 2 * TR[kind]["resolution"][key]  # data units per 0.01 mm
                for v in t[key]:
                    k = v / step
                    assert abs(k - round(k)) < 0.01, (kind, key, v)
    # the notebook's own printed cost at the far local minimum (cell 11) lies on the plotted plateau
    finals = [t["cost"][-1] for t in TR["far"]["trials"]]
    assert any(abs(c - 9.7189) < 0.05 for c in finals)


# ------------------------------------------------ the solver rule (no landscape)


def test_step_rule_is_rate_times_gradient_of_undivided_cost():
    for kind in ("far", "close"):
        s = TR[kind]["solver"]
        k = kappa_estimates([(t["err"], t["cost"]) for t in TR[kind]["trials"]], s["rate"])
        assert len(k) >= 50
        assert np.median(k) == pytest.approx(s["rate"], rel=0.05), (kind, np.median(k))


def test_clip_is_componentwise():
    s = TR["far"]["solver"]
    res = TR["far"]["resolution"]["err"]
    steps = np.concatenate([np.abs(np.diff(t["err"])) for t in TR["far"]["trials"]])
    # a norm clip would bound |Δx| (and so |Δerr|) by max_step; the traces exceed it
    assert (steps > s["max_step"] + 4 * res).sum() > 100
    # component-wise: |Δx| ≤ max_step·√2, reached when both components clip
    assert steps.max() <= s["max_step"] * math.sqrt(2) + 4 * res
    assert (np.abs(steps - s["max_step"] * math.sqrt(2)) < 4 * res).sum() >= 10


# ----------------------------------------------- this repo's landscape (oracle)


def oracle_landscape(oracle_mod):
    """(cost(x), value_and_gradient(x), N) of the notebook scene on the C oracle:
    the sensed cloud raycast at x_true, cost undivided (the callback's c)."""
    import test_notebook_pins as P
    from flash import Models
    from flash import rbf as host_rbf
    from flash.gradientdescent import gradient_from_accum
    pts, _ = P.oracle_notebook(oracle_mod)
    m = Models.two_link_arm(False)
    om = oracle_mod.OracleModel.from_manipulator(m)

    def acc(x):
        q = m.mechanism.normalize(np.asarray(x, np.float64))
        from flash.core import surface_poses
        solves = host_rbf.solve(m, q, np.zeros(0))
        return om.cost_accum(surface_poses(m, q), pts, rbf_rows=host_rbf.rows(solves)), solves

    def cost(x):
        return float(acc(x)[0][0])

    def value_and_gradient(x):
        a, solves = acc(x)
        return float(a[0]), gradient_from_accum(m, np.asarray(x, np.float64), a, solves, 10.0)
    return cost, value_and_gradient, len(pts)


@pytest.fixture(scope="module")
def landscape(oracle_mod):
    return oracle_landscape(oracle_mod)


def run_notebook_trial(value_and_gradient, x0, solver_kw):
    """The cell's estimate_state with the notebook session's objective (c, not
    c/N — pinned above) and its callback recording (err, cost)."""
    from flash.tracking import NaiveSolver
    errs, costs = [], []

    def wrapped(x):
        c, g = value_and_gradient(x)
        errs.append(angle_err(x))
        costs.append(c)
        return c, g
    NaiveSolver(2, **solver_kw).optimize(wrapped, x0)
    return errs, costs


def test_gradient_matches_finite_differences(landscape):
    cost, vg, _ = landscape
    for x in ([6.66999, 0.0956194], [3.3, 1.0], [0.5, -2.0]):
        x = np.asarray(x)
        _, g = vg(x)
        h = 1e-6
        fd = [(cost(x + h * e) - cost(x - h * e)) / (2 * h) for e in np.eye(2)]
        assert np.allclose(g, fd, rtol=1e-5, atol=1e-6), (x, g, fd)


def _rounded(v, res):
    step = 2 * res  # one 0.01-mm print step in data units
    return [round(x / step) * step for x in v]


@pytest.mark.parametrize("kind", ["far", "close"])
def test_solver_reproduces_the_traces_step_signatures(kind):
    """Our NaiveSolver (flash.tracking; fsdf_descend is bit-identical to it,
    tests/test_gpu_tracking.py) run with the cell's kwargs on a quadratic
    valley shaped like the notebook's near-truth landscape (a_s = 0.5, a_f = 4,
    both read off the close traces) and rounded to the plots' resolution gives
    back the traces' landscape-free signatures: κ = rate on the undivided cost,
    and (far) the component-wise clip's max |Δerr| = max_step·√2. A norm clip
    or the c/N objective fails them (negative controls)."""
    from flash.tracking import NaiveSolver
    R = np.array([[math.cos(0.4), -math.sin(0.4)], [math.sin(0.4), math.cos(0.4)]])
    A = R @ np.diag([0.5, 4.0]) @ R.T

    def vg(x):
        d = np.asarray(x) - X_TRUE
        return float(d @ A @ d), 2 * A @ d

    kw = {k: TR[kind]["solver"][k] for k in ("rate", "max_step", "iteration_limit")}
    res = TR[kind]["resolution"]
    r = np.random.Generator(np.random.PCG64(20261017))
    spread = 2 * math.pi if kind == "far" else 1.0

    def traces(solver_cls, scale=1.0):
        out = []
        for _ in range(100):
            e, c = [], []

            def wrapped(x):
                f, g = vg(x)
                e.append(angle_err(x))
                c.append(f)
                return f * scale, g * scale
            solver_cls(2, **kw).optimize(wrapped, X_TRUE + spread * (r.random(2) - 0.5))
            out.append((_rounded(e, res["err"]), _rounded(c, res["cost"])))
        return out

    def signatures(tr):
        k = kappa_estimates(tr, kw["rate"])
        steps = np.concatenate([np.abs(np.diff(e)) for e, _ in tr])
        return (np.median(k) if len(k) else float("nan")), steps.max(), len(k)

    ours = traces(NaiveSolver)  # default tolerance (1e-3), like the cells
    kappa, smax, n = signatures(ours)
    assert n >= 30
    assert kappa == pytest.approx(kw["rate"], rel=0.05)
    assert smax <= kw["max_step"] * math.sqrt(2) + 4 * res["err"]
    if kind == "far":
        assert smax == pytest.approx(kw["max_step"] * math.sqrt(2), abs=4 * res["err"])

        class NormClip(NaiveSolver):
            def optimize(self, f, x0):
                x = np.array(x0, np.float64)
                for _ in range(self.iteration_limit):
                    _, g = f(x)
                    s = -self.rate * g
                    n_ = np.linalg.norm(s)
                    x = x + (s * (self.max_step / n_) if n_ > self.max_step else s)
                return x, None
        assert signatures(traces(NormClip))[1] <= kw["max_step"] + 4 * res["err"]
    # the c/N objective (N = 58 sensed points) steps 58x shorter: κ = rate/58
    kappa_n, _, _ = signatures(traces(NaiveSolver, scale=1 / 58))
    assert not (abs(kappa_n / kw["rate"] - 1) < 0.5)


def test_default_tolerance_stops_like_the_notebook():
    """The notebook's trials stop early (7 far, 5 close of 100) although the
    cells pass no tolerance: NaiveSolver's default gradient_convergence_tolerance
    is positive. The close trials' stopping points bound it: they stop at
    err 5e-4…1.8e-3 where |∇c| ≈ 2·a_s·δ with a_s ≤ 0.5, while trials at
    err 1.0e-3 run on — so tol ∈ [~2.5e-4, ~2.5e-3]; 1e-3 is adopted
    (estimated, not pinned exactly)."""
    from flash.tracking import NaiveSolver
    assert NaiveSolver(2).gradient_convergence_tolerance == 1e-3
    short = {k: sum(len(t["err"]) < 30 for t in TR[k]["trials"]) for k in ("far", "close")}
    assert short == {"far": 7, "close": 5}
    stops = [t["err"][-1] for t in TR["close"]["trials"] if len(t["err"]) < 30]
    assert max(stops) < 2.5e-3 and min(stops) > 2.5e-4


def _pit(cost, kind, m=36):
    out = []
    th = np.linspace(0.0, 2 * math.pi, m, endpoint=False)
    res = TR[kind]["resolution"]["cost"]
    for t in TR[kind]["trials"]:
        e0, c0 = t["err"][0], t["cost"][0]
        d = e0 * np.stack([np.cos(th), np.sin(th)], -1)
        if kind == "close":
            inside = np.all(np.abs(d) <= 0.5, axis=1)
            d = d[inside] if inside.any() else d
        cs = np.array([cost(X_TRUE + di) for di in d])
        out.append((np.sum(cs < c0 - res) + 0.5 * np.sum(np.abs(cs - c0) <= res)) / len(cs))
    return np.array(out)


@pytest.fixture(scope="module")
def pit_values(landscape):
    cost = landscape[0]
    return {kind: _pit(cost, kind) for kind in ("far", "close")}


def test_landscape_divergence_is_the_measured_one(pit_values):
    """Test (a): the start-point PIT against Uniform(0,1). Pinned at the measured
    KS distances (documented divergence); the notebook's costs lie low in our
    circle distributions."""
    for kind, u in pit_values.items():
        ks = ks_uniform(u)
        assert ks == pytest.approx(MEASURED_KS[kind], abs=0.03), (kind, ks)
        assert np.median(u) < 0.4, kind


@pytest.mark.xfail(strict=True, reason="RBF landscape divergence: the start-point PIT of the notebook traces "
                                       "rejects f/|grad f| over r^3+affine (KS 0.32 / 0.31 > 0.136); DESIGN.md §2")
def test_landscape_matches_the_notebook_traces(pit_values):
    for kind, u in pit_values.items():
        assert ks_uniform(u) < KS_5PCT_100, kind


def _reproduce(cost, vg, trial, kind, m=72):
    """Test (b) for one trial: does a start on its err0 circle with cost0
    reproduce every (err, cost) point? Returns the best max error in units of
    the plot resolution."""
    e0, c0 = trial["err"][0], trial["cost"][0]
    th = np.linspace(0.0, 2 * math.pi, m, endpoint=False)
    dirs = np.stack([np.cos(th), np.sin(th)], -1)
    cs = np.array([cost(X_TRUE + e0 * d) for d in dirs]) - c0
    kw = {k: TR[kind]["solver"][k] for k in ("rate", "max_step", "iteration_limit")}
    best = math.inf
    for i in np.nonzero(np.sign(cs) != np.sign(np.roll(cs, -1)))[0]:
        a, b = th[i], th[(i + 1) % m] + (2 * math.pi if i == m - 1 else 0)
        for _ in range(30):  # bisection on the circle for cost = cost0
            mid = 0.5 * (a + b)
            v = cost(X_TRUE + e0 * np.array([math.cos(mid), math.sin(mid)])) - c0
            a, b = (mid, b) if np.sign(v) == np.sign(cs[i]) else (a, mid)
        x0 = X_TRUE + e0 * np.array([math.cos(a), math.sin(a)])
        e, c = run_notebook_trial(vg, x0, kw)
        n = len(trial["err"])
        if len(e) != n:  # stopped at another iteration: not a reproduction
            continue
        de = np.max(np.abs(np.array(e[:n]) - trial["err"])) / TR[kind]["resolution"]["err"]
        dc = np.max(np.abs(np.array(c[:n]) - trial["cost"])) / TR[kind]["resolution"]["cost"]
        best = min(best, max(de, dc))
    return best


@pytest.mark.xfail(strict=True, reason="RBF landscape divergence (see test (a)): no start on the err0 circle "
                                       "reproduces the notebook trials' 30-point (err, cost) traces")
def test_solver_reproduces_the_notebook_trials(landscape):
    cost, vg, _ = landscape
    ok = 0
    picks = [("far", i) for i in range(0, 100, 20)] + [("close", i) for i in range(0, 100, 20)]
    for kind, i in picks:
        ok += _reproduce(cost, vg, TR[kind]["trials"][i], kind) <= 20.0
    assert ok >= 8, ok
