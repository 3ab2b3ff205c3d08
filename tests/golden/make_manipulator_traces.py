#!/usr/bin/env python3
"""Extract the per-trial (iteration, err, cost) traces that the reference's own
notebook plots, as a small JSON fixture (tests/golden/manipulator_traces.json).

Source: /root/reference/examples/manipulator.ipynb (read as data; run here only,
the reference never travels). Every trial is a Gadfly `Geom.line` layer, drawn
as one SVG `<path d="M x,y L x y ...">` polyline with one vertex per callback
call (src/tracking.jl:19 fires the callback once per cost evaluation; the
notebook's callback pushes err and the undivided cost, cells 7 / 13):

  * cell 9  (exec 104) `trials`: err vs iteration, 100 random starts within
    ±π of [π, 1.3] (cell 7: x0 = x_true + 2π(rand − 0.5)), solver
    NaiveSolver(2, rate=0.05, max_step=0.2, iteration_limit=30)
  * cell 10 (exec 105) the same trials' cost
  * cell 14 (exec 108) `trials_close`: err (upper panel) and cost (lower
    panel), 100 starts within ±0.5 rad (cell 13: x0 = x_true + rand − 0.5),
    the DEFAULT solver NaiveSolver(2, rate=0.1, max_step=0.5,
    iteration_limit=30) (src/tracking.jl:12-15)

Execution order (execution counts): reload("Flash") 88, model + sensor 89,
true state / sensed_points 93, trials 103, plots 104-105, trials_close 107,
plots 108 — so both trial sets use the same sensed cloud and the reloaded
package.

Pixel → data: each axis is mapped through two of its tick labels (the
`guide xlabels` / `guide ylabels` text positions, which Gadfly places at the
exact tick coordinates). Coordinates are printed with 2 decimals (mm), so the
resolution is 0.005 mm ÷ (mm per unit), stored per panel.

Trial identity: layer i gets color i (a continuous 1…100 color key); the SVG
lists the layers in reverse order (its first stroke color is the key's top,
trial 100). The err and cost plots of one trial set list identical color
sequences, so polylines pair by position; we store trials in 1…100 order.

    python tests/golden/make_manipulator_traces.py [--notebook PATH] [--out PATH]
"""
from __future__ import annotations

import argparse
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
NOTEBOOK = "/root/reference/examples/manipulator.ipynb"

PATH_RE = re.compile(r'class="geometry color_"[^>]*stroke="(#[0-9A-Fa-f]{6})"[^>]*>\s*<path fill="none" d="([^"]*)"')
PANEL_RE = re.compile(r'class="plotpanel"')
LABELS_RE = re.compile(r'class="guide (xlabels|ylabels)"(.*?)</g>', re.S)
TEXT_RE = re.compile(r'<text x="(-?[\d.]+)" y="(-?[\d.]+)"[^>]*>([^<]*)<')


def svg_of(nb, cell):
    for o in nb["cells"][cell]["outputs"]:
        if "data" in o and "image/svg+xml" in o["data"]:
            return "".join(o["data"]["image/svg+xml"])
    raise ValueError(f"cell {cell} has no SVG output")


def axes(svg):
    """[(xlabels, ylabels)] per panel in document order; each a list of
    (pixel, value)."""
    groups = [(m.group(1), [(float(x), float(y), float(t)) for x, y, t in TEXT_RE.findall(m.group(2))])
              for m in LABELS_RE.finditer(svg)]
    xs = [[(x, v) for x, _, v in g] for k, g in groups if k == "xlabels"]
    ys = [[(y, v) for _, y, v in g] for k, g in groups if k == "ylabels"]
    return xs, ys


def affine(ticks):
    """pixel → value through the first and last tick (checked on the rest)."""
    (p0, v0), (p1, v1) = ticks[0], ticks[-1]
    scale = (v1 - v0) / (p1 - p0)
    for p, v in ticks:
        assert abs(v0 + (p - p0) * scale - v) < 2e-3 * abs(v1 - v0), (ticks, p, v)
    return (lambda p: v0 + (p - p0) * scale), abs(scale)


def polylines(svg_part):
    out = []
    for color, d in PATH_RE.findall(svg_part):
        nums = [float(v) for v in re.findall(r"-?\d+(?:\.\d+)?", d)]
        out.append((color, list(zip(nums[0::2], nums[1::2]))))
    return out


def panel_series(svg_part, xmap, ymap):
    """Per trial (1…100 order): [(iteration, value)]."""
    lines = polylines(svg_part)
    series = []
    for color, pts in reversed(lines):
        its = [xmap(px) for px, _ in pts]
        assert all(abs(it - round(it)) < 0.01 for it in its), its
        series.append((color, [(int(round(it)), ymap(py)) for (px, py), it in zip(pts, its)]))
    return series


def split_panels(svg):
    """The SVG text of each plotpanel (a vstack has two)."""
    starts = [m.start() for m in PANEL_RE.finditer(svg)] + [len(svg)]
    return [svg[a:b] for a, b in zip(starts[:-1], starts[1:])]


def trial_set(err_part, err_axes, cost_part, cost_axes):
    ex, exres = affine(err_axes[0])
    ey, eyres = affine(err_axes[1])
    cx, _ = affine(cost_axes[0])
    cy, cyres = affine(cost_axes[1])
    e = panel_series(err_part, ex, ey)
    c = panel_series(cost_part, cx, cy)
    assert len(e) == len(c) == 100
    trials = []
    for i, ((ce, se), (cc, sc)) in enumerate(zip(e, c)):
        assert ce == cc, (i, ce, cc)
        assert [it for it, _ in se] == [it for it, _ in sc] == list(range(1, len(se) + 1))
        trials.append({"trial": i + 1, "color": ce,
                       "err": [round(v, 6) for _, v in se], "cost": [round(v, 6) for _, v in sc]})
    # resolution: half of the 0.01 mm print step, in data units
    return trials, {"err": 0.005 * eyres, "cost": 0.005 * cyres}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--notebook", default=NOTEBOOK)
    ap.add_argument("--out", default=os.path.join(HERE, "manipulator_traces.json"))
    a = ap.parse_args()
    nb = json.load(open(a.notebook))

    # cells 9 / 10: one panel each
    s9, s10 = svg_of(nb, 9), svg_of(nb, 10)
    (x9,), (y9,) = axes(s9)
    (x10,), (y10,) = axes(s10)
    far, far_res = trial_set(s9, (x9, y9), s10, (x10, y10))

    # cell 14: vstack(err plot, cost plot). Label groups come panel by panel
    # in reverse drawing order; match each panel to its axes by y range.
    s14 = svg_of(nb, 14)
    xs, ys = axes(s14)
    parts = split_panels(s14)
    assert len(parts) == 2 and len(xs) == 2 and len(ys) == 2
    # the err panel is the upper one (smaller pixel y), the cost panel the lower
    by_top = sorted(range(2), key=lambda k: min(p for p, _ in ys[k]))
    err_k, cost_k = by_top
    assert max(v for _, v in ys[err_k]) < 1.0 < max(v for _, v in ys[cost_k])
    # panel text order: the panel whose paths lie in the upper half is the err panel
    def mean_y(part):
        pts = [p for _, ln in polylines(part) for p in ln]
        return sum(y for _, y in pts) / len(pts)
    err_part, cost_part = sorted(parts, key=mean_y)
    close, close_res = trial_set(err_part, (xs[err_k], ys[err_k]), cost_part, (xs[cost_k], ys[cost_k]))

    out = {
        "_source": ("Per-trial polylines of the reference's own plots in examples/manipulator.ipynb "
                    "(data read from the notebook's SVG outputs by tests/golden/make_manipulator_traces.py). "
                    "err = norm(angle_diff.(x, x_true)), cost = the undivided cost the tracking callback "
                    "receives (src/tracking.jl:19), one entry per callback call."),
        "x_true": [3.141592653589793, 1.3],
        "angle_diff": "mod(phi2 - phi1 + pi, 2pi) - pi with (phi1, phi2) = (x, x_true) (cell 5)",
        "far": {"where": "examples/manipulator.ipynb cells 7-10 (plots at :276 err, :2864 cost)",
                "start": "x_true + 2*pi*(rand(2) - 0.5)",
                "solver": {"rate": 0.05, "max_step": 0.2, "iteration_limit": 30},
                "resolution": far_res, "trials": far},
        "close": {"where": "examples/manipulator.ipynb cells 13-14 (plot at :7408)",
                  "start": "x_true + (rand(2) - 0.5)",
                  "solver": {"rate": 0.1, "max_step": 0.5, "iteration_limit": 30, "note": "default, src/tracking.jl:12-15"},
                  "resolution": close_res, "trials": close},
    }
    with open(a.out, "w") as f:
        json.dump(out, f, separators=(",", ":"))
        f.write("\n")
    n = sum(len(t["err"]) for s in (far, close) for t in s)
    print(f"wrote {a.out}: {len(far)} + {len(close)} trials, {n} (err, cost) pairs; "
          f"resolution far {far_res}, close {close_res}")


if __name__ == "__main__":
    main()
