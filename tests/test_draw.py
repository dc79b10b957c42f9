"""CPU: the matplotlib renderer (reference rrt.py:16-40,79-106,224-270, search.py:206-219) draws
the same primitives the reference does for a small tree built by the oracle's steer: one dashed
arc patch per curved edge, a dashed line per straight edge, bicycles (body line + 3 arrows) along a
path, and the Bresenham pixels of a Theta* path.  No GPU: the drawing is host-only."""
import builtins

import numpy as np
import pytest

import pkgload
import thetarrt_oracle as O

pkgload.load()
from theta_rrt_amd import config, draw  # noqa: E402

mpl = pytest.importorskip("matplotlib")
mpl.use("Agg")
import matplotlib.patches as patches  # noqa: E402
import matplotlib.pyplot as plt  # noqa: E402


def small_tree():
    config.ensure_defaults()
    P = O.Params()
    root = ((20.0, 20.0), 0.0)
    (p1, t1), u1 = O.steer(P, root[0], root[1], (60, 40), 30.0)
    n1 = ((float(p1[0]), float(p1[1])), float(t1))
    (p2, t2), u2 = O._straight(P, n1[0], n1[1], (90, 90))
    n2 = ((float(p2[0]), float(p2[1])), float(t2))
    G = {root: [n1], n1: [n2], n2: []}
    cameFrom = {root: None, n1: (root, u1), n2: (n1, u2)}
    assert u1[1] is not None and u2[1] is None
    return root, n1, n2, G, cameFrom


def test_drawtree_and_drawpath_primitives():
    root, n1, n2, G, cameFrom = small_tree()
    fig, ax = plt.subplots()
    builtins.ax = ax
    try:
        draw.drawtree(root, G, cameFrom)
        arcs = [p for p in ax.patches if isinstance(p, patches.Arc)]
        assert len(arcs) == 1
        assert np.allclose(arcs[0].center, cameFrom[n1][1][1])
        assert arcs[0].get_linestyle() == "--"
        dashed = [ln for ln in ax.lines if ln.get_linestyle() == "--"]
        assert len(dashed) == 1                          # the straight edge n1 -> n2
        assert np.allclose(dashed[0].get_xdata(), [n1[0][0], n2[0][0]])
        assert len(ax.collections) == 3                  # one leaf bicycle: 3 quiver arrows
        draw.drawpath(n2, cameFrom)
        assert len([p for p in ax.patches if isinstance(p, patches.Arc)]) == 2
        assert len(ax.collections) == 3 + 3 * 3          # solution + 2 segment bicycles
        draw.drawpath(root, cameFrom)                    # root: nothing to draw
        assert len(ax.collections) == 12
    finally:
        builtins.ax = None
        plt.close(fig)


def test_search_drawpath_pixels():
    fig, ax = plt.subplots()
    try:
        plt.sca(ax)
        path = [(0, 0), (10, 3), (10, 12)]
        draw.search_drawpath(path, O.bresenham)
        pts = ax.collections[0].get_offsets()
        want = O.bresenham(path[0], path[1]) + O.bresenham(path[1], path[2])
        assert np.array_equal(np.asarray(pts), np.asarray(want, float))
    finally:
        plt.close(fig)
