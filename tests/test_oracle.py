"""Pin the CPU oracle (oracle/thetarrt_oracle.py) against the reference's golden vectors.

Every fixture under tests/golden/ was produced by importing eshira/theta-rrt itself
(tests/golden/make_golden.py).  These tests run on CPU only.
"""
import math

import numpy as np
import pytest

from conftest import golden
import thetarrt_oracle as O

P = O.Params()


def test_scipy_restatement_matches_installed_scipy():
    from scipy.spatial.transform import Rotation as R
    rng = np.random.default_rng(11)
    for _ in range(2000):
        a1, a2 = rng.uniform(-400, 400, 2)
        d = np.rad2deg((R.from_euler('z', a1, degrees=True).inv() * R.from_euler('z', a2, degrees=True)).as_euler('xyz')[2])
        assert O.angle_diff(float(a1), float(a2)) == d
        v = rng.normal(size=3) * 20
        assert np.array_equal(O._zrot(float(a1), v), R.from_euler('z', a1, degrees=True).apply(v))


def test_angles_golden():
    f = golden("f5_steer.npz")
    got = [O.angle_diff(a, b) for a, b in f["adiff_in"].tolist()]
    assert np.array_equal(np.array(got), f["adiff_out"])
    got = [O.heading(v) for v in f["ab_in"]]
    assert np.array_equal(np.array(got), f["ab_out"])
    got = [O.wrap180(float(a)) for a in f["sa_in"]]
    assert np.array_equal(np.array(got), f["sa_out"])


def test_bresenham_golden():
    f = golden("f3_bres.npz")
    seg, off, pix = f["seg"], f["off"], f["pix"]
    for i, (a, b, c, d) in enumerate(seg.tolist()):
        assert O.bresenham((a, b), (c, d)) == [tuple(p) for p in pix[off[i]:off[i + 1]].tolist()]


def test_los_golden(maps):
    f = golden("f2_los.npz")
    g = O.Grid(maps["map2"])
    q, r = f["theta_q"], f["theta_r"]
    for i in range(0, len(q), 7):           # every 7th of the 30k Theta* queries
        a, b, c, d = q[i].tolist()
        assert g.los((a, b), (c, d)) == bool(r[i])
    for (a, b, c, d), rr in zip(f["rand_seg"].tolist(), f["rand_r"].tolist()):
        assert g.los((a, b), (c, d)) == bool(rr)


def test_circle_arc_golden(maps):
    f = golden("f4_arc.npz")
    g = O.Grid(maps["map2"])
    for i, (cx, cy, r) in enumerate(f["circ_in"].tolist()):
        ref = [tuple(p) for p in f["c_pix"][f["c_off"][i]:f["c_off"][i + 1]].tolist()]
        assert O.circle_pixels(g, (cx, cy), r) == ref
    for i, row in enumerate(f["arc_in"].tolist()):
        u = (row[4], None, None, row[8]) if row[9] else (row[4], np.array([row[5], row[6]]), row[7], row[8])
        ref = [tuple(p) for p in f["a_pix"][f["a_off"][i]:f["a_off"][i + 1]].tolist()]
        assert [tuple(map(int, p)) for p in O.arc_pixels(g, (row[0], row[1]), (row[2], row[3]), u)] == ref


def test_steer_drive_golden(maps):
    f = golden("f5_steer.npz")
    for row, out, u in zip(f["steer_in"].tolist(), f["steer_out"], f["steer_u"]):
        ox, oy, th, gx, gy, tg = row
        (gp, fa), uu = O.steer(P, (ox, oy), th, (int(gx), int(gy)), tg)
        assert [float(gp[0]), float(gp[1]), float(fa)] == out.tolist()
        if uu[1] is None:
            assert u[5] == 1 and uu[0] == u[0] and uu[3] == u[4]
        else:
            assert [uu[0], uu[1][0], uu[1][1], uu[2], uu[3], 0.0] == u.tolist()
    for row, out in zip(f["drive_in"].tolist(), f["drive_out"]):
        u = (row[3], np.array([row[4], row[5]]), row[6], row[7])
        (fp, fa), _ = O.drive(P, ((row[0], row[1]), row[2]), u)
        assert [float(fp[0]), float(fp[1]), float(fa)] == out.tolist()
    g = O.Grid(maps["map2"])
    for (x, y, t), bc, fc in zip(f["bikes"].tolist(), f["bike_clear"], f["front_clear"]):
        assert O.body_clear(g, P, ((x, y), t)) == bool(bc)
        assert O.body_clear(g, P, ((x, y), t), P.frontclearance) == bool(fc)


def test_rand_conf_golden():
    f = golden("f6_rand.npz")
    for name in ("g100", "g300", "g512"):
        shape = tuple(f[name + "_shape"].tolist())
        gx, gy, gt = f[name + "_goal"].tolist()
        goal = ((int(gx), int(gy)), gt)
        np.random.seed(0)
        s = [O.rand_conf(P, shape, goal) for _ in range(3000)]
        assert np.array_equal(np.array([q[0] for q in s]), f[name + "_xy"][:3000])
        assert np.array_equal(np.array([q[1] for q in s]), f[name + "_th"][:3000])
        np.random.seed(0)
        b = O.samples_from_gauss(P, shape, goal, np.random.standard_normal(3 * 10000))
        assert np.array_equal(np.array([q[0] for q in b]), f[name + "_xy"])
        assert np.array_equal(np.array([q[1] for q in b]), f[name + "_th"])


def test_nn_golden():
    f = golden("f7_nn.npz")
    for N in (1000, 100000):
        xy, q, idx = f["xy%d" % N], f["q%d" % N], f["idx%d" % N]
        assert np.array_equal(O.nn_numpy(xy[:, 0], xy[:, 1], q[:, 0], q[:, 1]), idx)
    xy, q = f["xy1000"], f["q1000"]
    assert [O.nn_loop(xy.tolist(), tuple(qq)) for qq in q[:50].tolist()] == f["idx1000"][:50].tolist()
    for pts, qq, i in zip(f["tie_xy"], f["tie_q"], f["tie_idx"]):
        assert O.nn_numpy(pts[:, 0], pts[:, 1], qq[:1], qq[1:]).tolist() == [i]
        assert O.nn_loop(pts.tolist(), tuple(qq.tolist())) == i


def test_findnearest_golden():
    """rrt.findnearest (rrt.py:117-128) on the F8 trees and on exact-tie trees (F10)."""
    f = golden("f10_findnearest.npz")
    P = O.Params()
    for tag in ("m1s0", "m2s0", "ties"):
        nodes, ec, goals = f[tag + "_nodes"], f[tag + "_e_child"], f[tag + "_goals"]
        for g, i, d in zip(goals, f[tag + "_idx"], f[tag + "_dist"]):
            oi, od = O.findnearest(P, nodes.tolist(), f[tag + "_e_par"], ec, ((g[0], g[1]), g[2]))
            assert oi == i and od == d, (tag, g, oi, i, od, d)


def _check_trace(T, sol, f, tag):
    nodes = np.array([[float(n[0][0]), float(n[0][1]), float(n[1])] for n in T.nodes])
    assert nodes.shape == f[tag + "_nodes"].shape
    assert np.array_equal(nodes, f[tag + "_nodes"])
    assert np.array_equal(np.array(T.parent), f[tag + "_parent"])
    e_off = np.cumsum([0] + [len(c) for c in T.children])
    assert np.array_equal(e_off, f[tag + "_e_off"])
    assert np.array_equal(np.array([c for cs in T.children for c in cs], np.int64), f[tag + "_e_child"])
    assert (-1 if sol is None else sol) == int(f[tag + "_sol"])


def _run(maps, meta, B):
    Pm = O.Params(K=meta["K"], tol_xy=meta["tol_xy"])
    g = O.Grid(maps[meta["map"]])
    np.random.seed(meta["seed"])
    start = (tuple(meta["start"][0]), meta["start"][1])
    goal = (tuple(meta["goal"][0]), meta["goal"][1])
    return O.rrt_batched(Pm, g, start, goal, B=B)


@pytest.mark.parametrize("tag", ["m1s0", "m1goal", "m2s0"])
def test_rrt_trace_b1_golden(maps, tag):
    meta = golden("f8_meta.json")[tag]
    sol, T = _run(maps, meta, 1)
    _check_trace(T, sol, golden("f8_rrt.npz"), tag)


def test_rrt_typeerror_golden(maps):
    meta = golden("f8_meta.json")["m1s7"]
    assert meta["error"].startswith("TypeError")
    with pytest.raises(TypeError):
        _run(maps, meta, 1)


@pytest.mark.parametrize("tag", ["m1b64", "m1b1", "m2b256", "m1b32g"])
def test_rrt_batch_golden(maps, tag):
    meta = golden("f9_meta.json")[tag]
    sol, T = _run(maps, meta, meta["B"])
    _check_trace(T, sol, golden("f9_batch.npz"), tag)


def test_astar_known_answer(maps):
    f = golden("f1_astar.json")
    g = O.Grid(maps["map2"])
    path, exp, _ = O.astar(O.Params(THETASTAR=True), g, (280, 0), (8, 280))
    assert [list(p) for p in path] == f["thetastar"]["path"] == f["main_py_57"]
    assert exp == f["thetastar"]["expanded"]
