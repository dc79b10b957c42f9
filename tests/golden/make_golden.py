"""Capture golden vectors from the eshira/theta-rrt reference (build container ONLY).

This script is the ONLY place that imports the reference.  It runs in the build container where
`/root/reference` exists; its outputs (small `.npz`/`.json` fixtures next to this file) are what
travel to the GPU box.  Nothing under `tests/`, `oracle/`, `bench.py` or the product reads
`/root/reference` at run time.

Import recipe: `search` must be imported before `rrt` (search.py:151 resolves the
name `rrt` lazily), the map goes to `builtins.imarray` (main.py:42), parameters are `builtins.*`
(main.py:14-32).

Fixtures F1..F9:
  maps.npz        map1/map2/blank as `convert('1')` bool arrays (inputs; main.py:37-42)
  f1_astar.json   Theta*/A* on map2 (280,0)->(8,280)            search.py:221-307, main.py:57
  f2_los.npz      LOS queries captured from F1 + random pairs    search.py:35-41
  f3_bres.npz     Bresenham pixel lists                           search.py:43-94
  f4_arc.npz      getCircle / getArc pixel lists                  search.py:96-182
  f5_steer.npz    steer / drive in -> out                         rrt.py:272-541
  f6_rand.npz     rand_conf stream, seed 0                        rrt.py:53-68
  f7_nn.npz       inline NN argmin                                rrt.py:155-158
  f8_rrt.npz      full rrt() traces (B=1)                         rrt.py:130-206
  f9_batch.npz    snapshot-batch traces built from reference functions (B>1: snapshot-batch semantics)

Run:  MPLBACKEND=Agg python -B tests/golden/make_golden.py
"""
import builtins
import contextlib
import io
import json
import math
import os
import sys
import time

os.environ.setdefault("MPLBACKEND", "Agg")
sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

import numpy as np  # noqa: E402
import scipy  # noqa: E402
import PIL  # noqa: E402
from PIL import Image  # noqa: E402

sys.path.insert(0, REF)
import search  # noqa: E402  (must precede rrt)
import rrt  # noqa: E402

MAPS = {m: np.array(Image.open(os.path.join(REF, m + ".png")).convert("1")) for m in ("map1", "map2", "blank")}
DEFAULTS = dict(THETASTAR=True, bikelength=5, FORWARDONLY=True, LEFTCONSTRAINT=-65, RIGHTCONSTRAINT=65,
                frontclearance=2, K=300, showtree=False, maxdrivedist=30, tol_xy=10, tol_ang=45,
                weightxy=.6, xystdv=0.4, anglestdv=100)


def set_params(**kw):
    for k, v in DEFAULTS.items():
        setattr(builtins, k, v)
    for k, v in kw.items():
        setattr(builtins, k, v)


def use_map(name):
    builtins.imarray = MAPS[name].copy()


def quiet(fn, *a, **k):
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        r = fn(*a, **k)
    return r, buf.getvalue()


def flat_lists(lists):
    """Ragged list-of-pixel-lists -> (offsets int64[n+1], pix int64[m,2])."""
    off = np.zeros(len(lists) + 1, np.int64)
    rows = []
    for i, l in enumerate(lists):
        off[i + 1] = off[i] + len(l)
        rows.extend([(int(p[0]), int(p[1])) for p in l])
    pix = np.array(rows, np.int64).reshape(-1, 2)
    return off, pix


def u_to_row(u):
    """u = (steer, ICC|None, rad|None, dist) -> [steer, iccx, iccy, rad, dist, straight]."""
    if u[1] is None:
        return [float(u[0]), 0.0, 0.0, 0.0, float(u[3]), 1.0]
    return [float(u[0]), float(u[1][0]), float(u[1][1]), float(u[2]), float(u[3]), 0.0]


def row_to_u(r):
    if r[5]:
        return (r[0], None, None, r[4])
    return (r[0], np.array([r[1], r[2]]), r[3], r[4])


# ---------------------------------------------------------------- F1 + F2 (Theta*, LOS log)
def f1_f2():
    use_map("map2")
    out = {}
    los_log = []
    orig = search.lineofsight

    def logged(n1, n2):
        r = orig(n1, n2)
        los_log.append((int(n1[0]), int(n1[1]), int(n2[0]), int(n2[1]), int(r)))
        return r

    for theta in (True, False):
        set_params(THETASTAR=theta)
        if theta:
            search.lineofsight = logged
        t0 = time.time()
        path, txt = quiet(search.astar, (280, 0), (8, 280))
        search.lineofsight = orig
        exp = [int(l.split(":")[1]) for l in txt.splitlines() if l.startswith("Expanded nodes")]
        out["thetastar" if theta else "astar"] = dict(
            path=[[int(p[0]), int(p[1])] for p in path], expanded=exp[0], seconds=time.time() - t0)
    out["main_py_57"] = [[280, 0], [73, 38], [72, 39], [33, 130], [15, 190], [8, 280]]
    # a few invalid-input cases (search.py:222-227 prints and returns False)
    set_params()
    for s, g in (((-1, 5), (8, 280)), ((280, 0), (300, 5)), ((0, 0), (8, 280))):
        r, txt = quiet(search.astar, s, g)
        ret = r if r is False else [[int(a), int(b)] for a, b in r]
        out.setdefault("invalid", []).append(dict(start=list(s), goal=list(g), ret=ret, msg=txt.strip()))
    with open(os.path.join(OUT, "f1_astar.json"), "w") as f:
        json.dump(out, f, indent=1)

    theta_los = np.array(los_log, np.int64)
    # random pairs incl. out-of-bounds and negative-fraction endpoints (int() truncates toward 0)
    rng = np.random.default_rng(2)
    n = 20000
    seg = rng.uniform(-12, 311, size=(n, 4))
    seg[: n // 4] = np.round(seg[: n // 4])  # integral endpoints
    seg[n // 4: n // 2] = rng.uniform(-0.99, 0.99, size=(n // 4, 4)) + rng.integers(0, 3, size=(n // 4, 4))
    res = np.array([int(search.lineofsight((a, b), (c, d))) for a, b, c, d in seg.tolist()], np.uint8)
    np.savez_compressed(os.path.join(OUT, "f2_los.npz"), theta_q=theta_los[:, :4].astype(np.int32),
                        theta_r=theta_los[:, 4].astype(np.uint8), rand_seg=seg, rand_r=res)


# ---------------------------------------------------------------- F3 (Bresenham lists)
def f3():
    rng = np.random.default_rng(3)
    n = 1000
    seg = rng.uniform(-20, 320, size=(n, 4))
    seg[:300] = np.round(seg[:300])
    seg[300:350, 2] = seg[300:350, 0]  # vertical
    seg[350:400, 3] = seg[350:400, 1]  # horizontal
    seg[400:420, 2:] = seg[400:420, :2]  # degenerate (single pixel)
    lists = [search.bresenham((a, b), (c, d)) for a, b, c, d in seg.tolist()]
    off, pix = flat_lists(lists)
    np.savez_compressed(os.path.join(OUT, "f3_bres.npz"), seg=seg, off=off, pix=pix)


# ---------------------------------------------------------------- F4 (circle / arc lists)
def f4(arc_log):
    use_map("map2")
    set_params()
    rng = np.random.default_rng(4)
    # getCircle on assorted centres/radii (incl. partially off-map and non-integer inputs)
    circ_in = []
    for _ in range(300):
        cx, cy = rng.uniform(-30, 330, 2)
        r = float(np.exp(rng.uniform(0, 6)))
        circ_in.append((cx, cy, r))
    circ_in += [(150.0, 150.0, float(r)) for r in range(0, 40)]
    circ_lists = [search.getCircle((cx, cy), r) for cx, cy, r in circ_in]
    c_off, c_pix = flat_lists(circ_lists)
    # getArc on triples logged from real RRT runs (+ straight ones)
    rows = arc_log
    arc_lists = [search.getArc((r[0], r[1]), (r[2], r[3]), row_to_u(r[4:10])) for r in rows]
    a_off, a_pix = flat_lists(arc_lists)
    np.savez_compressed(os.path.join(OUT, "f4_arc.npz"), circ_in=np.array(circ_in), c_off=c_off, c_pix=c_pix,
                        arc_in=np.array(rows, np.float64), a_off=a_off, a_pix=a_pix)


# ---------------------------------------------------------------- F5 (steer / drive)
def f5():
    use_map("map2")
    set_params()
    rng = np.random.default_rng(5)
    n = 10000
    ins = []
    for i in range(n):
        ox, oy = rng.uniform(0, 300, 2)
        if i % 10 == 0:
            ox, oy = float(int(ox)), float(int(oy))
        th = float(rng.uniform(-180, 180))
        gx, gy = (int(v) for v in rng.uniform(0, 300, 2))
        tg = float(rng.uniform(-180, 180))
        ins.append([ox, oy, th, gx, gy, tg])
    # dead-ahead / dead-astern straight cases and cardinal headings
    for (ox, oy, th, gx, gy) in [(100, 100, 0.0, 120, 100), (100, 100, 0.0, 180, 100), (100, 100, 90.0, 100, 40),
                                 (100, 100, -90.0, 100, 160), (100, 100, 180.0, 60, 100), (5, 5, 0.0, 95, 5),
                                 (50, 50, 45.0, 80, 20), (50, 50, 0.0, 50, 50), (100, 100, 0.0, 99, 100)]:
        ins.append([float(ox), float(oy), th, gx, gy, 0.0])
    outs, st_u = [], []
    for ox, oy, th, gx, gy, tg in ins:
        origin = (ox, oy)
        (gp, fa), u = rrt.steer(origin, th, (int(gx), int(gy)), tg)
        outs.append([float(gp[0]), float(gp[1]), float(fa)])
        st_u.append(u_to_row(u))
    # drive(qnear, u/3) on the curved ones, as rrt.py:170-171 does
    d_in, d_out = [], []
    for row, u in zip(ins, st_u):
        if u[5]:
            continue
        uu = row_to_u(u)
        uu = (uu[0], uu[1], uu[2], uu[3] / 3)
        (fp, fa), _ = rrt.drive(((row[0], row[1]), row[2]), uu)
        d_in.append([row[0], row[1], row[2]] + u_to_row(uu))
        d_out.append([float(fp[0]), float(fp[1]), float(fa)])
        if len(d_in) >= 3000:
            break
    # body clearance rays (rrt.py:208-222) on map2
    bikes = rng.uniform(0, 300, size=(3000, 3))
    bikes[:, 2] = rng.uniform(-180, 180, 3000)
    bc = [int(rrt.bike_clear(((x, y), t))) for x, y, t in bikes.tolist()]
    fc = [int(rrt.front_of_bike_clear(((x, y), t))) for x, y, t in bikes.tolist()]
    # angle helpers
    a12 = rng.uniform(-180, 180, size=(5000, 2))
    a12[:100, 1] = a12[:100, 0]
    a12[100:200, 1] = np.where(a12[100:200, 0] > 0, a12[100:200, 0] - 180, a12[100:200, 0] + 180)
    adiff = [float(rrt.anglediff(a, b)) for a, b in a12.tolist()]
    vecs = rng.normal(size=(5000, 2)) * 50
    vecs[:50] = 0
    vecs[50:100, 1] = 0
    ab = [float(rrt.anglebetween([1, 0], v)) for v in vecs]
    sa_in = rng.uniform(-1000, 1000, 2000)
    sa = [float(rrt.standardangle(float(a))) for a in sa_in]
    np.savez_compressed(os.path.join(OUT, "f5_steer.npz"), steer_in=np.array(ins), steer_out=np.array(outs),
                        steer_u=np.array(st_u), drive_in=np.array(d_in), drive_out=np.array(d_out),
                        bikes=bikes, bike_clear=np.array(bc, np.uint8), front_clear=np.array(fc, np.uint8),
                        adiff_in=a12, adiff_out=np.array(adiff), ab_in=vecs, ab_out=np.array(ab),
                        sa_in=sa_in, sa_out=np.array(sa))


# ---------------------------------------------------------------- F6 (rand_conf)
def f6():
    set_params()
    out = {}
    for name, shape, goal in (("g100", (100, 100), ((90, 90), 45.0)), ("g300", (300, 300), ((73, 38), -170.0)),
                              ("g512", (512, 512), ((256, 256), 0.0))):
        builtins.imarray = np.ones(shape, bool)
        np.random.seed(0)
        s = [rrt.rand_conf(goal) for _ in range(10000)]
        out[name + "_xy"] = np.array([q[0] for q in s], np.int64)
        out[name + "_th"] = np.array([q[1] for q in s], np.float64)
        out[name + "_goal"] = np.array([goal[0][0], goal[0][1], goal[1]], np.float64)
        out[name + "_shape"] = np.array(shape, np.int64)
    np.savez_compressed(os.path.join(OUT, "f6_rand.npz"), **out)


# ---------------------------------------------------------------- F7 (NN)
def ref_nn(keys, q):
    # verbatim call pattern of rrt.py:156-157
    return int(np.argmin([search.L2norm(item[0], q) for item in keys]))


def f7():
    rng = np.random.default_rng(7)
    out = {}
    for N, nq in ((1000, 500), (100000, 24)):
        xy = rng.uniform(0, 512, size=(N, 2))
        xy[: N // 10] = np.round(xy[: N // 10])  # some integral coords
        xy[N // 10: N // 10 + 50] = xy[N // 10 + 50: N // 10 + 100]  # exact duplicates at later index
        q = rng.integers(0, 512, size=(nq, 2))
        keys = [((x, y), 0.0) for x, y in xy.tolist()]
        ans = [ref_nn(keys, (int(a), int(b))) for a, b in q.tolist()]
        out["xy%d" % N], out["q%d" % N], out["idx%d" % N] = xy, q, np.array(ans, np.int64)
    # engineered ties: equal distances at different indices, and sqrt-collapsing near ties
    tie_xy, tie_q = [], []
    for i in range(200):
        qx, qy = int(rng.integers(20, 480)), int(rng.integers(20, 480))
        d = float(rng.uniform(1, 15))
        base = [(qx + d, qy), (qx, qy - d), (qx - d, qy), (qx, qy + d)]
        rng.shuffle(base)
        far = [tuple(v) for v in (rng.uniform(0, 512, size=(6, 2)) + 600).tolist()]
        # near tie: squared distance differs by ulps but sqrt may coincide
        s = d * d
        e = math.sqrt(np.nextafter(np.nextafter(s, 1e9), 1e9))
        near = [(qx + e, qy)]
        pts = far[:3] + near + base + far[3:]
        tie_xy.append(pts)
        tie_q.append((qx, qy))
    tie_xy = np.array(tie_xy)
    tie_ans = [ref_nn([((x, y), 0.0) for x, y in pts.tolist()], q) for pts, q in zip(tie_xy, tie_q)]
    out["tie_xy"], out["tie_q"], out["tie_idx"] = tie_xy, np.array(tie_q, np.int64), np.array(tie_ans, np.int64)
    np.savez_compressed(os.path.join(OUT, "f7_nn.npz"), **out)


# ---------------------------------------------------------------- F8 (full rrt traces)
def trace_arrays(start, sol, G, cameFrom):
    keys = list(G.keys())
    index = {k: i for i, k in enumerate(keys)}
    nodes = np.array([[float(k[0][0]), float(k[0][1]), float(k[1])] for k in keys], np.float64)
    parent = np.full(len(keys), -1, np.int64)
    u = np.zeros((len(keys), 6), np.float64)
    for k, v in cameFrom.items():
        if v is None:
            continue
        parent[index[k]] = index[v[0]]
        u[index[k]] = u_to_row(v[1])
    e_off = np.zeros(len(keys) + 1, np.int64)
    e_child = []
    for i, k in enumerate(keys):
        e_child.extend(index[c] for c in G[k])
        e_off[i + 1] = len(e_child)
    return dict(nodes=nodes, parent=parent, u=u, e_off=e_off, e_child=np.array(e_child, np.int64),
                sol=np.int64(-1 if sol is None else index[sol]))


def run_rrt_logged(mapname, seed, K, start, goal, tol_xy, arc_log, max_log=800):
    use_map(mapname)
    set_params(K=K, tol_xy=tol_xy)
    orig = search.getArc

    def logged(begin, land, u):
        r = orig(begin, land, u)
        if len(arc_log) < max_log:
            arc_log.append([float(begin[0]), float(begin[1]), float(land[0]), float(land[1])] + u_to_row(u))
        return r

    search.getArc = logged
    np.random.seed(seed)
    err = ""
    try:
        (sol, G, cameFrom), _ = quiet(rrt.rrt, start, goal)
    except TypeError as e:
        err = "TypeError: " + str(e)
        sol, G, cameFrom = None, {start: []}, {start: None}
    finally:
        search.getArc = orig
    return sol, G, cameFrom, err


def f8(arc_log):
    out = {}
    meta = {}
    runs = [("m1s0", "map1", 0, 1001, ((5, 5), 0.0), ((90, 90), 45.0), 0),
            ("m1s1", "map1", 1, 1001, ((5, 5), 0.0), ((90, 90), 45.0), 0),
            ("m1goal", "map1", 3, 1001, ((5, 5), 0.0), ((90, 90), 45.0), 10),
            ("m2s0", "map2", 0, 2001, ((280, 0), -170.0), ((73, 38), 0.0), 0),
            ("m1s7", "map1", 7, 1001, ((5, 5), 0.0), ((90, 90), 45.0), 0)]
    for tag, m, seed, K, start, goal, tol in runs:
        t0 = time.time()
        sol, G, cameFrom, err = run_rrt_logged(m, seed, K, start, goal, tol, arc_log)
        meta[tag] = dict(map=m, seed=seed, K=K, start=[list(start[0]), start[1]], goal=[list(goal[0]), goal[1]],
                         tol_xy=tol, error=err, seconds=time.time() - t0, nodes=len(G))
        if not err:
            for k, v in trace_arrays(start, sol, G, cameFrom).items():
                out[tag + "_" + k] = v
        print(tag, meta[tag], flush=True)
    np.savez_compressed(os.path.join(OUT, "f8_rrt.npz"), **out)
    with open(os.path.join(OUT, "f8_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


# ---------------------------------------------------------------- F9 (snapshot-batch semantics)
def batch_rrt_from_reference(start, goal, K, B):
    """Snapshot-batch RRT composed ONLY of reference functions (every sample of a batch sees the tree as it stood when the batch began).

    Per batch: every sample's decisions (freespace, membership, NN, steer, clearance, drive, arc) use
    the tree as it stood at batch start; accepted nodes are then appended in sample order with the
    reference's own bookkeeping rules (rrt.py:179-201), stopping at the first goal hit.
    """
    start = (start[0], rrt.standardangle(start[1]))
    goal = (goal[0], rrt.standardangle(goal[1]))
    G = {start: []}
    cameFrom = {start: None}
    sol = None
    total = K - 1
    done = 0
    while done < total and sol is None:
        b = min(B, total - done)
        done += b
        snap = list(G.keys())
        snapset = set(snap)
        recs = []
        for _ in range(b):
            qrand = rrt.rand_conf(goal)
            qrand = (qrand[0], rrt.standardangle(qrand[1]))
            if not search.freespace(qrand[0]) or qrand in snapset:
                continue
            qnear = snap[int(np.argmin([search.L2norm(it[0], qrand[0]) for it in snap]))]
            qdrive, u = rrt.steer(qnear[0], qnear[1], qrand[0], qrand[1])
            qnew = ((qdrive[0][0], qdrive[0][1]), qdrive[1])
            if not search.valid(qnew[0]) or not rrt.bike_clear(qnew) or not rrt.front_of_bike_clear(qnew):
                u = (u[0], u[1], u[2], u[3] / 3)
                qnew, u = rrt.drive(qnear, u)
            if False in [search.freespace(px) for px in search.getArc(qnear[0], qnew[0], u)]:
                continue
            recs.append((qnear, qnew, u))
        for qnear, qnew, u in recs:
            if qnew not in G:
                G[qnew] = []
            G[qnear].append(qnew)
            if qnew != qnear:
                cameFrom[qnew] = (qnear, u)
            d = rrt.anglediff(qnew[1], goal[1])
            if search.L2norm(qnew[0], goal[0]) < builtins.tol_xy and abs(d) < builtins.tol_ang:
                sol = qnew
                break
    return sol, G, cameFrom


def f9():
    out, meta = {}, {}
    for tag, m, seed, K, B, start, goal, tol in (
            ("m1b64", "map1", 0, 1281, 64, ((5, 5), 0.0), ((90, 90), 45.0), 0),
            ("m1b1", "map1", 2, 301, 1, ((5, 5), 0.0), ((90, 90), 45.0), 0),
            ("m2b256", "map2", 1, 1025, 256, ((280, 0), -170.0), ((73, 38), 0.0), 0),
            ("m1b32g", "map1", 3, 2001, 32, ((5, 5), 0.0), ((90, 90), 45.0), 10)):
        use_map(m)
        set_params(tol_xy=tol)
        np.random.seed(seed)
        t0 = time.time()
        err = ""
        try:
            sol, G, cameFrom = batch_rrt_from_reference(start, goal, K, B)
        except TypeError as e:
            err = "TypeError: " + str(e)
        meta[tag] = dict(map=m, seed=seed, K=K, B=B, start=[list(start[0]), start[1]],
                         goal=[list(goal[0]), goal[1]], tol_xy=tol, error=err, seconds=time.time() - t0)
        if not err:
            meta[tag]["nodes"] = len(G)
            for k, v in trace_arrays(start, sol, G, cameFrom).items():
                out[tag + "_" + k] = v
        print(tag, meta[tag], flush=True)
    np.savez_compressed(os.path.join(OUT, "f9_batch.npz"), **out)
    with open(os.path.join(OUT, "f9_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


# ---------------------------------------------------------------- F10 (findnearest)
def tree_from_arrays(nodes, e_off, e_child):
    """G dict (insertion order = node index, children in edge order) from trace arrays."""
    keys = [((float(x), float(y)), float(t)) for x, y, t in nodes]
    return {k: [keys[c] for c in e_child[e_off[i]:e_off[i + 1]]] for i, k in enumerate(keys)}


def f10():
    """rrt.findnearest (rrt.py:117-128) on the F8 trees and on hand-made trees with exact ties.

    Inputs per case: nodes [n][3], edges (e_par, e_child) in the reference's traversal order, goals
    [g][3]; outputs: the chosen child's node index and its distance."""
    set_params()
    f8 = np.load(os.path.join(OUT, "f8_rrt.npz"))
    rng = np.random.default_rng(10)
    # main.py:57-68 waypoint poses (goal angle = heading of the next leg)
    path = [(280, 0), (73, 38), (72, 39), (33, 130), (15, 190), (8, 280)]
    way = []
    for a, b, c in zip(path, path[1:], path[2:] + [None]):
        ang1 = rrt.anglebetween([1, 0], np.subtract(b, a))
        ang2 = ang1 if c is None else rrt.anglebetween([1, 0], np.subtract(c, b))
        way.append([float(b[0]), float(b[1]), float(rrt.standardangle(ang2))])
    cases = {}
    for tag in ("m1s0", "m2s0"):
        nodes, e_off, e_child = f8[tag + "_nodes"], f8[tag + "_e_off"], f8[tag + "_e_child"]
        goals = np.array(way + [[float(x), float(y), float(t)] for x, y, t in zip(
            rng.integers(0, 300, 12), rng.integers(0, 300, 12), rng.uniform(-180, 180, 12))])
        cases[tag] = (nodes, e_off, e_child, goals)
    # exact ties: children at equal L2 and equal heading, a child under two parents, integral poses
    pts = [((50.0, 50.0), 0.0), ((47.0, 50.0), 0.0), ((53.0, 50.0), 0.0), ((50.0, 47.0), 0.0),
           ((50.0, 53.0), 0.0), ((53.0, 50.0), 180.0), ((47.0, 50.0), -90.0), ((50.0, 50.0), 90.0)]
    kids = {0: [2, 1], 1: [3, 4], 2: [2], 3: [5, 6, 1], 4: [7], 5: [], 6: [], 7: [0]}
    nodes = np.array([[p[0][0], p[0][1], p[1]] for p in pts])
    e_off = np.zeros(len(pts) + 1, np.int64)
    e_child = []
    for i in range(len(pts)):
        e_child.extend(kids[i])
        e_off[i + 1] = len(e_child)
    goals = np.array([[50, 50, 0], [50, 50, 90], [50, 50, 180], [50, 50, -90], [0, 0, 45],
                      [50, 50, 45], [53, 50, 0], [47, 50, -90]], np.float64)
    cases["ties"] = (nodes, e_off, np.array(e_child, np.int64), goals)
    out = {}
    for tag, (nodes, e_off, e_child, goals) in cases.items():
        G = tree_from_arrays(nodes, e_off, e_child)
        keys = list(G.keys())
        index = {k: i for i, k in enumerate(keys)}
        idx, dist = [], []
        for g in goals:
            goal = ((g[0], g[1]), g[2])
            node, d = rrt.findnearest(G, goal)
            idx.append(-1 if node is None else index[node])
            dist.append(np.nan if d is None else float(d))
        e_par = np.repeat(np.arange(len(nodes)), np.diff(e_off))
        out.update({tag + "_nodes": nodes, tag + "_e_par": e_par, tag + "_e_child": e_child,
                    tag + "_goals": goals, tag + "_idx": np.array(idx, np.int64),
                    tag + "_dist": np.array(dist)})
        print(tag, idx, flush=True)
    np.savez_compressed(os.path.join(OUT, "f10_findnearest.npz"), **out)


def main():
    what = sys.argv[1:] or ["maps", "f1", "f3", "f5", "f6", "f7", "f8", "f9", "f10"]
    versions = dict(numpy=np.__version__, scipy=scipy.__version__, pillow=PIL.__version__,
                    python=sys.version.split()[0])
    with open(os.path.join(OUT, "versions.json"), "w") as f:
        json.dump(versions, f, indent=1)
    if "maps" in what:
        np.savez_compressed(os.path.join(OUT, "maps.npz"), **MAPS)
    t = time.time()
    if "f1" in what:
        f1_f2(); print("f1/f2", time.time() - t, flush=True)
    if "f3" in what:
        f3(); print("f3", time.time() - t, flush=True)
    if "f5" in what:
        f5(); print("f5", time.time() - t, flush=True)
    if "f6" in what:
        f6(); print("f6", time.time() - t, flush=True)
    if "f7" in what:
        f7(); print("f7", time.time() - t, flush=True)
    if "f8" in what:
        arc_log = []
        f8(arc_log)
        # straight-u getArc cases and large radii round out F4
        rng = np.random.default_rng(44)
        for _ in range(50):
            b = rng.uniform(0, 300, 2); l = b + rng.uniform(-30, 30, 2)
            arc_log.append([b[0], b[1], l[0], l[1], 0.0, 0.0, 0.0, 0.0, 1.0, 1.0])
        f4(arc_log); print("f8/f4", time.time() - t, flush=True)
    if "f9" in what:
        f9(); print("f9", time.time() - t, flush=True)
    if "f10" in what:
        f10(); print("f10", time.time() - t, flush=True)


if __name__ == "__main__":
    main()
