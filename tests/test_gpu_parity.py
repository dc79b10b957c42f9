"""GPU parity: every kernel through the C-ABI against the reference's golden vectors and the oracle.

Bar (BASELINE.json north_star): node indices / parents / decisions bit-identical; node coordinates
within 1e-6 (fp64 trig on the GPU differs from glibc/SVML in the last ulps).
"""
import builtins

import numpy as np
import pytest

from conftest import golden
import pkgload
import thetarrt_oracle as O

pkgload.load()
from theta_rrt_amd import _native, config, rrt, search, workloads  # noqa: E402

pytestmark = pytest.mark.gpu
TOL = 1e-6


@pytest.fixture(scope="module")
def eng():
    return _native.engine()


def use_map(eng, maps, name):
    builtins.imarray = maps[name]
    config.ensure_defaults()
    eng.set_params(config.native_params())
    eng.set_grid(maps[name])


@pytest.fixture(params=["cells", "cells_far_sweep", "sweep"])
def nn_path(request, eng):
    """Every nearest-node path: the cell lists with long second passes scanned by their block, the
    cell lists with those samples handed to the sweep as a list, and the sweep of every node."""
    old = [(k, eng.get_option(k)) for k in ("nn_grid", "nn_far_sweep", "nn_grid_min")]
    eng.set_option("nn_grid", 0 if request.param == "sweep" else 1)
    eng.set_option("nn_far_sweep", 0 if request.param == "cells_far_sweep" else 1 << 40)
    eng.set_option("nn_grid_min", 0)
    yield request.param
    for k, v in old:
        eng.set_option(k, v)


def test_nn_golden(eng, maps, nn_path):
    use_map(eng, maps, "map2")
    f = golden("f7_nn.npz")
    for N in (1000, 100000):
        xy, q, idx = f["xy%d" % N], f["q%d" % N], f["idx%d" % N]
        eng.tree_reset(N)
        eng.tree_append(np.c_[xy, np.zeros(N)])
        assert np.array_equal(eng.nn(q), idx)
    for pts, qq, i in zip(f["tie_xy"], f["tie_q"], f["tie_idx"]):
        eng.tree_reset(len(pts))
        eng.tree_append(np.c_[pts, np.zeros(len(pts))])
        assert eng.nn(qq[None])[0] == i


def test_nn_large_vs_oracle(eng, maps, nn_path):
    """cfg2-sized snapshot (N=100k) and a 4096-sample batch, plus chunk boundary duplicates."""
    use_map(eng, maps, "map2")
    rng = np.random.default_rng(21)
    N, B = 100000, 4096
    xy = rng.uniform(0, 512, size=(N, 2))
    xy[50000:50100] = xy[:100]                      # equal distances across chunks
    q = rng.integers(0, 512, size=(B, 2))
    eng.tree_reset(N)
    eng.tree_append(np.c_[xy, np.zeros(N)])
    assert np.array_equal(eng.nn(q), O.nn_numpy(xy[:, 0], xy[:, 1], q[:, 0], q[:, 1]))
    # integral tree (many exact ties) and tiny trees
    xy = rng.integers(0, 64, size=(5000, 2)).astype(np.float64)
    eng.tree_reset(5000)
    eng.tree_append(np.c_[xy, np.zeros(5000)])
    q = rng.integers(0, 64, size=(777, 2))
    assert np.array_equal(eng.nn(q), O.nn_numpy(xy[:, 0], xy[:, 1], q[:, 0], q[:, 1]))
    for n in (1, 2, 3, 65):
        eng.tree_reset(n)
        eng.tree_append(np.c_[xy[:n], np.zeros(n)])
        assert np.array_equal(eng.nn(q[:5]), O.nn_numpy(xy[:n, 0], xy[:n, 1], q[:5, 0], q[:5, 1]))


def test_nn_clustered_tree(eng, maps, nn_path):
    """A tree piled up in a few spots (thousands of nodes inside one pixel, as a grown RRT's
    is), nodes outside the map, and samples near to and far from the piles."""
    use_map(eng, maps, "map2")
    H, W = maps["map2"].shape
    rng = np.random.default_rng(33)
    piles = [(45.3, 17.6, 6000), (0.2, 0.1, 3000), (H - 0.5, W - 0.25, 3000), (300.0, 200.0, 500)]
    nodes = [rng.uniform(-12, max(H, W) + 12, size=(20000, 2))]
    for x, y, n in piles:
        nodes.append(np.c_[x, y] + rng.normal(0, 0.2, size=(n, 2)))
    xy = np.concatenate(nodes)
    xy = xy[rng.permutation(len(xy))]
    q = np.concatenate([rng.integers(0, min(H, W), size=(1500, 2)),
                        np.array([[0, 0], [H - 1, W - 1], [0, W - 1], [H - 1, 0], [45, 17], [46, 18]] * 20),
                        np.c_[np.zeros(200, np.int64), rng.integers(0, W, 200)]])
    eng.tree_reset(len(xy))
    # grown in steps: the cell lists merge each step's nodes into the last build
    for a in range(0, len(xy), 7000):
        eng.tree_append(np.c_[xy[a:a + 7000], np.zeros(len(xy[a:a + 7000]))])
        n = min(a + 7000, len(xy))
        assert np.array_equal(eng.nn(q), O.nn_numpy(xy[:n, 0], xy[:n, 1], q[:, 0], q[:, 1])), n


def test_nn_screen_adversarial(eng, maps, nn_path):
    """Near-ties for the fp32 screen: many nodes within a few ulps of the same fp64 distance, in
    different chunks and in reverse index order, on a centred tree (grid set) and on an uncentred
    one with large, negative and fractional coordinates."""
    rng = np.random.default_rng(5)
    for centred in (True, False):
        if centred:
            use_map(eng, maps, "map2")
            off = 150.0
        else:
            eng.set_grid(np.ones((4, 4), np.uint8))    # centre (2, 2); coordinates far from it
            off = -3000.5
        B = 300
        q = rng.integers(0, 300, size=(B, 2)) + (0 if centred else -3000)
        nodes = [rng.uniform(-200, 200, size=(20000, 2)) + off]
        for j in range(0, B, 3):                     # 12 near-equal nodes around every 3rd query
            r = rng.uniform(0.5, 40.0)
            ang = rng.uniform(0, 2 * np.pi, 12)
            pts = q[j] + np.c_[r * np.cos(ang), r * np.sin(ang)]
            pts[6:] = q[j] + np.c_[np.nextafter(r * np.cos(ang[:6]), np.inf), r * np.sin(ang[:6])]
            nodes.append(pts[::-1])
        xy = np.concatenate(nodes)
        perm = rng.permutation(len(xy))
        xy = xy[perm]
        eng.tree_reset(len(xy))
        eng.tree_append(np.c_[xy, np.zeros(len(xy))])
        want = O.nn_numpy(xy[:, 0], xy[:, 1], q[:, 0], q[:, 1])
        assert np.array_equal(eng.nn(q), want)


def test_los_golden(eng, maps):
    use_map(eng, maps, "map2")
    f = golden("f2_los.npz")
    q = f["theta_q"].astype(np.float64)
    assert np.array_equal(eng.los(q), f["theta_r"].astype(bool))
    assert np.array_equal(eng.los(f["rand_seg"]), f["rand_r"].astype(bool))
    # symmetry of the pixel set (search.py:43-56 iterates from the lower major-axis endpoint)
    s = f["rand_seg"]
    assert np.array_equal(eng.los(s), eng.los(s[:, [2, 3, 0, 1]]))


def test_bresenham_lists_golden(eng):
    f = golden("f3_bres.npz")
    for i, s in enumerate(f["seg"]):
        assert np.array_equal(eng.bresenham(s), f["pix"][f["off"][i]:f["off"][i + 1]])


def test_circle_arc_lists_golden(eng, maps):
    use_map(eng, maps, "map2")
    f = golden("f4_arc.npz")
    for i, (cx, cy, r) in enumerate(f["circ_in"]):
        assert np.array_equal(eng.circle(cx, cy, r), f["c_pix"][f["c_off"][i]:f["c_off"][i + 1]])
    for i, row in enumerate(f["arc_in"]):
        assert np.array_equal(eng.arc_pixels(row), f["a_pix"][f["a_off"][i]:f["a_off"][i + 1]])


def _arc_truth(g, rows):
    out = []
    for r in rows:
        u = (r[4], None, None, r[8]) if r[9] else (r[4], np.array([r[5], r[6]]), r[7], r[8])
        out.append(all(g.freespace(p) for p in O.arc_pixels(g, (r[0], r[1]), (r[2], r[3]), u)))
    return np.array(out)


def test_arc_clear_golden_and_large_radius(eng, maps):
    use_map(eng, maps, "map2")
    g = O.Grid(maps["map2"])
    rows = golden("f4_arc.npz")["arc_in"]
    assert np.array_equal(eng.arc_clear(rows), _arc_truth(g, rows))
    # large radii exercise the boxed candidate window (K > 64): 30 px arcs on circles of r 90..20000
    rng = np.random.default_rng(8)
    big = []
    for i in range(124):
        rad = float(np.exp(rng.uniform(np.log(90), np.log(3000)))) if i >= 4 else 20000.0 - i
        c = rng.uniform(0, 300, 2)
        a0 = rng.uniform(-np.pi, np.pi)
        sgn = rng.choice([-1.0, 1.0])
        da = sgn * 30.0 / rad * rng.uniform(0.2, 1.0)
        b = c + rad * np.array([np.cos(a0), np.sin(a0)])
        l = c + rad * np.array([np.cos(a0 + da), np.sin(a0 + da)])
        icc = b - rad * np.array([np.cos(a0), np.sin(a0)])
        big.append([b[0], b[1], l[0], l[1], sgn * 30.0, icc[0], icc[1], rad, 30.0, 0.0])
    big = np.array(big)
    keep = (big[:, 0] > -50) & (big[:, 0] < 350)
    big = big[keep]
    assert np.array_equal(eng.arc_clear(big), _arc_truth(g, big))


def test_steer_drive_body_golden(eng, maps):
    use_map(eng, maps, "map2")
    f = golden("f5_steer.npz")
    out = eng.steer(f["steer_in"])
    u = f["steer_u"]
    assert np.array_equal(out[:, 8], u[:, 5])                       # straight branch decisions
    assert np.max(np.abs(out[:, 3] - u[:, 0])) <= TOL                # steer angles
    assert np.max(np.abs(out[:, :3] - f["steer_out"])) <= TOL
    curved = u[:, 5] == 0
    assert np.max(np.abs(out[curved, 4:8] - u[curved, 1:5])) <= TOL
    print("steer bit-exact rows: %.3f" % np.mean(np.all(out[:, :3] == f["steer_out"], axis=1)))
    d_in = f["drive_in"]
    dout, ok = eng.drive(np.c_[d_in[:, :3], d_in[:, 3:8], d_in[:, 8]])
    assert ok.all()
    assert np.max(np.abs(dout - f["drive_out"])) <= TOL
    _, ok = eng.drive(np.array([[5, 5, 0, 0, 0, 0, 0, 1 / 3, 1.0]]))
    assert not ok[0]                                                # TypeError path
    bk = f["bikes"]
    assert np.array_equal(eng.body_clear(bk, 1.0), f["bike_clear"].astype(bool))
    assert np.array_equal(eng.body_clear(bk, 2.0), f["front_clear"].astype(bool))


def _run_native(maps, meta, B):
    builtins.imarray = maps[meta["map"]]
    config.ensure_defaults()
    builtins.K, builtins.tol_xy = meta["K"], meta["tol_xy"]
    try:
        np.random.seed(meta["seed"])
        start = (tuple(meta["start"][0]), meta["start"][1])
        goal = (tuple(meta["goal"][0]), meta["goal"][1])
        return rrt.run(start, goal, batch=B)
    finally:
        builtins.K, builtins.tol_xy = 300, 10


def _check_trace(sol, ex, f, tag):
    assert ex["nodes"].shape == f[tag + "_nodes"].shape
    assert np.array_equal(ex["parent"], f[tag + "_parent"])
    assert np.array_equal(ex["e_off"], f[tag + "_e_off"])
    assert np.array_equal(ex["e_child"], f[tag + "_e_child"])
    assert sol == int(f[tag + "_sol"])
    assert np.max(np.abs(ex["nodes"] - f[tag + "_nodes"])) <= TOL
    fu = f[tag + "_u"]
    assert np.array_equal(ex["u"][:, 5], fu[:, 5])
    # controls: the ICC of a near-singular 2x2 solve (cond up to 1e6, rrt.py:348) carries relative
    # error ~cond*eps, so u is compared relatively; node coordinates above are absolute 1e-6.
    assert np.allclose(ex["u"], fu, rtol=1e-8, atol=TOL)


@pytest.mark.parametrize("tag", ["m1s0", "m1s1", "m1goal", "m2s0"])
def test_rrt_trace_b1_golden(maps, tag):
    meta = golden("f8_meta.json")[tag]
    sol, ex = _run_native(maps, meta, 1)
    _check_trace(sol, ex, golden("f8_rrt.npz"), tag)


def test_rrt_typeerror_golden(maps):
    with pytest.raises(TypeError):
        _run_native(maps, golden("f8_meta.json")["m1s7"], 1)


@pytest.mark.parametrize("tag", ["m1b64", "m1b1", "m2b256", "m1b32g"])
def test_rrt_batch_golden(maps, tag):
    meta = golden("f9_meta.json")[tag]
    sol, ex = _run_native(maps, meta, meta["B"])
    _check_trace(sol, ex, golden("f9_batch.npz"), tag)


def test_rrt_api_dicts(maps):
    """rrt.rrt returns the reference's (sol, G, cameFrom) dict views."""
    meta = golden("f8_meta.json")["m1goal"]
    builtins.imarray = maps["map1"]
    builtins.K, builtins.tol_xy = 1001, 10
    try:
        np.random.seed(meta["seed"])
        sol, G, cameFrom = rrt.rrt(((5, 5), 0.0), ((90, 90), 45.0))
    finally:
        builtins.K, builtins.tol_xy = 300, 10
    f = golden("f8_rrt.npz")
    assert len(G) == len(f["m1goal_nodes"])
    assert sol is not None and cameFrom[((5, 5), 0.0)] is None
    assert sum(len(v) for v in G.values()) == len(f["m1goal_e_child"])


@pytest.mark.parametrize("seed,policy", [(5, "raise"), (5, "reject"), (6, "raise"), (9, "reject")])
def test_batched_rrt_vs_oracle_map2(maps, seed, policy):
    """B=512 snapshot batches on map2 (1.5k samples) against the oracle's batch driver; both raise
    the reference's TypeError together, or (policy "reject") both discard that candidate."""
    meta = dict(map="map2", seed=seed, K=1537, tol_xy=0, start=[[280, 0], -170.0], goal=[[73, 38], 0.0])
    np.random.seed(seed)
    try:
        osol, T = O.rrt_batched(O.Params(K=1537, tol_xy=0), O.Grid(maps["map2"]), ((280, 0), -170.0),
                                ((73, 38), 0.0), B=512, straight=policy)
    except TypeError:
        T = None
    builtins.rrt_straight = policy
    try:
        if T is None:
            with pytest.raises(TypeError):
                _run_native(maps, meta, 512)
            return
        sol, ex = _run_native(maps, meta, 512)
    finally:
        builtins.rrt_straight = "raise"
    nodes = np.array([[n[0][0], n[0][1], n[1]] for n in T.nodes])
    assert ex["nodes"].shape == nodes.shape
    assert np.array_equal(ex["parent"], np.array(T.parent))
    assert np.max(np.abs(ex["nodes"] - nodes)) <= TOL


def test_findnearest_golden_and_api(eng, maps):
    """rrt.py:117-128 on the GPU: the F10 fixture (F8 trees, main.py waypoints, exact ties), the dict
    API rrt.findnearest(G, goal), and an empty tree (the reference's (None, None))."""
    use_map(eng, maps, "map2")
    f = golden("f10_findnearest.npz")
    for tag in ("m1s0", "m2s0", "ties"):
        idx, dist = eng.findnearest(f[tag + "_nodes"], f[tag + "_e_par"], f[tag + "_e_child"],
                                    f[tag + "_goals"])
        assert np.array_equal(idx, f[tag + "_idx"]), tag
        assert np.allclose(dist, f[tag + "_dist"], rtol=0, atol=1e-9), tag
    n, ep, ec = f["ties_nodes"], f["ties_e_par"], f["ties_e_child"]
    keys = [((float(x), float(y)), float(t)) for x, y, t in n]
    G = {k: [] for k in keys}
    for p, c in zip(ep, ec):
        G[keys[p]].append(keys[c])
    for g, i in zip(f["ties_goals"], f["ties_idx"]):
        node, d = rrt.findnearest(G, ((g[0], g[1]), g[2]))
        assert node == keys[i]
    assert rrt.findnearest({((1.0, 2.0), 0.0): []}, ((5, 5), 0.0)) == (None, None)
    idx, dist = eng.findnearest(n, [], [], f["ties_goals"][:2])
    assert list(idx) == [-1, -1]


def test_findnearest_large_and_session(maps):
    """A 100k-edge tree with duplicate children and appended-order edges against the oracle, and
    tr_rrt_findnearest over a live session's tree against the batch entry point."""
    rng = np.random.default_rng(117)
    n = 60000
    nodes = np.c_[rng.uniform(0, 512, (n, 2)), rng.uniform(-180, 180, n)]
    nodes[1000:1100] = nodes[:100]                          # equal distances far apart in order
    ep = np.sort(rng.integers(0, n, 100000))
    ec = rng.integers(0, n, 100000)
    goals = np.c_[rng.uniform(0, 512, (4, 2)), rng.uniform(-180, 180, 4)]
    goals[0] = nodes[50]                                    # exact hits on duplicated poses
    e = _native.Engine()
    e.set_params(_native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1))
    idx, dist = e.findnearest(nodes, ep, ec, goals)
    P = O.Params()
    for g, i, d in zip(goals, idx, dist):
        oi, od = O.findnearest(P, nodes.tolist(), ep, ec, ((g[0], g[1]), g[2]))
        assert i == oi and abs(d - od) <= 1e-9
    # an append log (parents interleaved, each parent's children in order) = the traversal's answer
    r = rng.random(len(ep))
    r = r[np.lexsort((r, ep))]                              # ascending within each parent group
    log = np.argsort(r)
    idx2, dist2 = e.findnearest(nodes, ep[log], ec[log], goals)
    assert np.array_equal(idx2, idx) and np.array_equal(dist2, dist)
    # session: the engine's own tree, all batches committed
    free = maps["map2"]
    e.set_grid(free)
    e.rrt_begin([280.0, 0.0, -170.0], [73.0, 38.0, 0.0])
    G = np.random.RandomState(3).standard_normal((4, 3 * 512))
    for g in G:
        e.rrt_step(g)
    ex = e.book().export()
    ep2 = np.repeat(np.arange(len(ex["nodes"])), np.diff(ex["e_off"]))
    goals2 = np.array([[73, 38, 0], [100, 100, 45], [8, 280, 90]], np.float64)
    want = e.findnearest(ex["nodes"], ep2, ex["e_child"], goals2)
    got = e.rrt_findnearest(goals2)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    e.close()


def test_astar_native_golden(eng, maps):
    """tr_astar (search.py:221-307, one search on the host) against the reference's own runs on
    map2 (F1): lazy Theta* path and expansion count of main.py:57, the A* path, the invalid /
    degenerate cases."""
    use_map(eng, maps, "map2")
    f = golden("f1_astar.json")
    for theta, tag in ((True, "thetastar"), (False, "astar")):
        path, st = eng.astar((280, 0), (8, 280), theta)
        assert path.tolist() == f[tag]["path"], tag
        assert st["expanded"] == f[tag]["expanded"], (tag, st)
        assert (st["los_segments"] == st["expanded"] - 1) == theta    # one test per closed node
    for case in f["invalid"]:
        path, st = eng.astar(tuple(case["start"]), tuple(case["goal"]), True)
        if case["ret"] is False:
            assert path is None and st["status"] == 1
        else:
            assert path.tolist() == case["ret"]
            assert case["msg"] == "Expanded nodes: %d" % st["expanded"]
    path, st = eng.astar((280, 0), (150, 150), True)          # start free, goal on an obstacle
    assert maps["map2"][150, 150] or (path is None and st["status"] == 2)


def test_astar_device_batch_golden_and_host_parity(eng, maps):
    """tr_astar_batch (the search resident on the GPU, one wave per query): the reference's own
    runs on map2 (F1: main.py:57's lazy Theta* path with 30,384 expansions, the A* path, the
    degenerate cases), then random queries on map2, map1, a stroke map and a walled map with an
    unreachable region, each equal to the host search tr_astar in path, expansion count and status
    (free, blocked and out-of-range endpoints included), A* and Theta*."""
    use_map(eng, maps, "map2")
    f = golden("f1_astar.json")
    for theta, tag in ((True, "thetastar"), (False, "astar")):
        paths, st = eng.astar_batch([[280, 0, 8, 280]], theta)
        assert st[0, 3] == 0 and paths[0].tolist() == f[tag]["path"], (tag, st)
        assert st[0, 0] == f[tag]["expanded"], (tag, st)
    for case in f["invalid"]:
        paths, st = eng.astar_batch([list(case["start"]) + list(case["goal"])], True)
        if case["ret"] is False:
            assert paths[0] is None and st[0, 3] == 1
        else:
            assert paths[0].tolist() == case["ret"]
            assert case["msg"] == "Expanded nodes: %d" % st[0, 0]

    rs = np.random.RandomState(8)
    walled = np.ones((96, 96), np.uint8)
    walled[40, :] = 0                                  # nothing below row 40 reaches anything above
    walled[:, 70] = 0
    strokes = workloads.map2_style(160, seed=2).astype(np.uint8)
    for name, grid, nq in (("map2", maps["map2"], 48), ("map1", maps["map1"], 64),
                           ("strokes", strokes, 48), ("walled", walled, 48)):
        eng.set_grid(grid)
        H, W = grid.shape
        q = np.column_stack([rs.randint(-2, H + 2, nq), rs.randint(-2, W + 2, nq),
                             rs.randint(-2, H + 2, nq), rs.randint(-2, W + 2, nq)]).astype(np.int32)
        q[0, 2:] = q[0, :2]                            # start == goal
        for theta in (True, False):
            paths, st = eng.astar_batch(q, theta, cap=2048)
            seen = set()
            for i in range(nq):
                hp, hs = eng.astar((q[i, 0], q[i, 1]), (q[i, 2], q[i, 3]), theta)
                assert st[i, 3] == hs["status"], (name, theta, i, q[i], st[i], hs)
                seen.add(int(st[i, 3]))
                if hs["status"] == 0:
                    assert paths[i].tolist() == hp.tolist(), (name, theta, i, q[i])
                    assert st[i, 0] == hs["expanded"], (name, theta, i, st[i], hs)
                else:
                    assert paths[i] is None
                    if hs["status"] == 3:
                        assert st[i, 0] == hs["expanded"], (name, theta, i, st[i], hs)
            assert 0 in seen, (name, seen)
            if name == "walled":
                assert 3 in seen, seen                 # an exhausted queue: the reference's False
    config.grid_changed()                              # the shared engine's map was replaced here


def test_scalar_lineofsight_host_golden(maps):
    """tr_lineofsight (the scalar API call, host) on the reference's answers (F2)."""
    builtins.imarray = maps["map2"]
    f = golden("f2_los.npz")
    q, r = f["theta_q"], f["theta_r"]
    for i in range(0, len(q), 5):
        a, b, c, d = q[i].tolist()
        assert search.lineofsight((a, b), (c, d)) == bool(r[i])
    for (a, b, c, d), rr in zip(f["rand_seg"].tolist(), f["rand_r"].tolist()):
        assert search.lineofsight((a, b), (c, d)) == bool(rr)


def test_scalar_api_grid_upload_key(maps):
    """config.engine() re-uploads builtins.imarray only when it is another array or marked changed
    (getCircle(draw=True) marks it); the answers follow the map."""
    m = maps["map2"].copy()
    builtins.imarray = m
    seg = ((20, 20), (60, 20))
    clear = O.Grid(m).los(*seg)
    assert search.lineofsight(*seg) == clear
    m[20, 40] = not m[20, 40]                      # in place: invisible until marked
    config.grid_changed()
    assert search.lineofsight(*seg) == O.Grid(m).los(*seg)
    builtins.imarray = maps["map2"]                # another array: uploaded again
    assert search.lineofsight(*seg) == clear


def test_search_api(maps):
    builtins.imarray = maps["map2"]
    f = golden("f1_astar.json")
    assert search.lineofsight((10, 10), (12, 40)) == O.Grid(maps["map2"]).los((10, 10), (12, 40))
    assert search.bresenham((0, 0), (5, 2)) == O.bresenham((0, 0), (5, 2))
    path = search.astar((280, 0), (8, 280))
    assert [list(p) for p in path] == f["main_py_57"]
    assert search.astar((-1, 5), (8, 280)) is False
    many = search.astar_many([((280, 0), (8, 280)), ((-1, 5), (8, 280)), ((280, 0), (8, 280))])
    assert [list(p) for p in many[0]] == f["main_py_57"] and many[1] is False and many[2] == many[0]


def test_pipelined_session_equals_sequential(maps):
    """tr_rrt_pipe_* (NN over the begin snapshot overlapped with the host commit, then a delta sweep)
    builds the same tree as the one-call-per-batch session and as the oracle."""
    import torch
    free = maps["map2"]
    B, nb = 1024, 8
    rs = np.random.RandomState(3)
    G = rs.standard_normal((nb, 3 * B))
    p = _native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1)
    start, goal = [280.0, 0.0, -170.0], [73.0, 38.0, 0.0]

    a = _native.Engine()
    a.set_params(p)
    a.set_grid(free)
    a.rrt_begin(start, goal)
    for g in G:
        a.rrt_step(g)
    ref = a.book().export()

    b = _native.Engine()
    b.set_params(p)
    b.set_grid(free)
    b.rrt_begin(start, goal)
    b.rrt_reserve(20000, B)
    dev = torch.device("cuda", 0)
    gd = torch.from_numpy(G).to(dev)
    samp = torch.empty(B * 16, dtype=torch.uint8, device=dev)
    recs = torch.empty(B * 80, dtype=torch.uint8, device=dev)
    for i in range(nb):
        b.pipe_expand(gd[i].data_ptr(), B, samp.data_ptr(), recs.data_ptr())
        b.pipe_dedupe(samp.data_ptr(), recs.data_ptr(), B)
        if b.pending() > 1:
            b.pipe_commit()
    while b.pending():
        b.pipe_commit()
    got = b.book().export()
    for k in ("nodes", "parent", "u", "e_off", "e_child"):
        assert np.array_equal(got[k], ref[k]), k

    # look-ahead: batch i+1 staged (samples + snapshot NN sweep on the side stream) while batch i
    # expands; alternating sample/record buffers.  One stage is left unmatched and dropped.
    c = _native.Engine()
    c.set_params(p)
    c.set_grid(free)
    c.rrt_begin(start, goal)
    c.rrt_reserve(20000, B)
    samp2 = [torch.empty(B * 16, dtype=torch.uint8, device=dev) for _ in range(2)]
    recs2 = [torch.empty(B * 80, dtype=torch.uint8, device=dev) for _ in range(2)]
    for i in range(nb):
        k = i & 1
        c.pipe_expand(gd[i].data_ptr(), B, samp2[k].data_ptr(), recs2[k].data_ptr())
        if i + 1 < nb:
            nxt = samp2[k ^ 1] if i != 2 else samp
            c.pipe_stage(gd[i + 1].data_ptr(), B, nxt.data_ptr(), recs2[k ^ 1].data_ptr())
        c.pipe_dedupe(samp2[k].data_ptr(), recs2[k].data_ptr(), B)
        if c.pending() > 1:
            c.pipe_commit()
    while c.pending():
        c.pipe_commit()
    got = c.book().export()
    for k in ("nodes", "parent", "u", "e_off", "e_child"):
        assert np.array_equal(got[k], ref[k]), k

    # the native loop (tr_rrt_run) with look-ahead, and with the engine's RCCL communicator (one
    # rank: the all-gather is a copy, the sharded code path runs)
    # (depth 2: two look-aheads in flight, three rotating buffer sets; depth 0: no look-ahead)
    for comm, depth in ((False, 1), (True, 1), (False, 2), (True, 2), (False, 0)):
        d = _native.Engine()
        d.set_params(p)
        d.set_grid(free)
        if comm:
            d.comm_init(0, 1, _native.Engine.comm_unique_id())
        d.rrt_begin(start, goal)
        d.rrt_reserve(20000, B)
        ns = max(2, depth + 1)
        s2 = torch.empty(ns * B * 16, dtype=torch.uint8, device=dev)
        r2 = torch.empty(ns * B * 80, dtype=torch.uint8, device=dev)
        sa = torch.empty(2 * B * 16, dtype=torch.uint8, device=dev)
        ra = torch.empty(2 * B * 80, dtype=torch.uint8, device=dev)
        d.run(gd.data_ptr(), B, nb, s2.data_ptr(), r2.data_ptr(), lag=2, stage=depth,
              d_samples_all=sa.data_ptr() if comm else 0, d_records_all=ra.data_ptr() if comm else 0)
        got = d.book().export()
        for k in ("nodes", "parent", "u", "e_off", "e_child"):
            assert np.array_equal(got[k], ref[k]), (comm, depth, k)

    # ref (the one-call-per-batch rrt_step session) is pinned to the oracle's rrt_batched by
    # test_batched_rrt_vs_oracle_map2; the oracle at 8x1024 samples takes minutes, so it is not re-run here.


def test_two_engine_sharded_session_equals_single(maps):
    """bench.py's multi-GPU step on one device: two engines (ranks) each expand their contiguous
    slice of every batch (with look-ahead staging), the slices are concatenated in rank order (what
    the RCCL all-gather produces) and both engines deduplicate and commit the whole batch: both
    trees equal the one-engine run of the full batch."""
    import torch
    free = maps["map2"]
    B, nb, W = 1024, 6, 2
    G = np.random.RandomState(8).standard_normal((nb, 3 * B))
    p = _native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1)
    start, goal = [280.0, 0.0, -170.0], [73.0, 38.0, 0.0]
    ref = _native.Engine()
    ref.set_params(p)
    ref.set_grid(free)
    ref.rrt_begin(start, goal)
    for g in G:
        ref.rrt_step(g)
    want = ref.book().export()

    dev = torch.device("cuda", 0)
    gd = torch.from_numpy(G).to(dev)
    b = B // W
    engs = []
    for _ in range(W):
        e = _native.Engine()
        e.set_params(p)
        e.set_grid(free)
        e.rrt_begin(start, goal)
        e.rrt_reserve(20000, B)
        engs.append(e)
    samp = [[torch.empty(b * 16, dtype=torch.uint8, device=dev) for _ in range(2)] for _ in range(W)]
    recs = [[torch.empty(b * 80, dtype=torch.uint8, device=dev) for _ in range(2)] for _ in range(W)]
    s_all = [torch.empty(B * 16, dtype=torch.uint8, device=dev) for _ in range(2)]
    r_all = [torch.empty(B * 80, dtype=torch.uint8, device=dev) for _ in range(2)]
    for i in range(nb):
        k = i & 1
        for w, e in enumerate(engs):
            e.pipe_expand(gd[i][3 * b * w:].data_ptr(), b, samp[w][k].data_ptr(), recs[w][k].data_ptr())
            if i + 1 < nb:
                e.pipe_stage(gd[i + 1][3 * b * w:].data_ptr(), b, samp[w][k ^ 1].data_ptr(),
                             recs[w][k ^ 1].data_ptr())
        for e in engs:
            e.sync()
        torch.cuda.synchronize()
        s_all[k].copy_(torch.cat([samp[w][k] for w in range(W)]))
        r_all[k].copy_(torch.cat([recs[w][k] for w in range(W)]))
        torch.cuda.synchronize()
        for e in engs:
            e.pipe_dedupe(s_all[k].data_ptr(), r_all[k].data_ptr(), B)
            e.sync()
            while e.pending() > 1:
                e.pipe_commit()
    for e in engs:
        while e.pending():
            e.pipe_commit()
        got = e.book().export()
        for key in ("nodes", "parent", "u", "e_off", "e_child"):
            assert np.array_equal(got[key], want[key]), key
