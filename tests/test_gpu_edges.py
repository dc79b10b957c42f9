"""GPU edge cases through the C-ABI, each checked against the oracle.

* empty batches (B = 0 / n = 0) return at once; NN on an empty tree is a state error;
* `int()` truncation toward zero at the grid border (search.py:17-24: -0.9 -> 0 is valid, -1.0 is
  not), endpoints far outside the grid, fractional endpoints;
* non-square grids, where `valid` checks x against shape[0] and y against shape[1] (transposed) and
  `imarray[int(y)][int(x)]` raises IndexError (search.py:21,30) — unless `all()` has already
  stopped at an earlier blocked pixel, so the outcome depends on the pixel order of the ray;
* maximum sizes: rays across a whole 2048^2 grid (longer than the kernels' in-register pixel
  budget, so the long-line path runs), and NN with query coordinates at the int32 grid corners.
"""
import numpy as np
import pytest

import pkgload
import thetarrt_oracle as O

pkgload.load()
from theta_rrt_amd import _native, workloads  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    return _native.engine()


def oracle_los(grid, seg):
    """('ok', bool) or ('index', None) for one ray, the reference's lineofsight outcome."""
    try:
        return "ok", grid.los((seg[0], seg[1]), (seg[2], seg[3]))
    except IndexError:
        return "index", None


def engine_los(eng, seg):
    try:
        return "ok", bool(eng.los(np.asarray(seg, np.float64)[None])[0])
    except IndexError:
        return "index", None


def test_empty_batches(eng):
    eng.set_grid(np.ones((8, 8), np.uint8))
    eng.tree_reset(16)
    assert eng.nn(np.zeros((0, 2), np.int32)).shape == (0,)        # B = 0 before any node
    with pytest.raises(_native.NativeError):
        eng.nn(np.zeros((1, 2), np.int32))                          # empty tree
    assert eng.los(np.zeros((0, 4))).shape == (0,)
    eng.tree_append(np.array([[3.0, 4.0, 0.0]]))
    assert eng.nn(np.zeros((0, 2), np.int32)).shape == (0,)
    assert list(eng.nn(np.array([[0, 0], [7, 7]], np.int32))) == [0, 0]


def test_empty_first_step_of_a_fresh_session():
    """tr_rrt_step with B = 0 on a context whose commit slots were never used: the slot is
    allocated before the empty batch's head is written; the tree stays the start node, and the
    next real batch runs as usual."""
    e = _native.Engine(0)
    e.set_grid(np.ones((64, 64), np.uint8))
    e.rrt_begin([5.0, 5.0, 0.0], [40.0, 40.0, 0.0])
    n, sol = e.rrt_step(np.zeros(0))
    assert (n, sol) == (1, -1)
    n, sol = e.rrt_step(np.random.RandomState(0).standard_normal(3 * 64))
    assert n > 1 and e.book().size() == n
    e.close()


def test_nn_batch_returns_squared_distance(eng):
    rs = np.random.RandomState(12)
    eng.set_grid(np.ones((300, 300), np.uint8))
    tree = np.column_stack([rs.uniform(0, 300, 5000), rs.uniform(0, 300, 5000), np.zeros(5000)])
    eng.tree_reset(8192)
    eng.tree_append(tree)
    q = rs.randint(0, 300, (777, 2)).astype(np.int32)
    idx, d2 = eng.nn(q, d2=True)
    want = O.nn_numpy(tree[:, 0], tree[:, 1], q[:, 0], q[:, 1])
    assert np.array_equal(idx, want)
    dx, dy = q[:, 0] - tree[idx, 0], q[:, 1] - tree[idx, 1]
    assert np.array_equal(d2, dx * dx + dy * dy)          # the fp64 sum L2norm takes the root of


def test_los_border_truncation(eng):
    free = np.ones((16, 16), bool)
    free[5, 9] = False
    g = O.Grid(free)
    eng.set_grid(free.astype(np.uint8))
    rng = np.random.default_rng(3)
    segs = [(-0.9, -0.9, 15.9, 15.9), (-1.0, 0.0, 5.0, 5.0), (0.0, -1.0, 5.0, 5.0),
            (15.99, 0.0, 15.99, 15.99), (16.0, 3.0, 2.0, 3.0), (-0.5, 5.0, 15.5, 5.0),
            (9.7, 5.2, 9.1, 5.9), (3.5, 3.5, 3.5, 3.5), (-20.0, -20.0, 40.0, 40.0)]
    segs += [tuple(r) for r in rng.uniform(-3, 19, size=(400, 4))]
    segs += [tuple(r) for r in rng.integers(-2, 18, size=(400, 4)).astype(np.float64)]
    segs = np.array(segs)
    want = np.array([oracle_los(g, s)[1] for s in segs])
    assert np.array_equal(eng.los(segs), want)


@pytest.mark.parametrize("shape", [(24, 40), (40, 24)])
def test_los_non_square_index_error(eng, shape):
    """H != W: each ray alone, so that the IndexError (a whole-batch error, as the reference raises
    on the first such ray) is attributed to the ray that causes it."""
    H, W = shape
    rng = np.random.default_rng(H)
    free = rng.random((H, W)) > 0.04
    g = O.Grid(free)
    eng.set_grid(free.astype(np.uint8))
    m = max(H, W) + 4
    segs = np.r_[rng.uniform(-2, m, size=(300, 4)),
                 rng.integers(0, min(H, W), size=(100, 4)).astype(np.float64)]
    kinds = {"ok": 0, "index": 0}
    for s in segs:
        o = oracle_los(g, s)
        kinds[o[0]] += 1
        assert engine_los(eng, s) == o, s
    assert kinds["index"] > 0 and kinds["ok"] > 0
    # a batch of rays that all stay inside min(H, W) equals the per-ray oracle
    inside = rng.uniform(0, min(H, W) - 0.01, size=(500, 4))
    assert np.array_equal(eng.los(inside), [g.los(s[:2], s[2:]) for s in inside])


def _arc_outcome(fn):
    try:
        return "ok", fn()
    except IndexError:
        return "index", None


@pytest.mark.parametrize("shape", [(24, 40), (40, 24)])
def test_straight_arc_check_non_square_eager(eng, shape):
    """rrt.py:173-174 for a straight control: `False in [freespace(px) for px in bresenham(..)]`
    tests every pixel, so a pixel past a blocked one still raises IndexError on a non-square map
    (lineofsight, by contrast, stops at the first blocked pixel)."""
    H, W = shape
    rng = np.random.default_rng(7 + H)
    free = rng.random((H, W)) > 0.08
    g = O.Grid(free)
    eng.set_grid(free.astype(np.uint8))
    m = max(H, W) + 2
    segs = rng.uniform(0, m, size=(400, 4))
    kinds = {"ok": 0, "index": 0}
    blocked_then_raise = 0
    for s in segs:
        want = _arc_outcome(lambda: not (False in [g.freespace(p) for p in O.bresenham(s[:2], s[2:])]))
        row = np.array([s[0], s[1], s[2], s[3], 0.0, 0.0, 0.0, 0.0, 1.0, 1.0])
        got = _arc_outcome(lambda: bool(eng.arc_clear(row[None])[0]))
        assert got == want, s
        kinds[want[0]] += 1
        if want[0] == "index" and oracle_los(g, s) == ("ok", False):
            blocked_then_raise += 1                  # the case lineofsight semantics would miss
    assert kinds["index"] > 0 and kinds["ok"] > 0 and blocked_then_raise > 0, (kinds, blocked_then_raise)


def test_los_long_rays_2048(eng):
    free = workloads.map2_style(2048, seed=1)
    g = O.Grid(free)
    eng.set_grid(free.astype(np.uint8))
    rng = np.random.default_rng(11)
    segs = np.r_[[(0.0, 0.0, 2047.0, 2047.0), (2047.0, 0.0, 0.0, 2047.0), (0.0, 1000.0, 2047.0, 1000.0),
                  (1000.0, 0.0, 1000.0, 2047.0), (0.0, 0.0, 2047.0, 1.0), (-0.5, -0.5, 2047.9, 2047.9)],
                 rng.uniform(0, 2048, size=(120, 4))]
    # free corridors so that long clear rays occur too
    for s in segs[:6]:
        for px in O.bresenham((s[0], s[1]), (s[2], s[3])):
            if g.valid(px):
                free[int(px[1]), int(px[0])] = True
    g = O.Grid(free)
    eng.set_grid(free.astype(np.uint8))
    want = np.array([g.los(s[:2], s[2:]) for s in segs])
    assert want[:6].all() and not want.all()
    assert np.array_equal(eng.los(segs), want)
    assert np.array_equal(eng.los(segs[:, [2, 3, 0, 1]]), want)


def test_nn_extreme_queries(eng):
    """Queries at the grid corners and far outside it against a tree spread over [0, 2048), from
    the sweep (the default for a tree this sparse) and from the cell lists."""
    eng.set_grid(np.ones((2048, 2048), np.uint8))
    rng = np.random.default_rng(8)
    xy = rng.uniform(0, 2048, size=(70000, 2))
    eng.tree_reset(len(xy))
    eng.tree_append(np.c_[xy, np.zeros(len(xy))])
    q = np.r_[[[0, 0], [2047, 2047], [0, 2047], [2047, 0], [-5000, 9000], [100000, -100000]],
              rng.integers(0, 2048, size=(2000, 2))].astype(np.int32)
    want = O.nn_numpy(xy[:, 0], xy[:, 1], q[:, 0], q[:, 1])
    assert np.array_equal(eng.nn(q), want)
    old = [(k, eng.get_option(k)) for k in ("nn_grid_min", "nn_far_sweep")]
    try:
        for far in (1 << 40, 0):
            eng.set_option("nn_grid_min", 0)
            eng.set_option("nn_far_sweep", far)
            assert np.array_equal(eng.nn(q), want), far
    finally:
        for k, v in old:
            eng.set_option(k, v)


def test_nn_nonsquare_map_both_paths(eng):
    """Nearest nodes on a map whose sides differ (the cell lists pad it to a square of cells),
    nodes beyond every edge, queries inside and outside: the cell lists and the sweep agree with
    numpy's argmin."""
    eng.set_grid(np.ones((300, 700), np.uint8))
    rng = np.random.default_rng(12)
    xy = np.c_[rng.uniform(-20, 320, 30000), rng.uniform(-20, 720, 30000)]
    eng.tree_reset(len(xy))
    eng.tree_append(np.c_[xy, np.zeros(len(xy))])
    q = np.r_[np.c_[rng.integers(0, 300, 1500), rng.integers(0, 700, 1500)],
              [[0, 0], [299, 699], [0, 699], [299, 0], [-50, 350], [400, 800], [150, -90]]].astype(np.int32)
    want = O.nn_numpy(xy[:, 0], xy[:, 1], q[:, 0], q[:, 1])
    old = [(k, eng.get_option(k)) for k in ("nn_grid", "nn_grid_min", "nn_far_sweep")]
    try:
        for grid, far in ((1, 1 << 40), (1, 0), (0, 0)):
            eng.set_option("nn_grid", grid)
            eng.set_option("nn_grid_min", 0)
            eng.set_option("nn_far_sweep", far)
            assert np.array_equal(eng.nn(q), want), (grid, far)
    finally:
        for k, v in old:
            eng.set_option(k, v)


def _dup_source(seed, stride=3, offsets=(256, 400, 130)):
    """The legacy gaussian stream of `seed`, with sample k of every batch copied onto samples
    k + off (other 256-record blocks of the one-kernel dedupe k_dd, and the same block)."""
    rs = np.random.RandomState(seed)

    def src(n):
        g = rs.standard_normal(n).reshape(-1, 3)
        for k in range(0, min(len(g), 256), stride):
            for off in offsets:
                if k + off < len(g):
                    g[k + off] = g[k]
        return g.reshape(-1)
    return src


def test_duplicate_samples_across_dedupe_blocks(maps):
    """Copies of samples inside one batch: the same new pose from several records, first
    occurrences in earlier k_dd blocks, members re-reached.  Node indices, parents, controls and
    edge lists equal the oracle's batched driver (rrt.py:151,179-188)."""
    import builtins
    from theta_rrt_amd import config, rrt
    free = maps["map2"]
    B, K = 512, 1 + 2 * 512
    start, goal = ((280, 0), -170.0), ((73, 38), 0.0)
    _, T = O.rrt_batched(O.Params(K=K, tol_xy=0), O.Grid(free), start, goal, B=B,
                         gauss_source=_dup_source(21), straight="reject")
    builtins.imarray = free
    config.ensure_defaults()
    builtins.K, builtins.tol_xy, builtins.rrt_straight = K, 0, "reject"
    try:
        sol, ex = rrt.run(start, goal, batch=B, gauss_source=_dup_source(21))
    finally:
        builtins.K, builtins.tol_xy, builtins.rrt_straight = 300, 10, "raise"
    nodes = np.array([[n[0][0], n[0][1], n[1]] for n in T.nodes])
    assert ex["nodes"].shape == nodes.shape and len(nodes) > 500
    assert np.array_equal(ex["parent"], np.array(T.parent))
    assert np.max(np.abs(ex["nodes"] - nodes)) <= 1e-6
    for i in range(len(nodes)):
        assert list(ex["e_child"][ex["e_off"][i]:ex["e_off"][i + 1]]) == T.children[i], i
    dup_edges = sum(len(c) for c in T.children) - (len(nodes) - 1)
    assert dup_edges > 100                    # the copies did re-reach nodes of the same batch
