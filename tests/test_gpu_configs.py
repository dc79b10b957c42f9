"""GPU parity at the sizes of BASELINE.json configs 3 and 5, through the C-ABI.

cfg3 = 2048x2048 map2-style grid, 65536 samples per batch, a tree of ~1M nodes.  The oracle cannot
expand 65536 samples in seconds, so these tests check:
  * the nearest-node sweep over a frozen 1M-node tree for all 65536 queries against an independent
    fp64 argmin (torch on the GPU, first index of the smallest sqrt), and 64 queries against the
    oracle's own arithmetic (oracle.nn_numpy);
  * full batches: the pipelined native loop (look-ahead + delta) builds the same tree as the
    one-call-per-batch session, and a random subset of one batch's records equals the oracle's
    per-sample expansion (rrt.py:144-176) against the same snapshot;
  * cfg5's sharding: W engines expanding contiguous slices of every batch and deduplicating the
    concatenation in rank order build the single-engine tree (W = 8 here, on one device).
"""
import numpy as np
import pytest

import pkgload
import thetarrt_oracle as O

pkgload.load()
from theta_rrt_amd import _native, workloads  # noqa: E402

pytestmark = pytest.mark.gpu
TOL = 1e-6
P_NATIVE = (5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1)     # main.py defaults, tol_xy 0, reject


def _torch_nn(xy, q, chunk=32):
    """First index of the smallest fp64 sqrt distance (the reference's argmin), on the GPU."""
    import torch
    dev = torch.device("cuda", 0)
    tx = torch.from_numpy(np.ascontiguousarray(xy[:, 0])).to(dev)
    ty = torch.from_numpy(np.ascontiguousarray(xy[:, 1])).to(dev)
    ar = torch.arange(len(xy), device=dev)
    out = np.empty(len(q), np.int64)
    qd = torch.from_numpy(q.astype(np.float64)).to(dev)
    for s in range(0, len(q), chunk):
        a = qd[s:s + chunk, 0:1] - tx[None, :]
        b = qd[s:s + chunk, 1:2] - ty[None, :]
        r = torch.sqrt(a * a + b * b)
        m = r.min(dim=1, keepdim=True).values
        out[s:s + chunk] = torch.where(r == m, ar[None, :], len(xy)).min(dim=1).values.cpu().numpy()
    return out


def test_cfg3_nn_1m_nodes():
    rng = np.random.default_rng(33)
    N, B, n = 1_000_000, 65536, 2048
    xy = rng.uniform(0, n, size=(N, 2))
    xy[500000:500512] = xy[:512]                         # equal distances across far-apart chunks
    xy[700000:704000] = rng.integers(0, n, size=(4000, 2))   # integral nodes: exact ties
    eng = _native.Engine()
    eng.set_params(_native.tr_params(*P_NATIVE))
    eng.set_grid(np.ones((n, n), np.uint8))
    eng.tree_reset(N)
    eng.tree_append(np.c_[xy, np.zeros(N)])
    q = rng.integers(0, n, size=(B, 2))
    q[:4000] = xy[700000:704000].astype(np.int64)        # queries sitting on integral nodes
    got = eng.nn(q)
    sel = rng.choice(B, 64, replace=False)
    assert np.array_equal(got[sel], O.nn_numpy(xy[:, 0], xy[:, 1], q[sel, 0], q[sel, 1]))
    want = _torch_nn(xy, q)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (len(bad), bad[:5])


def _session(free, start, goal, B, reserve):
    e = _native.Engine()
    e.set_params(_native.tr_params(*P_NATIVE))
    e.set_grid(free)
    e.rrt_begin(start, goal)
    e.rrt_reserve(reserve, B)
    return e


def test_cfg3_batches_pipelined_and_oracle_subset():
    import torch
    n, B, nb = 2048, 65536, 6
    free = workloads.map2_style(n, seed=3)
    sx, sy = workloads.nearest_free(free, 64, 64)
    start, goal = [float(sx), float(sy), 0.0], [n / 2, n / 2, 0.0]
    G = np.random.RandomState(31).standard_normal((nb + 1, 3 * B))

    a = _session(free, start, goal, B, 600000)
    for g in G[:nb]:
        a.rrt_step(g)
    ref = a.book().export()
    assert len(ref["nodes"]) > 50000

    dev = torch.device("cuda", 0)
    gd = torch.from_numpy(G[:nb]).to(dev)
    for depth in (1, 2):
        b = _session(free, start, goal, B, 600000)
        ns = depth + 1 if depth > 1 else 2
        s2 = torch.empty(ns * B * 16, dtype=torch.uint8, device=dev)
        r2 = torch.empty(ns * B * 80, dtype=torch.uint8, device=dev)
        b.run(gd.data_ptr(), B, nb, s2.data_ptr(), r2.data_ptr(), lag=3, stage=depth)
        got = b.book().export()
        for k in ("nodes", "parent", "u", "e_off", "e_child"):
            assert np.array_equal(got[k], ref[k]), (depth, k)

    # one more batch on `a`, its records read back and a subset re-expanded by the oracle
    snap = ref["nodes"]
    g7 = torch.from_numpy(G[nb]).to(dev)
    smp = torch.empty(B * 16, dtype=torch.uint8, device=dev)
    rec = torch.empty(B * 80, dtype=torch.uint8, device=dev)
    a.pipe_expand(g7.data_ptr(), B, smp.data_ptr(), rec.data_ptr())
    a.sync()
    torch.cuda.synchronize()
    R = rec.cpu().numpy().view(_native.RECORD_DTYPE)
    P = O.Params(K=10, tol_xy=0)
    qs = O.samples_from_gauss(P, free.shape, ((n / 2, n / 2), 0.0), G[nb])
    keys = {(float(x), float(y), float(t)) for x, y, t in snap}
    grid = O.Grid(free)
    poses = [((x, y), t) for x, y, t in snap]
    rng = np.random.default_rng(7)
    checked = 0
    for j in rng.permutation(B):
        if checked == 24:
            break
        qx, qy = qs[j][0]
        if (float(qx), float(qy), float(qs[j][1])) in keys:
            continue                                     # a member sample: decided in the dedupe
        r = R[j]
        if r["status"] in (_native.ST_OK, _native.ST_COLLISION) and abs(r["rad"]) > 400:
            continue                                     # the oracle walks the whole circle
        nn = int(O.nn_numpy(snap[:, 0], snap[:, 1], [qx], [qy])[0])
        e = O.expand_one(P, grid, poses, qs[j], nn)
        want = {"blocked_sample": _native.ST_SKIP, "collision": _native.ST_COLLISION,
                "ok": _native.ST_OK, "straight_drive": _native.ST_STRAIGHT}[e.status]
        assert r["status"] == want, (j, e.status, r["status"])
        if e.status != "blocked_sample":
            assert r["near"] == nn, j
        if e.status in ("ok", "collision"):
            assert abs(r["x"] - e.qnew[0][0]) <= TOL and abs(r["y"] - e.qnew[0][1]) <= TOL, j
            assert abs(r["th"] - e.qnew[1]) <= TOL, j
        checked += 1
    assert checked == 24


def test_cfg5_sharded_w8_equals_single():
    """cfg5's scheme at reduced size: 8 ranks (engines on one device) expand contiguous slices of
    each batch; the rank-order concatenation (what the RCCL all-gather yields) deduplicated by
    every rank gives every rank the single-engine tree."""
    import torch
    n, W, b, nb = 1024, 8, 512, 5
    B = W * b
    free = workloads.map2_style(n, seed=5)
    sx, sy = workloads.nearest_free(free, 40, 40)
    start, goal = [float(sx), float(sy), 0.0], [n / 2, n / 2, 0.0]
    G = np.random.RandomState(55).standard_normal((nb, 3 * B))
    ref = _session(free, start, goal, B, 100000)
    for g in G:
        ref.rrt_step(g)
    want = ref.book().export()

    dev = torch.device("cuda", 0)
    gd = torch.from_numpy(G).to(dev)
    engs = [_session(free, start, goal, B, 100000) for _ in range(W)]
    samp = [torch.empty(b * 16, dtype=torch.uint8, device=dev) for _ in range(W)]
    recs = [torch.empty(b * 80, dtype=torch.uint8, device=dev) for _ in range(W)]
    for i in range(nb):
        for w, e in enumerate(engs):
            e.pipe_expand(gd[i][3 * b * w:].data_ptr(), b, samp[w].data_ptr(), recs[w].data_ptr())
        for e in engs:
            e.sync()
        torch.cuda.synchronize()
        s_all = torch.cat(samp)
        r_all = torch.cat(recs)
        torch.cuda.synchronize()
        for e in engs:
            e.pipe_dedupe(s_all.data_ptr(), r_all.data_ptr(), B)
            e.sync()
            while e.pending():
                e.pipe_commit()
    for e in engs:
        got = e.book().export()
        for k in ("nodes", "parent", "u", "e_off", "e_child"):
            assert np.array_equal(got[k], want[k]), k
