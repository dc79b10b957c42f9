"""GPU parity on the configurations bench.py measures (BASELINE.json configs 2 and 5).

cfg2: the bench workload itself (workloads.map2_style(512, 0), B = 4096, start/goal as bench.py,
engine-drawn gaussians), grown by the native loop to both ends of the bench's timed tree range
(46k and 96k nodes); then one more batch whose records are checked against the oracle's per-sample
expansion (rrt.py:144-176) on a random subset, against the same snapshot.

cfg5: the native sharded loop (tr_rrt_run's sharded branch: per-batch all-gather of every rank's
records in rank order, dedupe over the global batch, look-ahead, lagged commits), every rank a
process on one GPU with the exchange through gloo (tr_comm_init_host; RCCL cannot put two ranks on
one device): at cfg5's own shape (world = 8, 2048^2 grid, 65536 samples per rank = 524288 per
global batch, the replicated tree grown past 1M nodes and then three more global batches), at
world = 2 with the same per-rank shape, and at world = 4 with small batches.  Every rank's tree
must equal the single-engine tree of the same global batches.
"""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT  # noqa: F401
import pkgload
import thetarrt_oracle as O

pkgload.load()
from theta_rrt_amd import _native, workloads  # noqa: E402

pytestmark = pytest.mark.gpu
TOL = 1e-6
P_NATIVE = (5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1)     # bench.py's parameters
KEYS = ("nodes", "parent", "u", "e_off", "e_child")


def _engine(free, start3, goal3, seed, reserve, batch):
    e = _native.Engine(0)
    e.set_params(_native.tr_params(*P_NATIVE))
    e.set_grid(free)
    e.rrt_begin(start3, goal3)
    e.rrt_reserve(reserve, batch)
    e.rng_set_state(np.random.RandomState(seed).get_state())
    return e


@pytest.mark.parametrize("grow_to", [46000, 96000])
def test_cfg2_bench_workload_oracle_subset(grow_to):
    """The bench's own workload at both ends of its timed tree range: the next batch of its stream
    against the oracle, sample by sample on a random subset that includes member samples (the
    record must carry TR_FL_MEMBER) and arcs of every radius (a few of the largest: the oracle
    walks the whole circle)."""
    import torch
    cfg = workloads.CONFIGS["cfg2"]
    n, B = cfg["grid"], cfg["batch"]
    free = workloads.map2_style(n, seed=0)
    sx, sy = workloads.nearest_free(free, cfg["start"], cfg["start"])
    start3, goal3 = [float(sx), float(sy), 0.0], [n / 2, n / 2, 0.0]
    e = _engine(free, start3, goal3, 0, 150000, B)
    dev = torch.device("cuda", 0)
    s2 = torch.empty(2 * B * 16, dtype=torch.uint8, device=dev)
    r2 = torch.empty(2 * B * 80, dtype=torch.uint8, device=dev)
    nodes = 1
    while nodes < grow_to:
        nodes, _ = e.run(None, B, 2, s2.data_ptr(), r2.data_ptr(), lag=4, stage=1)
    assert grow_to <= nodes < grow_to + 8000
    snap = e.book().nodes()
    assert len(snap) == nodes

    # the next batch of the bench's stream, drawn on the device, expanded against the snapshot
    g = torch.empty(3 * B, dtype=torch.float64, device=dev)
    e.rng_gauss_dev(3 * B, g.data_ptr())
    smp = torch.empty(B * 16, dtype=torch.uint8, device=dev)
    rec = torch.empty(B * 80, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    e.pipe_expand(g.data_ptr(), B, smp.data_ptr(), rec.data_ptr())
    e.sync()
    torch.cuda.synchronize()
    G = g.cpu().numpy()
    R = rec.cpu().numpy().view(_native.RECORD_DTYPE)
    S = smp.cpu().numpy().view(_native.SAMPLE_DTYPE)
    P = O.Params(K=10, tol_xy=0)
    qs = O.samples_from_gauss(P, free.shape, (tuple(goal3[:2]), goal3[2]), G)
    assert np.array_equal(S["x"], [q[0][0] for q in qs]) and np.array_equal(S["th"], [q[1] for q in qs])
    keys = {(float(x), float(y), float(t)) for x, y, t in snap}
    grid = O.Grid(free)
    poses = [((x, y), t) for x, y, t in snap]
    rng = np.random.default_rng(2)
    checked, huge = {}, 0
    order = list(rng.permutation(B))
    # the widest arcs of the batch first (radius 1e3 .. 2e4 px: the box-clipped candidate walk)
    wide = [j for j in np.argsort(-np.abs(R["rad"])) if R[j]["status"] in (_native.ST_OK, _native.ST_COLLISION)][:3]
    for j in wide + order:
        if sum(checked.values()) == 43:
            break
        qx, qy = qs[j][0]
        r = R[j]
        member = (float(qx), float(qy), float(qs[j][1])) in keys
        assert bool(r["flags"] & _native.FL_MEMBER) == member, j      # rrt.py:151, decided on the GPU
        if r["status"] in (_native.ST_OK, _native.ST_COLLISION) and abs(r["rad"]) > 400:
            if huge == 3:
                continue                                 # the oracle walks the whole circle: a few
            huge += 1
        nn = int(O.nn_numpy(snap[:, 0], snap[:, 1], [qx], [qy])[0])
        x = O.expand_one(P, grid, poses, qs[j], nn)
        want = {"blocked_sample": _native.ST_SKIP, "collision": _native.ST_COLLISION,
                "ok": _native.ST_OK, "straight_drive": _native.ST_STRAIGHT}[x.status]
        assert r["status"] == want, (j, x.status, r["status"])
        if x.status != "blocked_sample":
            assert r["near"] == nn, j
        if x.status in ("ok", "collision"):
            assert abs(r["x"] - x.qnew[0][0]) <= TOL and abs(r["y"] - x.qnew[0][1]) <= TOL, j
            assert abs(r["th"] - x.qnew[1]) <= TOL, j
            assert bool(r["flags"] & _native.FL_DROVE) == bool(x.drove), j
        checked[x.status] = checked.get(x.status, 0) + 1
    assert sum(checked.values()) == 43 and checked.get("ok", 0) >= 10 and huge >= 1, (checked, huge)


# ------------------------------------------------------------------ sharded native loop
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _case(name):
    if name == "cfg5_w8":      # BASELINE.json configs[4] as specified: 8 ranks x 65536 samples,
        # a replicated tree of >= 1M nodes (grown by the sharded loop itself), then 3 global batches
        return dict(world=8, grid=2048, b=65536, rows=3, grow_to=1_000_000, stage=0, lag=2,
                    seed=5, start=64, reserve=3_200_000)
    if name == "cfg5_w2":      # cfg5's per-rank shape: 2048^2 grid, 65536 samples per rank
        return dict(world=2, grid=2048, b=65536, rows=10, stage=1, lag=4, seed=5, start=64)
    if name == "cfg2_w4_s0":   # bench.py's N > 2 setting: no look-ahead, cfg2's per-rank batch
        return dict(world=4, grid=512, b=4096, rows=12, stage=0, lag=4, seed=3, start=32)
    return dict(world=4, grid=512, b=1024, rows=24, stage=2, lag=3, seed=9, start=16)


def _inputs(c):
    free = workloads.map2_style(c["grid"], seed=c["seed"])
    sx, sy = workloads.nearest_free(free, c["start"], c["start"])
    return free, [float(sx), float(sy), 0.0], [c["grid"] / 2, c["grid"] / 2, 0.0]


def _run(e, c, B, world):
    import torch
    dev = torch.device("cuda", 0)
    ns = max(2, c["stage"] + 1)
    s2 = torch.empty(ns * B * 16, dtype=torch.uint8, device=dev)
    r2 = torch.empty(ns * B * 80, dtype=torch.uint8, device=dev)
    sa = ra = None
    if world > 1:
        sa = torch.empty(2 * B * world * 16, dtype=torch.uint8, device=dev)
        ra = torch.empty(2 * B * world * 80, dtype=torch.uint8, device=dev)
    def go(rows):
        return e.run(None, B, rows, s2.data_ptr(), r2.data_ptr(), lag=c["lag"], stage=c["stage"],
                     d_samples_all=sa.data_ptr() if sa is not None else 0,
                     d_records_all=ra.data_ptr() if ra is not None else 0)
    n, grown = 1, 0
    while n < c.get("grow_to", 0):                    # every replica sees the same count
        n, _ = go(1)
        grown += 1
        assert grown <= 12, "the tree does not reach grow_to"
    before = n
    n, sol = go(c["rows"])
    return n, sol, (grown, before)


def _rank(rank, name, port, out):
    import torch
    import torch.distributed as dist
    c = _case(name)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=c["world"])
    torch.cuda.set_device(0)
    free, start3, goal3 = _inputs(c)

    def gather(buf):
        t = torch.frombuffer(bytearray(buf), dtype=torch.uint8)
        parts = [torch.empty_like(t) for _ in range(c["world"])]
        dist.all_gather(parts, t)
        return b"".join(p.numpy().tobytes() for p in parts)

    # (the communicator first: tr_rrt_reserve sizes the per-rank scratch from the world size)
    e = _native.Engine(0)
    e.set_params(_native.tr_params(*P_NATIVE))
    e.set_grid(free)
    e.comm_init_host(rank, c["world"], gather)
    book = not (name == "small_w4" and rank % 2)      # small_w4: odd ranks keep no host book
    e.set_option("book", 1 if book else 0)
    e.rrt_begin(start3, goal3)
    e.rrt_reserve(c.get("reserve", 2_000_000), c["b"] * c["world"])
    e.rng_set_state(np.random.RandomState(c["seed"]).get_state())
    n, sol, grown = _run(e, c, c["b"], c["world"])
    st = e.rng_get_state()
    ex = e.book().export() if book else {}
    np.savez(out % rank, n=n, sol=sol, grown=grown, book=book, key=st[1], pos=st[2], **ex)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name", ["cfg5_w8", "cfg5_w2", "small_w4", "cfg2_w4_s0"])
def test_native_sharded_loop_equals_single_engine(tmp_path, name):
    import torch.multiprocessing as mp
    c = _case(name)
    out = str(tmp_path / "rank%d.npz")
    mp.spawn(_rank, args=(name, _free_port(), out), nprocs=c["world"], join=True)

    free, start3, goal3 = _inputs(c)
    BT = c["b"] * c["world"]
    ref = _engine(free, start3, goal3, c["seed"], c.get("reserve", 2_000_000), BT)
    n, sol, grown = _run(ref, c, BT, 1)
    want = ref.book().export()
    st = ref.rng_get_state()
    assert n > 1 + c["rows"] * BT // 10, n           # the batches did grow the tree
    if "grow_to" in c:                               # the last c["rows"] batches saw >= grow_to nodes
        assert grown[1] >= c["grow_to"], grown
    for r in range(c["world"]):
        got = np.load(out % r)
        assert int(got["n"]) == n and int(got["sol"]) == sol and tuple(got["grown"]) == grown, r
        if bool(got["book"]):
            for k in KEYS:
                assert np.array_equal(got[k], want[k]), (r, k)
        assert np.array_equal(got["key"], st[1]) and int(got["pos"]) == st[2], r
    ref.close()


def test_pipelined_first_batches_without_reserve_many_seeds():
    """Regression: lazily allocated device scratch (the dedupe's batch tables on the first batch of a
    session without tr_rrt_reserve) must be cleared in stream order.  A clear on the legacy null
    stream raced the first dedupe (about 1 run in 12 diverged in batch 0)."""
    import torch
    free = np.ones((128, 128), np.uint8)
    B, rows = 256, 8
    dev = torch.device("cuda", 0)

    def fresh():
        e = _native.Engine(0)
        e.set_params(_native.tr_params(*P_NATIVE))
        e.set_grid(free)
        e.rrt_begin([10.0, 10.0, 0.0], [60.0, 60.0, 0.0])
        return e
    for seed in range(16):
        G = np.random.RandomState(seed).standard_normal((rows, 3 * B))
        a = fresh()
        for g in G:
            a.rrt_step(g)
        want = a.book().export()
        b = fresh()
        b.rng_set_state(np.random.RandomState(seed).get_state())
        s2 = torch.empty(3 * B * 16, dtype=torch.uint8, device=dev)
        r2 = torch.empty(3 * B * 80, dtype=torch.uint8, device=dev)
        b.run(None, B, rows, s2.data_ptr(), r2.data_ptr(), lag=5, stage=1 + seed % 2)
        got = b.book().export()
        for k in KEYS:
            assert np.array_equal(got[k], want[k]), (seed, k)
        a.close()
        b.close()


def test_pipelined_cell_lists_from_the_first_node_many_seeds():
    """The look-ahead's cell lists merged batch after batch from a one-node tree (several changes of
    the cell size on the way, samples far from a sparse tree: descents, refined block-wide passes),
    with and without the far list: the pipelined run builds the tree of the step-by-step session
    whose nearest nodes come from the sweep."""
    import torch
    free = workloads.map2_style(256, seed=9)
    B, rows = 512, 24
    dev = torch.device("cuda", 0)

    def fresh(opts):
        e = _native.Engine(0)
        e.set_params(_native.tr_params(*P_NATIVE))
        e.set_grid(free)
        for k, v in opts.items():
            e.set_option(k, v)
        e.rrt_begin([20.0, 20.0, 0.0], [128.0, 128.0, 0.0])
        return e
    for seed in range(6):
        G = np.random.RandomState(seed).standard_normal((rows, 3 * B))
        a = fresh({"nn_grid": 0})
        for g in G:
            a.rrt_step(g)
        want = a.book().export()
        a.close()
        assert len(want["parent"]) > 2000
        for far in (1 << 40, 0):
            b = fresh({"nn_grid_min": 0, "nn_far_sweep": far, "nn_far_nodes": 300})
            b.rng_set_state(np.random.RandomState(seed).get_state())
            s2 = torch.empty(3 * B * 16, dtype=torch.uint8, device=dev)
            r2 = torch.empty(3 * B * 80, dtype=torch.uint8, device=dev)
            b.run(None, B, rows, s2.data_ptr(), r2.data_ptr(), lag=4, stage=1 + seed % 2)
            got = b.book().export()
            for k in KEYS:
                assert np.array_equal(got[k], want[k]), (seed, far, k)
            # (a head that reached the host after its ready flag was waited for, never replayed)
            assert 0 <= b.get_option("head_waits") <= rows
            b.close()


@pytest.mark.parametrize("opt", [("gate", 0), ("dd_gatefold", 0), ("dd_fused", 0), ("fused_delta", 0),
                                 ("delta_bins", 0), ("nn_grid", 0), ("nn_grid_min", 0), ("nn_far_sweep", 0)])
def test_pipeline_edge_modes_equal(opt):
    """The pipelined loop under its alternative edges and dedupe paths (event edges, what a context
    created under rocprofv3 --pmc uses; a k_gate launch instead of the gate inside k_dd; the
    three-kernel dedupe; the look-ahead correction as its own kernel, or scanning every appended
    node instead of the bins around each sample; nearest nodes from the sweep of every node only, or
    from the cell lists from the first node on instead of from a tree dense enough on its map,
    or with the far samples of every batch handed to the sweep) builds the same tree as the default loop on the same np.random stream."""
    import torch
    free = workloads.map2_style(512, seed=4)
    B, rows = 2048, 14
    dev = torch.device("cuda", 0)

    def run(option):
        e = _engine(free, [20.0, 20.0, 0.0], [256.0, 256.0, 0.0], 17, 200000, B)
        if e.get_option("gate") != 1:             # (the probe of tr_create: two streams' kernels
            e.close()                             # did not run at the same time in this process)
            pytest.skip("this context got event edges: the gate modes cannot be compared here")
        if option:
            e.set_option(*option)
            assert e.get_option(option[0]) == option[1]
        s2 = torch.empty(2 * B * 16, dtype=torch.uint8, device=dev)
        r2 = torch.empty(2 * B * 80, dtype=torch.uint8, device=dev)
        e.run(None, B, rows, s2.data_ptr(), r2.data_ptr(), lag=4, stage=1)
        out = e.book().export()
        e.close()
        return out
    want, got = run(None), run(opt)
    assert len(want["parent"]) > 5000
    for k in KEYS:
        assert np.array_equal(got[k], want[k]), k


def test_context_without_book_follows_the_device_tree():
    """Option book = 0 (the ranks of a sharded run that do not report the tree): same node counts
    per run, same goal batch and goal node as a context with its book, and the stream position."""
    import torch
    free = workloads.map2_style(256, seed=6)
    B, rows = 512, 12
    dev = torch.device("cuda", 0)
    outs = []
    for book in (1, 0):
        e = _native.Engine(0)
        e.set_params(_native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 10, 45, 1, 1))   # tol_xy 10
        e.set_grid(free)
        e.set_option("book", book)
        e.rrt_begin([20.0, 20.0, 0.0], [128.0, 128.0, 0.0])
        e.rng_set_state(np.random.RandomState(3).get_state())
        s2 = torch.empty(2 * B * 16, dtype=torch.uint8, device=dev)
        r2 = torch.empty(2 * B * 80, dtype=torch.uint8, device=dev)
        n, sol = e.run(None, B, rows, s2.data_ptr(), r2.data_ptr(), lag=3, stage=1)
        st = e.rng_get_state()
        outs.append((sol, st[2], st[1].copy(), n, e.book().size()))
        e.close()
    (sol1, pos1, key1, n1, size1), (sol0, pos0, key0, n0, size0) = outs
    assert sol1 >= 0, "the case is meant to reach the goal"
    assert sol0 == sol1 and pos0 == pos1 and np.array_equal(key0, key1)
    assert size1 == n1 and size0 == 1 and n0 >= n1     # device count: every first occurrence
