"""Sample-sharded batches on 2 ranks (gloo, CPU): the multi-GPU path of bench.py.

Each rank expands a contiguous slice of every batch against the replicated snapshot (here with the
CPU oracle in place of the HIP kernels), the records are all-gathered in rank order, and every rank
appends them with the host bookkeeping (tr_book_ingest).  Both ranks must end with the same tree,
and that tree must equal the single-process batched run (oracle rrt_batched)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, golden  # noqa: F401
import pkgload

pkgload.load()
from theta_rrt_amd import _native  # noqa: E402
import thetarrt_oracle as O  # noqa: E402

B, NB, WORLD = 64, 4, 2
START, GOAL = ((280, 0), -170.0), ((73, 38), 0.0)


def _records(P, grid, snap, qs):
    """Oracle expansions of samples qs against snapshot poses -> (tr_sample, tr_record) arrays."""
    s = np.zeros(len(qs), _native.SAMPLE_DTYPE)
    r = np.zeros(len(qs), _native.RECORD_DTYPE)
    txy = np.array([[float(n[0][0]), float(n[0][1])] for n in snap])
    for j, q in enumerate(qs):
        s[j] = (q[0][0], q[0][1], q[1])
        r[j]["near"] = -1
        if not grid.freespace(q[0]):
            r[j]["status"] = _native.ST_SKIP
            continue
        nn = int(O.nn_numpy(txy[:, 0], txy[:, 1], [q[0][0]], [q[0][1]])[0])
        e = O.expand_one(P, grid, snap, q, nn)
        fl = _native.FL_DROVE if e.drove else 0
        r[j]["near"] = nn
        if e.u is not None:
            straight = e.u[1] is None
            fl |= _native.FL_STRAIGHT if straight else 0
            r[j]["steer"], r[j]["dist"] = e.u[0], e.u[3]
            if not straight:
                r[j]["iccx"], r[j]["iccy"], r[j]["rad"] = e.u[1][0], e.u[1][1], e.u[2]
        if e.qnew is not None:
            r[j]["x"], r[j]["y"], r[j]["th"] = e.qnew[0][0], e.qnew[0][1], e.qnew[1]
        r[j]["status"] = {"ok": _native.ST_OK, "collision": _native.ST_COLLISION,
                          "straight_drive": _native.ST_STRAIGHT}[e.status]
        r[j]["flags"] = fl
    return s, r


def _rank(rank, port, free, gauss, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    P = O.Params(tol_xy=0)
    grid = O.Grid(free)
    book = _native.Book()
    book.set_straight_reject(1)                              # as rrt_batched(straight="reject")
    book.reset([START[0][0], START[0][1], START[1]])
    for g in gauss:
        qs = O.samples_from_gauss(P, free.shape, GOAL, g)
        snap = [((x, y), t) for x, y, t in book.nodes()]
        lo, hi = rank * B // WORLD, (rank + 1) * B // WORLD
        s, r = _records(P, grid, snap, qs[lo:hi])            # this rank's slice
        sb = torch.from_numpy(s.view(np.uint8).copy())
        rb = torch.from_numpy(r.view(np.uint8).copy())
        s_all = [torch.empty_like(sb) for _ in range(WORLD)]
        r_all = [torch.empty_like(rb) for _ in range(WORLD)]
        dist.all_gather(s_all, sb)
        dist.all_gather(r_all, rb)
        S = np.concatenate([t.numpy() for t in s_all]).view(_native.SAMPLE_DTYPE)
        R = np.concatenate([t.numpy() for t in r_all]).view(_native.RECORD_DTYPE)
        book.ingest(S, R, n_snap=book.size())
    ex = book.export()
    np.savez(out % rank, **ex)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_sharded_batches_equal_single_process(tmp_path, maps):
    free = maps["map2"]
    gauss = np.random.RandomState(11).standard_normal((NB, 3 * B))
    out = str(tmp_path / "rank%d.npz")
    mp.spawn(_rank, args=(_free_port(), free, gauss, out), nprocs=WORLD, join=True)
    a, b = np.load(out % 0), np.load(out % 1)
    for k in ("nodes", "parent", "u", "e_off", "e_child"):
        assert np.array_equal(a[k], b[k]), k
    it = iter(list(gauss))
    _, T = O.rrt_batched(O.Params(K=NB * B + 1, tol_xy=0), O.Grid(free), START, GOAL, B=B,
                         gauss_source=lambda n: next(it), straight="reject")
    assert np.array_equal(a["parent"], np.array(T.parent))
    nodes = np.array([[n[0][0], n[0][1], n[1]] for n in T.nodes], np.float64)
    assert np.array_equal(a["nodes"], nodes)
    assert len(T.nodes) > 1 + B // 4           # the batches did grow the tree
