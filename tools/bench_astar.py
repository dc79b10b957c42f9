"""Theta* / A* search timing (search.py:221-307) on map2, (280, 0) -> (8, 280) as main.py:50 runs it:
tr_astar (one search on the host, the reference's queue order) and tr_astar_batch (searches resident
on the GPU, one wave per query: one query alone, then batches of random queries) against the
pure-Python oracle on one host core.  One JSON
line.  usage: python tools/bench_astar.py"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from theta_rrt_amd import _native  # noqa: E402


def main():
    maps = np.load(os.path.join(ROOT, "tests", "golden", "maps.npz"))
    eng = _native.Engine(0)
    eng.set_grid(maps["map2"])
    eng.astar((280, 0), (8, 280), True)                       # warm-up
    runs = {}
    for theta in (True, False):
        t0 = time.perf_counter()
        path, st = eng.astar((280, 0), (8, 280), theta)
        dt = time.perf_counter() - t0
        runs["%s_host" % ("thetastar" if theta else "astar")] = dict(seconds=dt, path_len=len(path), **st)
    # the search resident on the GPU (tr_astar_batch, one wave per query): one query alone, then
    # batches of the same query and of random free-to-free queries, against the host search
    dev = {}
    q1 = np.array([[280, 0, 8, 280]], np.int32)
    eng.astar_batch(q1, True)
    t0 = time.perf_counter()
    paths, st = eng.astar_batch(q1, True)
    dev["single_query_s"] = time.perf_counter() - t0
    dev["single_query"] = dict(expanded=int(st[0, 0]), consumed=int(st[0, 1]), far_pushes=int(st[0, 2]),
                               path=paths[0].tolist())
    rs = np.random.RandomState(1)
    ys, xs = np.nonzero(maps["map2"])
    for nq in (256, 1024, 4096):
        a, b = rs.randint(0, len(xs), nq), rs.randint(0, len(xs), nq)
        q = np.column_stack([xs[a], ys[a], xs[b], ys[b]]).astype(np.int32)
        eng.astar_batch(q, True, cap=1024)             # sizes the context's work buffers
        t0 = time.perf_counter()
        paths, st = eng.astar_batch(q, True, cap=1024)
        dt = time.perf_counter() - t0
        m = min(nq, 64)
        t0 = time.perf_counter()
        for i in range(m):
            eng.astar((q[i, 0], q[i, 1]), (q[i, 2], q[i, 3]), True)
        host = (time.perf_counter() - t0) / m
        dev["random_%d" % nq] = dict(seconds=dt, queries_per_s=nq / dt, found=int((st[:, 3] == 0).sum()),
                                     mean_expanded=float(st[:, 0].mean()),
                                     host_queries_per_s_one_core=1.0 / host)
    runs["device_resident"] = dev
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import thetarrt_oracle as O
    t0 = time.perf_counter()
    opath, oexp, _ = O.astar(O.Params(), O.Grid(maps["map2"]), (280, 0), (8, 280))
    cpu = time.perf_counter() - t0
    best = runs["thetastar_host"]
    print(json.dumps({"metric": "lazy Theta* search on map2 (280,0)->(8,280), seconds",
                      "value": best["seconds"], "unit": "s", "higher_is_better": False,
                      "expanded": best["expanded"], "runs": runs,
                      "matches_oracle": [list(map(int, p)) for p in opath] == [list(map(int, p)) for p in
                                        eng.astar((280, 0), (8, 280), True)[0].tolist()],
                      "cpu_baseline": {"value": cpu, "unit": "s", "cores": 1, "kind": "port",
                                       "sample": "the same search, pure-Python oracle (%d expanded)"
                                                 % oexp}}))


if __name__ == "__main__":
    main()
