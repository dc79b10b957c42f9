"""Theta* / A* search timing (search.py:221-307) on map2, (280, 0) -> (8, 280) as main.py:50 runs it:
tr_astar (host queue in the reference's order; lazy-Theta* line of sight on the host, spec 0, or
on the GPU in speculative batches of several widths) against the pure-Python oracle on one host
core.  One JSON
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
        for spec in ((0, 1, 64, 1024) if theta else (0,)):
            t0 = time.perf_counter()
            path, st = eng.astar((280, 0), (8, 280), theta, spec=spec)
            dt = time.perf_counter() - t0
            runs["%s_spec%d" % ("thetastar" if theta else "astar", spec)] = dict(
                seconds=dt, path_len=len(path), **st)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import thetarrt_oracle as O
    t0 = time.perf_counter()
    opath, oexp, _ = O.astar(O.Params(), O.Grid(maps["map2"]), (280, 0), (8, 280))
    cpu = time.perf_counter() - t0
    best = runs["thetastar_spec0"]
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
