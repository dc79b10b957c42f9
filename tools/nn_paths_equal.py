"""Whole-tree equality of the nearest-node paths at bench scale: the same device-drawn batches run
with the default paths and with the sweep of every node must leave identical books.
python tools/nn_paths_equal.py [batch] [rows]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from theta_rrt_amd import _native, workloads  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 40
n_grid = int(sys.argv[3]) if len(sys.argv) > 3 else 512
free = workloads.map2_style(n_grid, seed=0)
sx, sy = workloads.nearest_free(free, 16, 16)
dev = torch.device("cuda", 0)
outs = []
for opts in ({}, {"nn_grid": 0}, {"nn_grid_min": 0, "nn_far_sweep": 0}):
    e = _native.Engine(0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    e.set_stream(stream.cuda_stream)
    e.set_params(_native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1))
    e.set_grid(free)
    for k, v in opts.items():
        e.set_option(k, v)
    e.rng_set_state(np.random.RandomState(1).get_state())
    e.rrt_begin([float(sx), float(sy), 0.0], [n_grid / 2, n_grid / 2, 0.0])
    s2 = torch.empty(2 * B * 16, dtype=torch.uint8, device=dev)
    r2 = torch.empty(2 * B * 80, dtype=torch.uint8, device=dev)
    stage = 1 if B <= 8192 else 0
    n = 1
    for q in range(0, rows, 8):
        n, _ = e.run(None, B, min(8, rows - q), s2.data_ptr(), r2.data_ptr(), lag=4, stage=stage)
    outs.append(e.book().export())
    print(opts or "default", "nodes", n, flush=True)
    e.close()
for o in outs[1:]:
    for k in ("nodes", "parent", "u", "e_off", "e_child"):
        assert np.array_equal(o[k], outs[0][k]), k
print("equal: %d nodes" % len(outs[0]["parent"]))
