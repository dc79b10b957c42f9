"""Grow a cfg2 tree with the engine and dump it with one batch of samples (NN workload analysis)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from theta_rrt_amd import _native, workloads  # noqa: E402

n_grid, B = workloads.CONFIGS["cfg2"]["grid"], workloads.CONFIGS["cfg2"]["batch"]
free = workloads.map2_style(n_grid, seed=0)
sx, sy = workloads.nearest_free(free, 16, 16)
eng = _native.Engine(0)
eng.set_params(_native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1))
eng.set_grid(free)
eng.rrt_begin([sx, sy, 0.0], [n_grid // 2, n_grid // 2, 0.0])
rs = np.random.RandomState(0)
target = int(sys.argv[1]) if len(sys.argv) > 1 else 80000
n = 1
while n < target:
    n, _ = eng.rrt_step(rs.standard_normal(3 * B))
nodes = eng.book().nodes()
g = rs.standard_normal(3 * B)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "nnprobe.npz"), nodes=nodes, gauss=g, free=free)
print("tree", len(nodes))
