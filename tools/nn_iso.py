"""Isolated nearest-node timing (no pipeline around it): a frozen random tree of N nodes on a
512x512 map, B integer queries, `reps` calls of tr_nn_batch (k_nn_pass1 + k_nn_resolve).  Run under
rocprofv3 --kernel-trace to read the kernels' durations:  python tools/nn_iso.py [N] [B] [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from theta_rrt_amd import _native  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 75000
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
rs = np.random.RandomState(0)
eng = _native.Engine(0)
eng.set_params(_native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1))
eng.set_grid(np.ones((512, 512), np.uint8))
xyt = np.column_stack([rs.uniform(0, 511, N), rs.uniform(0, 511, N), rs.uniform(-180, 180, N)])
eng.tree_reset(N)
eng.tree_append(xyt)
q = rs.randint(0, 512, (B, 2)).astype(np.int32)
got = eng.nn(q)
d = (q[:, None, 0] - xyt[None, :2048, 0]) ** 2 + (q[:, None, 1] - xyt[None, :2048, 1]) ** 2
t = time.perf_counter()
for _ in range(reps):
    eng.nn(q)
dt = (time.perf_counter() - t) / reps
sub = q[:256].astype(np.float64)
dd = (sub[:, None, 0] - xyt[None, :, 0]) ** 2 + (sub[:, None, 1] - xyt[None, :, 1]) ** 2
ok = np.array_equal(got[:256], np.argmin(np.sqrt(dd), axis=1))
print("N %d B %d: %.1f us per call (host-inclusive), first 256 exact: %s" % (N, B, dt * 1e6, ok))
