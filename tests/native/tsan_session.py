"""Test driver (GPU, no torch): pipelined RRT sessions through the C-ABI for a sanitizer build of
libthetarrt (THETARRT_LIB) -- the native loop with its replay worker thread and commit ring at
several look-ahead depths and lags, and the pipe_* calls with commits interleaved.  Device buffers
come from hipMalloc through ctypes.  Prints the node counts; exit 0 = ran to the end."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from theta_rrt_amd import _native, workloads  # noqa: E402

hip = C.CDLL("libamdhip64.so")


def dmalloc(n):
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), C.c_size_t(n)) == 0
    return p.value


def main():
    free = workloads.map2_style(512, seed=0)
    sx, sy = workloads.nearest_free(free, 16, 16)
    B = 2048
    e = _native.Engine(0)
    e.set_params(_native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1))
    e.set_grid(free)
    e.rrt_begin([float(sx), float(sy), 0.0], [256.0, 256.0, 0.0])
    e.rrt_reserve(200000, B)
    e.rng_set_state(np.random.RandomState(0).get_state())
    s2, r2 = dmalloc(3 * B * 16), dmalloc(3 * B * 80)
    for stage, lag in ((1, 4), (2, 2), (0, 5), (1, 1)):
        n, _ = e.run(None, B, 10, s2, r2, lag=lag, stage=stage)
        print("run stage %d lag %d: %d nodes" % (stage, lag, n), flush=True)
    g = dmalloc(3 * B * 8)
    for i in range(8):
        e.rng_gauss_dev(3 * B, g)
        e.pipe_expand(g, B, s2, r2)
        e.pipe_dedupe(s2, r2, B)
        if e.pending() > 2:
            e.pipe_commit()
    while e.pending():
        n, _ = e.pipe_commit()
    ex = e.book().export()
    print("pipe: %d nodes, %d edges" % (len(ex["nodes"]), len(ex["e_child"])), flush=True)
    e.close()


if __name__ == "__main__":
    main()
