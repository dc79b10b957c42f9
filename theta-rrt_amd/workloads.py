"""Synthetic inputs for the benchmark configurations.

map2-style grid: random 3-5 px thick straight strokes of length [n/20, n/4) until `occ` of the cells
are occupied (map2.png is 7.81 % occupied with ~40 strokes).  Seeded, deterministic.
"""
import numpy as np


def map2_style(n, seed=0, occ=0.08):
    rng = np.random.default_rng(seed)
    free = np.ones((n, n), bool)
    while 1.0 - free.mean() < occ:
        length = rng.uniform(n / 20, n / 4)
        ang = rng.uniform(0, np.pi)
        w = int(rng.integers(3, 6))
        x0, y0 = rng.uniform(0, n, 2)
        t = np.arange(0.0, length, 0.5)
        xs = np.clip((x0 + t * np.cos(ang)).astype(np.int64), 0, n - 1)
        ys = np.clip((y0 + t * np.sin(ang)).astype(np.int64), 0, n - 1)
        for dx in range(-(w // 2), w - w // 2):
            for dy in range(-(w // 2), w - w // 2):
                free[np.clip(ys + dy, 0, n - 1), np.clip(xs + dx, 0, n - 1)] = False
    return free


def nearest_free(free, x, y):
    """Nudge (x, y) to the closest free cell (grid is [y][x])."""
    if free[y, x]:
        return x, y
    ys, xs = np.nonzero(free)
    k = int(np.argmin((xs - x) ** 2 + (ys - y) ** 2))
    return int(xs[k]), int(ys[k])


CONFIGS = {
    # BASELINE.json configs[1], [2], [4]: grid n, samples per GPU per batch, the
    # untimed tree size before a timed window, start cell (nudged to free space), goal = centre.
    # cfg2's prefill: 20 timed steps of 4096 samples add ~52k nodes, so a window that starts within
    # one step of 45k nodes ends just under the configuration's 100k-node bound
    "cfg2": {"grid": 512, "batch": 4096, "prefill": 45000, "start": 16},
    "cfg3": {"grid": 2048, "batch": 65536, "prefill": 1000000, "start": 64},
    # cfg5 = cfg3's inputs with the 8 x 65536-sample global batch sharded 8 ways (one rank per
    # GPU, replicated 1M-node tree, RCCL all-gather of the records): bench.py --config cfg5 under
    # torchrun --nproc-per-node 8; per GPU the same shape as cfg3.
    "cfg5": {"grid": 2048, "batch": 65536, "prefill": 1000000, "start": 64, "world": 8},
}
