"""cfg4 (BASELINE.json configs[3]): the Theta* line-of-sight batch on the GPU.

The 10k first LOS queries lazy Theta* issues on map2 (search.py:258-263, captured from the reference
in tests/golden/f2_los.npz) as one device-resident batch of int32 segments, `reps` launches of
tr_los_batch_dev (k_los_i32: one wave per ray, Bresenham pixels tested in parallel) timed with HIP
events on the engine's stream.  Prints one JSON line: rays/s, pixels/s (pixels = sum over rays of
max(|dx|, |dy|) + 1, search.py:43-94), the per-launch time, a check against the reference's answers,
and the pure-Python oracle timed on one host core over the same rays (CPU baseline).

usage: python tools/bench_los.py [n_rays] [reps]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from theta_rrt_amd import _native  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    f = np.load(os.path.join(ROOT, "tests", "golden", "f2_los.npz"))
    maps = np.load(os.path.join(ROOT, "tests", "golden", "maps.npz"))
    seg = np.ascontiguousarray(f["theta_q"][:n].astype(np.int32))
    want = f["theta_r"][:n].astype(bool)
    px = int(np.sum(np.maximum(np.abs(seg[:, 2] - seg[:, 0]), np.abs(seg[:, 3] - seg[:, 1])) + 1))

    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    eng = _native.Engine(0)
    eng.set_stream(stream.cuda_stream)
    eng.set_grid(maps["map2"])
    d_seg = torch.from_numpy(seg).to(dev)
    d_out = torch.empty(n, dtype=torch.uint8, device=dev)
    L = _native.lib()

    def launch():
        _native.check(L.tr_los_batch_dev(eng.h, d_seg.data_ptr(), n, d_out.data_ptr()))

    for _ in range(10):
        launch()
    torch.cuda.synchronize()
    ok = bool(np.array_equal(d_out.cpu().numpy().astype(bool), want))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import thetarrt_oracle as O
    g = O.Grid(maps["map2"])
    t0 = time.perf_counter()
    cpu = [g.los((int(a), int(b)), (int(c), int(d))) for a, b, c, d in seg.tolist()]
    cpu_s = time.perf_counter() - t0
    assert np.array_equal(np.array(cpu), want)

    print(json.dumps({
        "metric": "Theta* LOS batch (cfg4): line-of-sight rays/s", "value": n / (us * 1e-6),
        "unit": "rays/s", "pixels_per_s": px / (us * 1e-6), "launch_us": us, "rays": n,
        "pixels": px, "reps": reps, "matches_reference": ok, "kernel": "k_los_i32",
        "workload": "first %d lazy-Theta* LOS queries of search.astar((280,0),(8,280)) on map2 "
                    "(captured from the reference, tests/golden/f2_los.npz), device-resident" % n,
        "cpu_baseline": {"value": n / cpu_s, "unit": "rays/s", "cores": 1, "kind": "port",
                         "sample": "the same %d rays, pure-Python oracle Bresenham, %.2fs"
                                   % (n, cpu_s)}}))


if __name__ == "__main__":
    main()
