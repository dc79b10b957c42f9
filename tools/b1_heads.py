import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import pkgload; pkgload.load()
from theta_rrt_amd import _native, workloads
free = workloads.map2_style(300, seed=0)
sx, sy = workloads.nearest_free(free, 16, 16)
dev = torch.device("cuda", 0)
tot = 0
fails = 0
for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    eng = _native.Engine(0)
    eng.set_params(_native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1))
    eng.set_grid(free)
    eng.rng_set_state(np.random.RandomState(seed).get_state())
    eng.rrt_begin([float(sx), float(sy), 0.0], [150.0, 150.0, 0.0])
    B = 1
    s2 = torch.empty(3 * B * 16, dtype=torch.uint8, device=dev)
    r2 = torch.empty(3 * B * 80, dtype=torch.uint8, device=dev)
    try:
        if len(sys.argv) > 2 and sys.argv[2] == "step":      # one synchronous step per sample
            G = np.random.RandomState(seed).standard_normal((1500, 3))
            for g in G:
                n, _ = eng.rrt_step(g)
        else:
            n, _ = eng.run(None, B, 3000, s2.data_ptr(), r2.data_ptr(), lag=4, stage=2)
        if seed % 20 == 0 or eng.get_option("head_waits"):
            print("seed", seed, "nodes", n, "head_waits", eng.get_option("head_waits"), flush=True)
    except Exception as ex:
        fails += 1
        print("seed", seed, "FAILED", ex, "head_waits", eng.get_option("head_waits"), flush=True)
    tot += eng.get_option("head_waits")
    eng.close()
print("total head_waits", tot, "failed runs", fails)
