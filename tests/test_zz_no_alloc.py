"""tr_expand_dev_noalloc (static device scratch, no allocation) against tr_expand_dev, through the
C-ABI: identical samples and records on two calls in a row, the second with a smaller batch, and
no change in the device's free memory across the calls."""
import numpy as np
import pytest

import pkgload

pkgload.load()
from theta_rrt_amd import _native, workloads  # noqa: E402

pytestmark = pytest.mark.gpu


def _expand(e, g, B, goal3, noalloc):
    import torch
    dev = g.device
    smp = torch.zeros(B * 16, dtype=torch.uint8, device=dev)
    rec = torch.zeros(B * 80, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()                     # the fills above ran on torch's stream
    free0 = torch.cuda.mem_get_info(dev)[0]
    e.expand_dev(g.data_ptr(), B, goal3, smp.data_ptr(), rec.data_ptr(), noalloc=noalloc)
    e.sync()
    free1 = torch.cuda.mem_get_info(dev)[0]
    return smp.cpu().numpy(), rec.cpu().numpy(), free0 - free1


def test_expand_noalloc_equals_expand_dev_two_calls():
    import torch
    dev = torch.device("cuda", 0)
    n = 512
    free = workloads.map2_style(n, seed=3)
    rs = np.random.RandomState(5)
    ys, xs = np.nonzero(free)
    pick = rs.choice(len(xs), 60000, replace=False)
    tree = np.column_stack([xs[pick] + rs.uniform(0, 1, len(pick)), ys[pick] + rs.uniform(0, 1, len(pick)),
                            rs.uniform(-180, 180, len(pick))])
    goal3 = [n / 2, n / 2, 0.0]
    e = _native.Engine(0)
    e.set_params(_native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1))
    e.set_grid(free)
    e.tree_reset(1 << 17)
    e.tree_append(tree)
    for B in (4096, 1500):                       # the second call is smaller: stale scratch behind it
        g = torch.from_numpy(rs.standard_normal(3 * B)).to(dev)
        s_ref, r_ref, _ = _expand(e, g, B, goal3, noalloc=False)
        s_na, r_na, used = _expand(e, g, B, goal3, noalloc=True)
        assert used == 0, "the no-alloc entry point changed the device's free memory"
        assert np.array_equal(s_na, s_ref), B
        assert np.array_equal(r_na, r_ref), B
        R = r_ref.view(_native.RECORD_DTYPE)
        assert (R["status"] == _native.ST_OK).sum() > B // 4       # a real workload, not all skips

    # beyond the static scratch: refused with a message, nothing launched
    big = 1 << 17
    g = torch.zeros(3 * big, dtype=torch.float64, device=dev)
    smp = torch.zeros(big * 16, dtype=torch.uint8, device=dev)
    rec = torch.zeros(big * 80, dtype=torch.uint8, device=dev)
    with pytest.raises(_native.NativeError, match="static buffer"):
        e.expand_dev(g.data_ptr(), big, goal3, smp.data_ptr(), rec.data_ptr(), noalloc=True)
    e.close()
