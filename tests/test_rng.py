"""The np.random gaussian stream on the device (rng.hip, legacy_gauss.hpp): rand_conf's three legacy
gaussians per iteration (rrt.py:58,66) drawn on the GPU, bit for bit what RandomState returns.

CPU: the restatement compiled for the host (tests/native/gauss_check.cpp, g++) against libm's log
(math.log; numpy's array log is its own SIMD code, not the libm log legacy_gauss calls) and against
RandomState.standard_normal, including the cached-gaussian state.
GPU: tr_rng_gauss_dev against RandomState at 10M draws and across odd offsets; tr_rrt_run drawing
its own gaussians builds the same tree as the run fed numpy's gaussians, and leaves the stream where
numpy's would be after the batches the run used (also when it stops at the goal).
"""
import ctypes as C
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

HARNESS = os.path.join(ROOT, "tests", "native", "gauss_check.cpp")


@pytest.fixture(scope="module")
def gc(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("gc") / "gc.so")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fPIC", "-shared", "-o", so, HARNESS],
                   check=True)
    return C.CDLL(so)


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def test_legacy_log_equals_libm(gc):
    rs = np.random.RandomState(5)
    x1, x2 = 2 * rs.random_sample(150_000) - 1, 2 * rs.random_sample(150_000) - 1
    r2 = x1 * x1 + x2 * x2
    r2 = r2[(r2 < 1) & (r2 != 0)]
    near1 = 1 - rs.random_sample(50_000) * 0.07                 # glibc's |x - 1| < 2^-4 branch
    edges = [1.0, 0.5, 2.0 ** -104, 0.9375, np.nextafter(0.9375, 0), np.nextafter(1.0, 0),
             1.0 + float.fromhex('0x1.08p-4'), 1e-300, 3.0]
    x = np.concatenate([r2, near1, edges])
    out = np.empty_like(x)
    gc.gc_log(_dp(x), C.c_int64(len(x)), _dp(out))
    want = np.array([math.log(v) for v in x])
    assert np.array_equal(out.view(np.uint64), want.view(np.uint64))


@pytest.mark.parametrize("seed,skip", [(0, 0), (1, 7), (12345, 2), (2 ** 31, 623)])
def test_stream_equals_randomstate(gc, seed, skip):
    rs = np.random.RandomState(seed)
    rs.standard_normal(skip)                                    # odd skips leave has_gauss set
    st = rs.get_state()
    key = np.array(st[1], np.uint32)
    pos, has, g = C.c_int32(st[2]), C.c_int32(st[3]), C.c_double(st[4])
    n = 200_001
    out = np.empty(n)
    gc.gc_stream(key.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(pos), C.byref(has),
                 C.byref(g), C.c_int64(n), _dp(out))
    want = rs.standard_normal(n)
    st2 = rs.get_state()
    assert np.array_equal(out.view(np.uint64), want.view(np.uint64))
    assert np.array_equal(key, st2[1]) and pos.value == st2[2] and has.value == st2[3]
    assert g.value == st2[4]


# ------------------------------------------------------------------------------------ GPU
def _engine():
    import pkgload
    pkgload.load()
    from theta_rrt_amd import _native
    return _native, _native.Engine()


@pytest.mark.gpu
def test_gpu_gauss_equals_randomstate_10m():
    import torch
    _, eng = _engine()
    dev = torch.device("cuda", 0)
    for seed, skip, n in [(0, 0, 10_000_000), (7, 3, 3 * 4096 * 5 + 1), (99, 1, 1), (3, 0, 2)]:
        rs = np.random.RandomState(seed)
        rs.standard_normal(skip)
        eng.rng_set_state(rs.get_state())
        out = torch.empty(max(n, 1), dtype=torch.float64, device=dev)
        eng.rng_gauss_dev(n, out.data_ptr())
        eng.sync()
        got = out[:n].cpu().numpy()
        want = rs.standard_normal(n)
        bad = np.nonzero(got.view(np.uint64) != want.view(np.uint64))[0]
        assert len(bad) == 0, (seed, n, len(bad), bad[:5])
        st = eng.rng_get_state()
        # the next draws continue numpy's stream exactly
        rs2 = np.random.RandomState()
        rs2.set_state(st)
        assert np.array_equal(rs2.standard_normal(1001), rs.standard_normal(1001)), seed


@pytest.mark.gpu
def test_gpu_gauss_chunks_continue_the_stream():
    """Many small draws in a row (chunk boundaries at every parity of the cached gaussian)."""
    import torch
    _, eng = _engine()
    rs = np.random.RandomState(2024)
    eng.rng_set_state(rs.get_state())
    dev = torch.device("cuda", 0)
    sizes = [1, 2, 3, 5, 8, 13, 4096 * 3, 1, 77, 624, 625, 2]
    out = torch.empty(sum(sizes), dtype=torch.float64, device=dev)
    o = 0
    for n in sizes:
        eng.rng_gauss_dev(n, out[o:].data_ptr())
        o += n
    eng.sync()
    assert np.array_equal(out.cpu().numpy(), rs.standard_normal(sum(sizes)))


def _session(_native, free, start, goal, B):
    e = _native.Engine()
    e.set_params(_native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1))
    e.set_grid(free)
    e.rrt_begin(start, goal)
    e.rrt_reserve(200000, B)
    return e


@pytest.mark.gpu
@pytest.mark.parametrize("B,rows,stage", [(4096, 11, 1), (1000, 9, 2), (4096, 3, 0)])
def test_gpu_run_draws_numpy_stream(B, rows, stage):
    """tr_rrt_run(d_gauss=NULL) == tr_rrt_run fed RandomState.standard_normal rows."""
    import torch
    from theta_rrt_amd import workloads
    _native, _ = _engine()
    free = workloads.map2_style(512, seed=0)
    sx, sy = workloads.nearest_free(free, 16, 16)
    start, goal = [float(sx), float(sy), 0.0], [256.0, 256.0, 0.0]
    dev = torch.device("cuda", 0)
    ns = max(2, stage + 1)
    rs = np.random.RandomState(11)
    st0 = rs.get_state()
    G = torch.from_numpy(rs.standard_normal((rows, 3 * B))).to(dev)

    outs = []
    for own in (False, True):
        e = _session(_native, free, start, goal, B)
        s2 = torch.empty(ns * B * 16, dtype=torch.uint8, device=dev)
        r2 = torch.empty(ns * B * 80, dtype=torch.uint8, device=dev)
        if own:
            e.rng_set_state(st0)
        e.run(None if own else G.data_ptr(), B, rows, s2.data_ptr(), r2.data_ptr(), lag=3,
              stage=stage)
        outs.append(e.book().export())
        if own:
            rs_after = np.random.RandomState()
            rs_after.set_state(e.rng_get_state())
            assert np.array_equal(rs_after.standard_normal(100), rs.standard_normal(100))
    for k in ("nodes", "parent", "u", "e_off", "e_child"):
        assert np.array_equal(outs[0][k], outs[1][k]), k


@pytest.mark.gpu
def test_gpu_run_stream_rewinds_to_goal_batch():
    """A run that reaches the goal leaves the stream after the goal batch (rows after it unused)."""
    import torch
    _native, _ = _engine()
    from theta_rrt_amd import workloads
    free = np.ones((128, 128), np.uint8)
    B, rows = 256, 40
    e = _native.Engine()
    e.set_params(_native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 10, 45, 1, 1))   # tol_xy 10
    e.set_grid(free)
    e.rrt_begin([10.0, 10.0, 0.0], [60.0, 60.0, 0.0])
    rs = np.random.RandomState(4)
    e.rng_set_state(rs.get_state())
    dev = torch.device("cuda", 0)
    s2 = torch.empty(2 * B * 16, dtype=torch.uint8, device=dev)
    r2 = torch.empty(2 * B * 80, dtype=torch.uint8, device=dev)
    n, sol = e.run(None, B, rows, s2.data_ptr(), r2.data_ptr(), lag=5, stage=1)
    assert sol >= 0

    # the batch that reached it, replayed with numpy's gaussians
    f = _native.Engine()
    f.set_params(_native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 10, 45, 1, 1))
    f.set_grid(free)
    f.rrt_begin([10.0, 10.0, 0.0], [60.0, 60.0, 0.0])
    used = 0
    for _ in range(rows):
        _, s = f.rrt_step(rs.standard_normal(3 * B))
        used += 1
        if s >= 0:
            break
    assert s == sol and used < rows
    rs_after = np.random.RandomState()
    rs_after.set_state(e.rng_get_state())
    assert np.array_equal(rs_after.standard_normal(50), rs.standard_normal(50))


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [0, 2, 4])
def test_gpu_run_goal_in_the_last_batches_rewinds_again(extra):
    """The goal turns up in a batch the loop had already enqueued together with every later one
    (fewer than `lag` rows behind it): the run has by then placed the stream after its last row,
    and places it again after the goal batch."""
    import torch
    _native, _ = _engine()
    free = np.ones((512, 512), np.uint8)
    B = 64
    par = _native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 10, 45, 1, 1)
    rs = np.random.RandomState(4)
    f = _native.Engine()
    f.set_params(par)
    f.set_grid(free)
    f.rrt_begin([10.0, 10.0, 0.0], [400.0, 400.0, 0.0])
    used, s = 0, -1
    while s < 0 and used < 400:
        _, s = f.rrt_step(rs.standard_normal(3 * B))
        used += 1
    assert s >= 0 and used > 5, used
    e = _native.Engine()
    e.set_params(par)
    e.set_grid(free)
    e.rrt_begin([10.0, 10.0, 0.0], [400.0, 400.0, 0.0])
    e.rng_set_state(np.random.RandomState(4).get_state())
    dev = torch.device("cuda", 0)
    s2 = torch.empty(3 * B * 16, dtype=torch.uint8, device=dev)
    r2 = torch.empty(3 * B * 80, dtype=torch.uint8, device=dev)
    n, sol = e.run(None, B, used + extra, s2.data_ptr(), r2.data_ptr(), lag=5, stage=2)
    assert sol == s
    got, want = e.book().export(), f.book().export()
    for k in ("nodes", "parent", "u", "e_off", "e_child"):
        assert np.array_equal(got[k], want[k]), k
    rs_after = np.random.RandomState()
    rs_after.set_state(e.rng_get_state())
    assert np.array_equal(rs_after.standard_normal(50), rs.standard_normal(50))
    e.close()
    f.close()


@pytest.mark.gpu
def test_rrt_run_device_stream_keeps_np_random_in_step(maps):
    """rrt.run(batch > 1) draws the np.random stream on the device (full batches in the native loop,
    a partial last batch on the host) and leaves np.random where host draws would have."""
    import builtins
    import pkgload
    pkgload.load()
    from theta_rrt_amd import config, rrt
    builtins.imarray = maps["map2"]
    config.ensure_defaults()
    old = builtins.K, builtins.tol_xy
    builtins.K, builtins.tol_xy = 1 + 7 * 256 + 100, 0       # 7 full batches + a partial one
    try:
        start, goal = ((280, 0), -170.0), ((73, 38), 0.0)
        np.random.seed(21)
        sol_d, ex_d = rrt.run(start, goal, batch=256)
        after_d = np.random.get_state()
        np.random.seed(21)
        rs = np.random.RandomState(21)
        sol_h, ex_h = rrt.run(start, goal, batch=256, gauss_source=lambda n: rs.standard_normal(n))
        assert sol_d == sol_h
        for k in ("nodes", "parent", "u", "e_off", "e_child"):
            assert np.array_equal(ex_d[k], ex_h[k]), k
        after_h = rs.get_state()
        assert np.array_equal(after_d[1], after_h[1]) and after_d[2:] == after_h[2:]
    finally:
        builtins.K, builtins.tol_xy = old


@pytest.mark.gpu
def test_gauss_dev_then_run_share_one_stream_position():
    """tr_rng_gauss_dev (context stream, asynchronous) followed at once by a run that draws its own
    gaussians (rng stream): the run starts from the position the draw leaves, whatever is still in
    flight.  Checked against RandomState: draw n, then the run's batches."""
    import torch
    from theta_rrt_amd import workloads
    _native, _ = _engine()
    free = workloads.map2_style(256, seed=1)
    B, rows, n0 = 1024, 6, 3 * 4096 + 1          # odd: the draw leaves a cached second gaussian
    dev = torch.device("cuda", 0)
    rs = np.random.RandomState(77)
    st0 = rs.get_state()
    head = rs.standard_normal(n0)
    G = torch.from_numpy(rs.standard_normal((rows, 3 * B))).to(dev)
    outs = []
    for own in (False, True):
        e = _session(_native, free, [20.0, 20.0, 0.0], [128.0, 128.0, 0.0], B)
        s2 = torch.empty(2 * B * 16, dtype=torch.uint8, device=dev)
        r2 = torch.empty(2 * B * 80, dtype=torch.uint8, device=dev)
        if own:
            e.rng_set_state(st0)
            # sized once, so the second pass below meets no synchronizing reallocation
            e.run(None, B, 2, s2.data_ptr(), r2.data_ptr(), lag=3, stage=1)
            e.rrt_begin([20.0, 20.0, 0.0], [128.0, 128.0, 0.0])
            e.rng_set_state(st0)
            out = torch.empty(n0, dtype=torch.float64, device=dev)
            e.rng_gauss_dev(n0, out.data_ptr())
            e.run(None, B, rows, s2.data_ptr(), r2.data_ptr(), lag=3, stage=1)
            assert np.array_equal(out.cpu().numpy(), head)
        else:
            e.run(G.data_ptr(), B, rows, s2.data_ptr(), r2.data_ptr(), lag=3, stage=1)
        outs.append(e.book().export())
        e.close()
    for k in ("nodes", "parent", "u", "e_off", "e_child"):
        assert np.array_equal(outs[0][k], outs[1][k]), k


@pytest.mark.gpu
def test_rrt_run_raising_batch_leaves_np_random_like_the_host_loop(maps):
    """Where the reference raises (TypeError: a straight control that needs shortening), rrt.run's
    device-drawn loop leaves np.random after the raising batch, as the host-drawn loop does."""
    import builtins
    import pkgload
    pkgload.load()
    from theta_rrt_amd import config, rrt
    builtins.imarray = maps["map1"]
    config.ensure_defaults()
    old = builtins.K, builtins.tol_xy
    builtins.K, builtins.tol_xy = 1 + 40 * 64, 0
    try:
        start, goal = ((5, 5), 0.0), ((90, 90), 45.0)
        hit = None
        for seed in range(40):
            np.random.seed(seed)
            try:
                rrt.run(start, goal, batch=64)
            except TypeError:
                hit = seed
                break
        assert hit is not None, "no seed raised: pick other parameters"
        after_d = np.random.get_state()
        rs = np.random.RandomState(hit)
        with pytest.raises(TypeError):
            rrt.run(start, goal, batch=64, gauss_source=lambda n: rs.standard_normal(n))
        after_h = rs.get_state()
        assert np.array_equal(after_d[1], after_h[1]) and after_d[2:] == after_h[2:]
    finally:
        builtins.K, builtins.tol_xy = old


def test_mt_jump_table_against_numpy_stream():
    """The generated jump-ahead polynomials (csrc/mt_jump.hpp, tools/gen_mt_jump.py): the state
    block w * MT_SEG - 624 words past a window of MT_HIST words of numpy's MT19937 stream is the
    XOR of the window's words at each polynomial's set bits (rng.hip's k_mt_jump), for a stream
    the generator did not see."""
    import re
    txt = open(os.path.join(ROOT, "theta-rrt_amd", "csrc", "mt_jump.hpp")).read()
    hist, segb, nseg = (int(re.search(r"%s = (\d+)" % k, txt).group(1))
                        for k in ("MT_HIST", "MT_SEG_BLOCKS", "MT_NSEG"))
    words = np.array([int(v, 16) for v in re.findall(r"0x([0-9a-f]{8})u", txt)], np.uint32)
    table = words.reshape(nseg - 1, 624)
    rs = np.random.RandomState(20261114)
    blocks = [rs.get_state()[1].copy()]
    for _ in range(nseg * segb + 40):
        rs.bytes(4 * 624)
        blocks.append(rs.get_state()[1].copy())
    x = np.concatenate(blocks).astype(np.uint32)
    end = 36 * 624
    m = end - hist
    for w in (1, 2, 7, nseg - 1):
        bits = np.unpackbits(table[w - 1].view(np.uint8), bitorder="little")
        idx = np.nonzero(bits)[0]
        assert idx.max() < 19937
        a = end + w * segb * 624 - 624
        ks = np.array([0, 1, 63, 64, 311, 622, 623])
        got = np.array([np.bitwise_xor.reduce(x[m + idx + k]) for k in ks], np.uint32)
        assert np.array_equal(got, x[a + ks]), w


@pytest.mark.gpu
def test_gpu_gauss_serial_and_parallel_generation_mix():
    """Draw sizes on both sides of the parallel-generation threshold, with ring regrowth between
    them (a small ring's history is not enough for a jump: the generator fills it in serially)."""
    import torch
    _, eng = _engine()
    rs = np.random.RandomState(424242)
    eng.rng_set_state(rs.get_state())
    dev = torch.device("cuda", 0)
    sizes = [5, 20000, 7, 600000, 3, 50001, 2000001, 11, 400000]
    out = torch.empty(sum(sizes), dtype=torch.float64, device=dev)
    o = 0
    for n in sizes:
        eng.rng_gauss_dev(n, out[o:].data_ptr())
        o += n
    eng.sync()
    got, want = out.cpu().numpy(), rs.standard_normal(sum(sizes))
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (len(bad), bad[:5], np.cumsum(sizes))
    st = eng.rng_get_state()
    rs2 = np.random.RandomState()
    rs2.set_state(st)
    assert np.array_equal(rs2.standard_normal(1000), rs.standard_normal(1000))
