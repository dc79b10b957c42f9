"""Per-phase wall-clock profile of k_expand_arc from the diagnosis build (build.py --variant
phases): grows the cfg2 bench tree to ~70k nodes, runs a few more batches and reads the stamps of
the last launch (one row per sample) through tr_diag_phases.

THETARRT_LIB=theta-rrt_amd/libthetarrt_phases.so python tools/phases.py [--set option=value]
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pkgload  # noqa: E402

pkgload.load()
from theta_rrt_amd import _native, workloads  # noqa: E402
import torch  # noqa: E402

NAMES = ["loads", "delta", "steer", "rays", "drive", "arc-plan", "arc-loop", "look"]


def print_timeline(lib, last_us):
    """Launches of the pipeline's kernels over the last `last_us` microseconds of the block log
    (diaglog.hpp): a launch = a cluster of blocks in time."""
    names = {0: "k_samples", 1: "k_nn_pass1", 2: "k_nn_resolve", 3: "k_expand_arc", 4: "k_dd", 5: "k_gate",
             6: "k_mt_gen", 7: "k_mt_jump", 8: "k_mt_gen_par", 9: "k_gauss_count", 10: "k_gauss_emit",
             11: "k_nn_grid", 12: "k_cell_new", 13: "k_cell_scan", 14: "k_cell_move"}
    rows = []
    for fn in ("tr_diag_log_k", "tr_diag_log_nn", "tr_diag_log_dd", "tr_diag_log_rng", "tr_diag_log_nng"):
        buf = np.zeros((1 << 16, 3), np.uint64)
        cnt = C.c_uint(0)
        assert getattr(lib, fn)(buf.ctypes.data_as(C.c_void_p), C.byref(cnt)) == 0
        rows.append(buf[:min(cnt.value, 1 << 16)].astype(np.int64))
    log = np.concatenate(rows)
    tend = log[:, 2].max()
    log = log[log[:, 1] > tend - int(last_us * 100)]
    launches = []
    for kid, nm in names.items():
        sel = log[log[:, 0] == kid]
        sel = sel[np.argsort(sel[:, 1])]
        cur = None
        for _, t0, t1 in sel:                                 # a new launch: its blocks start after
            if cur is None or t0 > cur[3] + 300:              # every block of the last one ended + 3 us
                cur = [nm, t0, t0, t1, 0, []]
                launches.append(cur)
            cur[2] = max(cur[2], t0)
            cur[3] = max(cur[3], t1)
            cur[4] += 1
            cur[5].append(t1 - t0)
    launches.sort(key=lambda r: r[1])
    base = launches[0][1]
    print("timeline (us since the first logged block; last-start = when the launch's last block began):")
    for nm, a, b, c, nblk, durs in launches:
        stream = "main" if nm in ("k_expand_arc", "k_dd") else ("rng" if nm[2] in "mg" and nm != "k_gate" else "side")
        q = np.percentile(np.array(durs) * 0.01, [10, 50, 90, 100])
        print("  %8.2f -> %8.2f  %-13s %-4s blocks %4d  span %6.2f  last block started +%.2f  "
              "block us p10 %.1f p50 %.1f p90 %.1f max %.1f" % (
                  (a - base) * 0.01, (c - base) * 0.01, nm, stream, nblk, (c - a) * 0.01, (b - a) * 0.01, *q))


def main():
    B = int(os.environ.get("PHASES_B", "4096"))
    free = workloads.map2_style(512, seed=0)
    sx, sy = workloads.nearest_free(free, 16, 16)
    dev = torch.device("cuda", 0)
    eng = _native.Engine(0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    eng.set_params(_native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1))
    eng.set_grid(free)
    eng.rng_set_state(np.random.RandomState(0).get_state())
    for kv in sys.argv[1:]:
        if "=" in kv:
            k, v = kv.split("=")
            eng.set_option(k, int(v))
    s2 = torch.empty(2 * B * 16, dtype=torch.uint8, device=dev)
    r2 = torch.empty(2 * B * 80, dtype=torch.uint8, device=dev)
    eng.rrt_begin([float(sx), float(sy), 0.0], [256.0, 256.0, 0.0])
    eng.rrt_reserve(200000, B)
    n = 1
    while n < int(os.environ.get("PHASES_NODES", "70000")):
        n, _ = eng.run(None, B, 4, s2.data_ptr(), r2.data_ptr(), lag=4, stage=1)
    lib = C.CDLL(_native.LIB_PATH)          # the same handle the engine loaded
    ring = np.zeros((8, 4096, 10), np.uint64)              # the first 4096 samples of each launch
    nrows = int(os.environ.get("PHASES_ROWS", "8"))
    n, _ = eng.run(None, B, nrows, s2.data_ptr(), r2.data_ptr(), lag=4, stage=1)
    torch.cuda.synchronize()
    rc = lib.tr_diag_phases(ring.ctypes.data_as(C.c_void_p))
    assert rc == 0, rc
    dds = np.zeros((8, 4), np.uint64)
    assert lib.tr_diag_dd(dds.ctypes.data_as(C.c_void_p)) == 0
    order = np.argsort(ring[:, 0, 9] >> np.uint64(16))        # by dedupe epoch: oldest launch first
    # main-stream timeline: expansion of the batch after dedupe epoch e (its rows carry e), then
    # the dedupe of epoch e + 1
    tl = []
    for slot in order:
        e = int(ring[slot, 0, 9] >> np.uint64(16))
        t = ring[slot, :, :9].astype(np.int64)
        d = dds[(e + 1) % 8].astype(np.int64)
        if int(d[3]) != e + 1:
            continue
        tl.append((e, t[:, 0].min(), t[:, 8].max(), d[0], d[1], d[2]))
    for i, (e, x0, x1, d0, d1, d2) in enumerate(tl):
        gap = (x0 - tl[i - 1][5]) * 0.01 if i else float("nan")
        print("epoch %d: [dd gate passed -> expand start %.2f] expand %.2f [-> dd start %.2f] dd %.2f "
              "gate wait %.2f | period %.2f us" % (e, gap, (x1 - x0) * 0.01, (d0 - x1) * 0.01, (d1 - d0) * 0.01,
                                                (d2 - d1) * 0.01, (x0 - tl[i - 1][1]) * 0.01 if i else float("nan")))
    for slot in order:
        o = ring[slot]
        tt = o[:, :9].astype(np.int64)
        wy = ((o[:, 9] >> np.uint64(8)) & np.uint64(0xff)).astype(np.int64)
        print("ring slot %d: epoch %d span %.2f us, scans: %d box, %d overflow" % (
            slot, int(o[0, 9] >> np.uint64(16)), (tt[:, 8].max() - tt[:, 0].min()) * 0.01,
            (wy & 1).astype(bool).sum(), (wy & 2).astype(bool).sum()) + " %d read the overflow list" % (wy & 4).astype(bool).sum())
    spans = []
    for slot in order[5:8]:                                   # mid-run launches (look-ahead behind them)
        out = ring[slot]
        t = out[:, :9].astype(np.int64)
        st = (out[:, 9] & np.uint64(0xff)).astype(np.int64)
        why = ((out[:, 9] >> np.uint64(8)) & np.uint64(0xff)).astype(np.int64)
        live = st != 0                                        # expanded samples (TR_ST_SKIP = 0 are not)
        t0 = t[:, 0].min()
        spans.append((t[:, 8].max() - t0) * 0.01)
        print("epoch %d: kernel span %.2f us (first start to last end), %d expanded samples; scans: "
              "%d box too large, %d bin overflow" % (int(out[0, 9] >> np.uint64(16)), spans[-1], live.sum(),
                                                      (why & 1).astype(bool).sum(), (why & 2).astype(bool).sum()))
        print("  start skew: mean %.2f max %.2f us" % ((t[:, 0] - t0).mean() * 0.01, (t[:, 0] - t0).max() * 0.01))
        tt = t[live].copy()
        for q in range(1, 9):                                 # a stamp not reached stays 0: carry forward
            tt[:, q] = np.where(tt[:, q] == 0, tt[:, q - 1], tt[:, q])
        d = np.diff(tt, axis=1) * 0.01
        for q, nm in enumerate(NAMES):
            col = d[:, q]
            print("  %-9s mean %6.2f  p50 %6.2f  p90 %6.2f  p99 %6.2f  max %6.2f" % (
                nm, col.mean(), np.percentile(col, 50), np.percentile(col, 90), np.percentile(col, 99), col.max()))
        tot = (tt[:, 8] - tt[:, 0]) * 0.01
        print("  %-9s mean %6.2f  p50 %6.2f  p90 %6.2f  p99 %6.2f  max %6.2f" % (
            "total", tot.mean(), np.percentile(tot, 50), np.percentile(tot, 90), np.percentile(tot, 99), tot.max()))
        for w in np.argsort(tot)[-3:]:
            print("    slow sample: status %d phases %s" % (st[live][w], np.round(d[w], 1).tolist()))
    print("kernel spans of the mid-run launches: %s" % np.round(spans, 1).tolist())
    print_timeline(lib, 600 if nrows <= 8 else 120 * nrows)
    eng.close()


if __name__ == "__main__":
    main()
