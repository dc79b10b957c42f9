"""Benchmark: RRT candidate-sample expansions/s on MI355X (BASELINE.json metric).

One step = one batch iteration of the hot path (rrt.py:141-201 for B samples), everything inside
the timed region: the legacy gaussians rand_conf draws (rrt.py:58,66; drawn on the GPU from a
numpy RandomState state, bit for bit the np.random stream, rng.hip), sample -> NN argmin over the
whole tree -> steer -> body rays -> drive -> arc check, the device dedupe / append, and the host
bookkeeping replay of every record.

Workload = cfg2 by default: a 512x512 map2-style synthetic grid, 4096 samples per
GPU per step, a tree of <= 100k nodes.  The timed steps run in windows: before each window the
engine regrows its tree from the start pose to the prefill size (45k nodes, untimed; the --warmup
steps are the first steps of the first regrowth), and the window's 20 steps grow it further (to
just under 100k at N=1), so every timed step sees a tree in the same range however many steps are
timed.  value = all timed samples / the sum of the window times.  No timed window carries
instrumentation: the HIP-event kernel timings come from one extra, untimed window run first.

Multi-GPU (torchrun, one rank per GPU): every rank expands a contiguous slice of the step's global
batch against the replicated tree; the engine all-gathers the records over RCCL in rank order (=
global sample order) and every rank appends the same records.  Weak scaling: samples per GPU
fixed; the window is shortened to window/N steps so the timed node range stays the same.

Roofline: the dominant kernel by its mean HIP-event duration in the untimed instrumented window
(every batch, on the stream the kernel runs on; the events cost GPU time, which is why that
window is not part of `value`); HBM traffic per launch of that kernel from rocprofv3 PMC
passes (FETCH_SIZE x2 on gfx950 + WRITE_SIZE) of this same configuration, run as child processes
before this process touches the GPU.  Prints ONE JSON line on rank 0.
"""
import argparse
import csv
import glob
import json
import math
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "RRT node expansions/sec, batch=4096, 512x512 grid; 1/2/4/8 GPU"
NN_SCREEN_CEILING = 0.58     # 64 MFMA cycles of every ~110 (MFMA + 8 v_min3, serialized; tools/ubench_mfma_min.hip)
FP32_PEAK_TF = 157.3         # MI355X FP32 peak, matrix (v_mfma_f32_32x32x2_f32) = vector (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E peak (MI355X_MICROARCH.md)
NN_FLOP_PER_PAIR = 4         # the screen s = fma(ax, x, fma(by, y, w)): 2 FMA per (sample, node) pair
EXPAND_BYTES_PER_SAMPLE = 132   # k_expand_arc: sample 16 + near index 8 + near pose 24 + live 4 + record 80
PMC_KERNELS = ("k_expand_arc", "k_nn_pass1", "k_nn_grid")


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ------------------------------------------------------------------ PMC traffic (child passes)
def _short(name):
    return name.split("(")[0].replace("tr::", "").strip()


def pmc_traffic(args):
    """HBM bytes per launch of PMC_KERNELS over the timed window of a short run of this config:
    one rocprofv3 pass per counter (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass),
    FETCH_SIZE doubled (gfx950 counts half of wide coalesced reads), KB -> bytes."""
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    tmp = tempfile.mkdtemp(prefix="bench_pmc_")
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--config", args.config,
             "--seed", str(args.seed), "--lag", str(args.lag), "--stage", str(args.stage)]
    if args.batch:
        child += ["--batch", str(args.batch)]
    if args.prefill is not None:
        child += ["--prefill", str(args.prefill)]
    for kv in args.set:
        child += ["--set", kv]
    per = {}
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr)
            cmd = [prof, "--pmc", ctr, "--kernel-include-regex", "|".join(PMC_KERNELS), "-d", d,
                   "-o", "run", "--output-format", "csv", "--"] + child
            # counter collection serializes the dispatches of all streams; the engine finds that
            # out when the child creates its context and uses event edges there (option "gate");
            # the per-launch traffic of the kernels does not depend on the edges
            r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=180)
            if r.returncode != 0:
                tail = r.stderr.decode(errors="replace").strip().splitlines()[-1:] or [""]
                return None, "rocprofv3 %s pass failed (rc %d): %s" % (ctr, r.returncode, tail[0][:200])
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if not files:
                return None, "no counter_collection.csv from the %s pass" % ctr
            rows = list(csv.DictReader(open(files[0])))
            key = "Dispatch_Id" if "Dispatch_Id" in rows[0] else "Correlation_Id"
            rows.sort(key=lambda q: int(q[key]))
            for k in PMC_KERNELS:
                v = [float(q["Counter_Value"]) for q in rows
                     if _short(q["Kernel_Name"]) == k and q["Counter_Name"] == ctr]
                v = v[-args.window:]                        # the child's timed window
                per.setdefault(k, {})[ctr] = (sum(v) / len(v), len(v)) if v else (None, 0)
    except (subprocess.TimeoutExpired, OSError, KeyError, IndexError, ValueError) as e:
        return None, "PMC pass failed: %r" % (e,)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    out = {}
    for k, d in per.items():
        f, w = d.get("FETCH_SIZE", (None, 0)), d.get("WRITE_SIZE", (None, 0))
        if f[0] is None or w[0] is None:
            continue
        out[k] = {"hbm_bytes": 2 * f[0] * 1024 + w[0] * 1024, "fetch_bytes": 2 * f[0] * 1024,
                  "write_bytes": w[0] * 1024, "launches": f[1]}
    return out, "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, last %d launches of a %s window; " \
                "FETCH_SIZE x2 (gfx950), KB x 1024" % (args.window, args.config)


# ------------------------------------------------------------------ CPU baseline
def cpu_baseline(free, goal, nodes_xyt, budget_s, seed):
    """Pure-Python restatement (oracle) timed on one host core: per-sample expansion (NN over the
    whole snapshot + steer + rays + drive + arc) against the tree the GPU run ended with."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import thetarrt_oracle as O
    P = O.Params(tol_xy=0)
    g = O.Grid(free)
    snap = [((float(x), float(y)), float(t)) for x, y, t in nodes_xyt]
    rng = np.random.RandomState(seed + 1)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        q = O.samples_from_gauss(P, free.shape, goal, rng.standard_normal(3))[0]
        O.expand_one(P, g, snap, q)
        n += 1
    dt = time.perf_counter() - t0
    return n / dt, n, dt


def _config_batch(name):
    """Samples per GPU of a workloads.CONFIGS entry, read before anything touches the GPU
    (workloads.py imports only numpy; the package's __init__ is not run)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "tr_workloads", os.path.join(os.path.dirname(os.path.abspath(__file__)), "theta-rrt_amd", "workloads.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.CONFIGS[name]["batch"] if name in mod.CONFIGS else 4096


def finite(o):
    """The JSON line without NaN / Infinity tokens (a timing that was not taken reads null)."""
    if isinstance(o, dict):
        return {k: finite(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [finite(v) for v in o]
    if isinstance(o, (float, np.floating)):
        return float(o) if math.isfinite(o) else None
    return o


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--window", type=int, default=None,
                    help="timed steps per window (default 20 / N): the tree is regrown to the "
                         "prefill size before each window")
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--batch", type=int, default=None, help="samples per GPU per step")
    ap.add_argument("--prefill", type=int, default=None, help="untimed tree size before a window")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU-baseline work")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 traffic passes")
    ap.add_argument("--no-events", action="store_true",
                    help="skip the untimed instrumented window (no kernel_us / roofline times)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--lag", type=int, default=4, choices=range(1, 6),
                    help="batches between a dedupe and its commit (commit ring of 6)")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="collective backend for N > 1 (nccl = RCCL over xGMI)")
    ap.add_argument("--same-device", action="store_true",
                    help="all ranks on GPU 0 (rehearsal of the multi-rank path, with gloo)")
    ap.add_argument("--force-comm", action="store_true",
                    help="engine RCCL communicator even at N=1 (exercises the sharded code path)")
    ap.add_argument("--python-loop", action="store_true",
                    help="drive the batches from Python (the gloo rehearsal loop) also at N=1")
    ap.add_argument("--stage", type=int, default=None, choices=(0, 1, 2),
                    help="look-ahead depth: batches whose NN sweep runs ahead on the side stream "
                         "(default 1 for a global batch of up to 8192 samples, else 0)")
    ap.add_argument("--set", action="append", default=[], metavar="OPTION=VALUE",
                    help="engine option for an A/B run (tr_set_option; recorded in "
                         "config.engine_options)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.stage is None:
        # the look-ahead's correction scans every node the last global batch appended: measured
        # on one GPU (profiles/r02/scale/, profiles/r02/cfg3/), past a global batch of 8192 the NN
        # sweep on the batch's own stream costs less than the correction (cfg2 at N <= 2)
        bt = (args.batch or _config_batch(args.config)) * world
        args.stage = 1 if bt <= 8192 else 0
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.window is None:
        args.window = max(2, 20 // world)
    if args.pmc_child:
        args.steps, args.warmup, args.no_cpu = args.window, 1, True

    # PMC passes first: this process has not initialised the GPU yet (children own it meanwhile)
    traffic, traffic_note = None, "not collected (N > 1 or --no-pmc)"
    if rank == 0 and world == 1 and not args.no_pmc and not args.pmc_child:
        traffic, traffic_note = pmc_traffic(args)

    # The JSON line is the only thing on stdout: native libraries (RCCL's init banner) write to
    # fd 1, so fd 1 is pointed at stderr for the run and the result goes to the saved stdout.
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)
    import torch
    import pkgload
    pkgload.load()
    from theta_rrt_amd import _native, workloads

    if args.config not in workloads.CONFIGS:
        sys.exit("unknown config %s (have %s)" % (args.config, sorted(workloads.CONFIGS)))
    if args.same_device:                  # rehearsal of the multi-rank path on one GPU
        local = 0
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)

    cfg = workloads.CONFIGS[args.config]
    n_grid = cfg["grid"]
    B = args.batch or cfg["batch"]
    BT = B * world
    prefill = cfg["prefill"] if args.prefill is None else args.prefill

    free = workloads.map2_style(n_grid, seed=args.seed)
    sx, sy = workloads.nearest_free(free, cfg["start"], cfg["start"])
    start3 = [float(sx), float(sy), 0.0]
    goal3 = [n_grid / 2, n_grid / 2, 0.0]

    dev = torch.device("cuda", local)
    eng = _native.Engine(local)
    # One explicit stream for the engine AND every torch op of the loop: torch's default stream is
    # the legacy null stream, which the engine's non-blocking streams do not order against.
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    eng.set_params(_native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1))  # tol_xy 0, reject
    eng.set_grid(free)
    eng.rng_set_state(np.random.RandomState(args.seed).get_state())   # rand_conf's np.random stream
    # HIP-event timing of the kernels (every batch of a run, on each kernel's stream) costs GPU
    # time: it runs in an extra untimed window before the timed ones, which run without events
    events = not args.no_events and not args.pmc_child
    # the library reads nothing from the environment; what can change its paths is recorded
    for kv in args.set:
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    options = {}
    for k in ("gate", "dd_fused", "dd_fused_max", "dd_gatefold", "fused_delta", "delta_bins", "nn_grid", "nn_far_sweep", "nn_far_nodes", "nn_grid_min",
              "book"):
        try:
            options[k] = eng.get_option(k)
        except _native.NativeError:            # (an older build of the library in an A/B run)
            pass
    tr_env = sorted(k for k in os.environ if k.startswith("TR_"))
    if tr_env:
        sys.exit("bench.py: TR_* environment variables are set (%s); the engine has no "
                 "environment knobs, unset them" % ", ".join(tr_env))

    nslot = max(2, args.stage + 1)                 # sample / record sets the look-ahead rotates
    samp2 = torch.empty(nslot * B * 16, dtype=torch.uint8, device=dev)
    recs2 = torch.empty(nslot * B * 80, dtype=torch.uint8, device=dev)
    native = not args.python_loop and (world == 1 or args.backend == "nccl")
    use_comm = native and (world > 1 or args.force_comm)
    samp_all2 = recs_all2 = None
    if use_comm:
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            uid = torch.tensor(list(eng.comm_unique_id()), dtype=torch.uint8)
        if dist:
            uid = uid.to(dev)
            dist.broadcast(uid, 0)
        eng.comm_init(rank, world, bytes(uid.cpu().tolist()))
        if rank:                          # one rank reports the tree: the others keep the device
            eng.set_option("book", 0)     # replica only (no host replay of the global batches)
        samp_all2 = torch.empty(2 * BT * 16, dtype=torch.uint8, device=dev)
        recs_all2 = torch.empty(2 * BT * 80, dtype=torch.uint8, device=dev)

    # gloo rehearsal (Python loop): the all-gather goes through the host
    if not native:
        samp = [torch.empty(B * 16, dtype=torch.uint8, device=dev) for _ in range(2)]
        recs = [torch.empty(B * 80, dtype=torch.uint8, device=dev) for _ in range(2)]
        samp_all = [torch.empty(BT * 16, dtype=torch.uint8, device=dev) for _ in range(2)]
        recs_all = [torch.empty(BT * 80, dtype=torch.uint8, device=dev) for _ in range(2)]
        gbuf = [torch.empty(3 * BT, dtype=torch.float64, device=dev) for _ in range(2)]

    def gather(out, inp):
        if args.backend == "nccl":
            dist.all_gather_into_tensor(out, inp)
        else:
            parts = [torch.empty_like(inp, device="cpu") for _ in range(world)]
            dist.all_gather(parts, inp.cpu())
            out.copy_(torch.cat(parts).to(out.device))

    def run_steps(rows):
        """`rows` batches; the engine draws their gaussians.  Returns the node count after."""
        if native:
            n, _ = eng.run(None, B, rows, samp2.data_ptr(), recs2.data_ptr(), lag=args.lag,
                           stage=args.stage,
                           d_samples_all=samp_all2.data_ptr() if use_comm else 0,
                           d_records_all=recs_all2.data_ptr() if use_comm else 0)
            return n
        n = eng.book().size()
        for i in range(rows):
            k = i & 1
            eng.rng_gauss_dev(3 * BT, gbuf[k].data_ptr())
            eng.pipe_expand(gbuf[k][3 * B * rank:].data_ptr(), B, samp[k].data_ptr(), recs[k].data_ptr())
            if world > 1:
                gather(samp_all[k], samp[k])
                gather(recs_all[k], recs[k])
                eng.pipe_dedupe(samp_all[k].data_ptr(), recs_all[k].data_ptr(), BT)
            else:
                eng.pipe_dedupe(samp[k].data_ptr(), recs[k].data_ptr(), BT)
            if eng.pending() > args.lag:
                n, _ = eng.pipe_commit()
        while eng.pending():
            n, _ = eng.pipe_commit()
        return n

    warm = [args.warmup]                            # untimed warm-up: the first regrowth's first steps

    def fresh_tree():
        """Regrow the tree from the start pose to >= prefill nodes (untimed): runs of 4 steps, then
        single steps, so the window starts within one step's growth of the prefill size."""
        eng.rrt_begin(start3, goal3)
        eng.rrt_reserve(int(prefill * 1.3) + (args.window + 8) * BT, BT)
        n, grow = 1, 0
        if warm[0]:
            n = run_steps(warm[0])
            warm[0] = 0
        while n < prefill:
            k = 4 if n + 6 * grow < prefill else 1
            m = run_steps(k)
            grow = max(grow, (m - n) // k)
            n = m
        return n

    n_win = (args.steps + args.window - 1) // args.window
    wins = []                                       # (steps, seconds, n0, n1, run stats)
    t_pre = 0.0
    kern_win = ({}, (0, 0))
    kern_last = None
    if native and events:                           # the instrumented window: untimed, not in value
        tp = time.perf_counter()
        fresh_tree()
        # (with look-ahead: level 1's events on every batch, each kernel on its own stream;
        # without: every phase of a batch on the context stream, level 2)
        eng.enable_timing(3 if args.stage > 0 else 2)
        run_steps(min(args.window, args.steps))
        kern_win = eng.last_run_kernel_us()
        kern_last = eng.last_run_stats()[0]          # the window's last batch, phase by phase
        eng.enable_timing(0)
        t_pre += time.perf_counter() - tp
    for w in range(n_win):
        rows = min(args.window, args.steps - w * args.window)
        tp = time.perf_counter()
        n0 = fresh_tree()
        t_pre += time.perf_counter() - tp
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n1 = run_steps(rows)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        st, _ = eng.last_run_stats() if native else ([0.0] * 11, 0)
        wins.append((rows, el, n0, n1, st))
    log(rank, "%d timed windows of <= %d steps; untimed tree regrowth + instrumented window %.1fs"
        % (n_win, args.window, t_pre))
    if args.pmc_child:
        return

    K = sum(wn[0] for wn in wins)
    el = sum(wn[1] for wn in wins)
    value = K * BT / el
    rates = np.array([wn[0] * BT / wn[1] for wn in wins])
    n_lo, n_hi = min(wn[2] for wn in wins), max(wn[3] for wn in wins)

    # kernel means over every batch of the instrumented window.  The nearest-node work is timed
    # as two spans on its stream: the sweep and its resolve, or (cell lists, the default up to
    # option nn_grid) the three build launches and the query (with the far list: and its sweep).
    nmin = options.get("nn_grid_min", -1)
    cells = bool(options.get("nn_grid")) and prefill >= (nmin if nmin >= 0 else n_grid * n_grid // 8)
    far_sweep = cells and BT >= options.get("nn_far_sweep", 1 << 62)
    nn_a, nn_b = (("cell_build", "k_nn_grid+far_sweep" if far_sweep else "k_nn_grid") if cells
                  else ("k_nn_pass1", "k_nn_resolve"))
    samples = kern_win[1]
    raw = kern_win[0]
    kern_us = {nn_a: raw.get("k_nn_pass1", float("nan")) if samples[0] else float("nan"),
               nn_b: raw.get("k_nn_resolve", float("nan")) if samples[0] else float("nan")}
    for k in ("k_nn_delta", "k_expand_arc", "dedupe"):
        kern_us[k] = raw.get(k, float("nan")) if samples[1] else float("nan")
    last_only = False
    if kern_last is not None and not samples[0] and not samples[1]:
        # a run without look-ahead (global batches past 8192 samples) samples no batch that way:
        # the HIP events around the phases of the instrumented window's last batch instead (the
        # nearest-node span then holds the cell lists' build as well)
        if kern_last[1] > 0:
            kern_us[nn_b] = kern_last[0]
            kern_us["k_expand_arc"] = kern_last[1]
            kern_us["dedupe"] = kern_last[3]
            samples = (1, 1)
            last_only = True

    n_mid = float(np.mean([0.5 * (wn[2] + wn[3]) for wn in wins]))
    grow = float(np.mean([(wn[3] - wn[2]) / wn[0] for wn in wins]))
    if cells:
        # Roofline of the cell-list query: per sample the 8-byte sample and its live word, the item
        # ranges of the 3 x 3 cells around it (18 words), those cells' nodes (24-byte items; the
        # cell side the engine plans for the tree size: about 12 nodes per cell at twice the nodes)
        # and 16 bytes out; HBM-side bytes, although the loads are dependent round trips
        side = math.sqrt(12.0 * n_grid * n_grid / (2.0 * n_mid))
        cs = 0
        while cs < 8 and (2 << cs) <= side:
            cs += 1
        per_cell = n_mid * (1 << cs) ** 2 / float(n_grid * n_grid)
        q_bytes = B * (12 + 72 + 24 * 9 * per_cell + 16)
        tr_nn = (traffic or {}).get("k_nn_grid")
        t_nn = kern_us[nn_b]
        roof_nn = {"kernel": nn_b, "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                   "achieved": q_bytes / (t_nn * 1e-6) / 1e9, "launch_us": t_nn,
                   "algorithmic_bytes": q_bytes, "traffic": tr_nn["hbm_bytes"] if tr_nn else None,
                   "note": "latency-bound: three dependent round trips per sample (sample, cell "
                           "ranges, nodes) by 16 lanes; the sweep it replaces evaluated %.3g "
                           "(sample, node) pairs per batch" % (B * n_mid)}
        roof_nn["frac"] = roof_nn["achieved"] / roof_nn["peak"]
    else:
        # Roofline of the k_nn_pass1 sweep: 4 flop per (sample, node) pair on the
        # f32 matrix cores; a sweep staged `stage` batches ahead covers the tree `stage` steps back.
        pairs = B * max(1.0, n_mid - max(args.stage, 0) * grow)
        tr_nn = (traffic or {}).get("k_nn_pass1")
        t_nn = kern_us["k_nn_pass1"]
        roof_nn = {"kernel": "k_nn_pass1", "bound": "mfma", "unit": "TFLOP/s", "peak": FP32_PEAK_TF,
                   "achieved": NN_FLOP_PER_PAIR * pairs / (t_nn * 1e-6) / 1e12, "launch_us": t_nn,
                   "pairs_per_launch": pairs, "algorithmic_bytes": 16 * n_mid + 8 * B,
                   "traffic": tr_nn["hbm_bytes"] if tr_nn else None,
                   # the HBM side of the same launch: measured bytes per launch time, against 8 TB/s
                   "hbm_gbs": (tr_nn["hbm_bytes"] / (t_nn * 1e-6) / 1e9) if tr_nn and t_nn > 0 else None,
                   "hbm_frac": (tr_nn["hbm_bytes"] / (t_nn * 1e-6) / 1e9 / HBM_PEAK_GBS)
                               if tr_nn and t_nn > 0 else None}
        roof_nn["frac"] = roof_nn["achieved"] / roof_nn["peak"]
        # the f32-input MFMA does not overlap the minimum trees' v_min3 on its SIMD (measured: 65 +
        # 45 = 104 cycles per MFMA slot, tools/ubench_mfma_min.hip), so the screen tops out here
        roof_nn["ceiling_frac"] = NN_SCREEN_CEILING
        roof_nn["frac_of_ceiling"] = roof_nn["frac"] / NN_SCREEN_CEILING
    # k_expand_arc: latency-bound fp64 chains; its algorithmic bytes per launch are the per-sample
    # operands and record (EXPAND_BYTES_PER_SAMPLE) plus the grid read once.
    tr_ex = (traffic or {}).get("k_expand_arc")
    t_ex = kern_us["k_expand_arc"]
    ex_bytes = EXPAND_BYTES_PER_SAMPLE * BT + n_grid * n_grid
    roof_ex = {"kernel": "k_expand_arc", "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
               "achieved": ex_bytes / (t_ex * 1e-6) / 1e9, "launch_us": t_ex,
               "algorithmic_bytes": ex_bytes, "traffic": tr_ex["hbm_bytes"] if tr_ex else None,
               "note": "latency-bound: one sample's dependent fp64 steer/arc chain per 16 lanes"}
    roof_ex["frac"] = roof_ex["achieved"] / roof_ex["peak"]
    dominant = roof_ex if not (t_nn > t_ex) else roof_nn
    other = roof_nn if dominant is roof_ex else roof_ex
    roof = dict(dominant)
    roof["traffic_source"] = traffic_note
    roof["timing"] = ("mean HIP-event duration on the kernel's stream over %d batches (every batch "
                      "of an untimed instrumented window run before the timed ones)" %
                      (samples[1] if dominant is roof_ex else samples[0])) if not last_only else (
        "HIP events around the phases of the last batch of an untimed instrumented window (a run "
        "without look-ahead: every phase on the context stream)")

    st = np.mean([wn[4] for wn in wins], axis=0)
    out = {
        "metric": METRIC, "value": value, "unit": "candidate-sample expansions/s", "n_gpus": world,
        "steps": K, "warmup": args.warmup, "ms_per_step": el / K * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "%s: %dx%d map2-style grid (8%% occupied), %d samples/GPU/step; tree "
                               "regrown to %d nodes before each of %d windows of <= %d timed steps "
                               "(timed tree range %d..%d nodes); gaussians drawn on the GPU inside "
                               "the timed steps" % (args.config, n_grid, n_grid, B, prefill, n_win,
                                                    args.window, n_lo, n_hi),
                   "global_batch": BT, "grid": [n_grid, n_grid], "tree_nodes": [n_lo, n_hi],
                   "windows": n_win, "window_steps": args.window, "engine_options": options,
                   "parallelism": "sample-sharded x%d, replicated tree, RCCL all-gather of records"
                                  % world + ("" if native else " (Python loop)")},
        "window_rates": {"median": float(np.median(rates)), "min": float(rates.min()),
                         "max": float(rates.max()), "n": int(len(rates)),
                         "all": [round(float(r)) for r in rates]},
        "kernel_us": kern_us, "kernel_us_samples": {"side": samples[0], "main": samples[1]},
        "host_us_per_step": {"commit_wait": st[8], "replay": st[9], "enqueue": st[10]},
        "roofline": roof, "roofline_secondary": other,
    }
    try:                                   # batches whose commit head reached the host after their flag
        out["host_us_per_step"]["head_waits"] = eng.get_option("head_waits")
    except _native.NativeError:
        pass
    if rank == 0 and world == 1 and not args.no_cpu:
        nodes = eng.book().nodes()
        rate, n, dt = cpu_baseline(free, (tuple(goal3[:2]), goal3[2]), nodes, args.cpu_budget, args.seed)
        out["cpu_baseline"] = {"value": rate, "unit": "candidate-sample expansions/s", "cores": 1,
                               "kind": "port", "cpu": cpu_model(),
                               "sample": "%d samples expanded one by one (pure-Python oracle, reference "
                                         "call pattern) against the final %d-node tree, %.1fs on one "
                                         "host core" % (n, len(nodes), dt)}
    if rank == 0:
        os.write(out_fd, (json.dumps(finite(out)) + "\n").encode())
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
