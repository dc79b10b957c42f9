"""Benchmark: RRT candidate-sample expansions/s on MI355X (BASELINE.json metric).

One step = one batch iteration of the hot path (rrt.py:141-201 for B samples): the fused GPU pass
(sample -> NN argmin over the whole tree -> steer -> body rays -> drive -> arc check) followed by the
host bookkeeping append and the device tree update.  Default workload = cfg2: a
512x512 map2-style synthetic grid, 4096 samples per GPU per step, tree grown by the engine itself
(untimed prefill) to >= 50k nodes before the timed steps, which keep growing it.

Multi-GPU (torchrun, one rank per GPU): every rank expands a contiguous slice of the step's global
batch against the replicated tree, the accepted-node records are all-gathered over RCCL in rank
order (= global sample order), and every rank appends the same records, so trees stay identical.
Weak scaling: samples per GPU fixed.

Inputs (the legacy-gaussian stream rand_conf consumes, rrt.py:58,66) are pre-generated and resident
in HBM before the timed region.  Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from theta_rrt_amd import _native, workloads  # noqa: E402

DEBUG = os.environ.get("BENCH_DEBUG") is not None
if DEBUG:
    import faulthandler
    faulthandler.dump_traceback_later(int(os.environ.get("BENCH_DEBUG") or 60), exit=True)
METRIC = "RRT node expansions/sec, batch=4096, 512x512 grid; 1/2/4/8 GPU"
FP32_PEAK_TF = 157.3         # MI355X FP32 peak, matrix (v_mfma_f32_32x32x2_f32) = vector (MI355X_MICROARCH.md)
NN_FLOP_PER_PAIR = 4         # the screen s = fma(ax, x, fma(by, y, w)): 2 FMA per (sample, node) pair


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def pmc_traffic(kern):
    """HBM bytes per k_nn_pass1 launch from the committed rocprofv3 PMC passes (FETCH_SIZE x 2 for
    gfx950's half-counted wide reads + WRITE_SIZE, KB -> bytes; tools/pmc_traffic.py), or None."""
    f = os.path.join(ROOT, "profiles", "r01", "nn_pass1_pmc.json")
    if not kern.startswith("k_nn_pass1 (") or not os.path.exists(f):
        return None
    with open(f) as fh:
        return json.load(fh).get("hbm_bytes_per_launch")


def cpu_baseline(free, start, goal, nodes_xyt, budget_s, seed):
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


def main():
    # The JSON line is the only thing on stdout: native libraries (RCCL's init banner) write to
    # fd 1, so fd 1 is pointed at stderr for the run and the result goes to the saved stdout.
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg2", choices=sorted(workloads.CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="samples per GPU per step")
    ap.add_argument("--prefill", type=int, default=None, help="untimed tree growth target (nodes)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="seconds of CPU-baseline work")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--phases", action="store_true", help="HIP-event time every phase (adds gaps)")
    ap.add_argument("--lag", type=int, default=4, choices=range(1, 6),
                    help="batches between a dedupe and its commit (commit ring of 6)")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="collective backend for N > 1 (nccl = RCCL over xGMI)")
    ap.add_argument("--same-device", action="store_true",
                    help="all ranks on GPU 0 (rehearsal of the multi-rank path, with gloo)")
    ap.add_argument("--force-comm", action="store_true",
                    help="engine RCCL communicator even at N=1 (exercises the sharded code path)")
    ap.add_argument("--python-loop", action="store_true",
                    help="drive the batches from Python (the multi-GPU loop) also at N=1")
    ap.add_argument("--stage", type=int, default=1, choices=(0, 1, 2),
                    help="look-ahead depth: batches whose NN sweep runs ahead on the side stream")
    ap.add_argument("--no-stage", dest="stage", action="store_const", const=0,
                    help="no look-ahead (= --stage 0)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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

    n_grid, b_default, pre_default = workloads.CONFIGS[args.config]
    B = args.batch or b_default
    BT = B * world
    prefill = pre_default if args.prefill is None else args.prefill

    free = workloads.map2_style(n_grid, seed=args.seed)
    sx, sy = workloads.nearest_free(free, 16, 16)
    start = ((sx, sy), 0.0)
    goal = ((n_grid // 2, n_grid // 2), 0.0)

    eng = _native.Engine(local)
    # One explicit stream for the engine AND every torch op of the loop (the all-gather of records,
    # its copies): torch's default stream is the legacy null stream, which the engine's
    # non-blocking streams do not order against.
    stream = torch.cuda.Stream(device=torch.device("cuda", local))
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    p = _native.tr_params(5, -65, 65, 2, 30, .6, .4, 100, 0, 45, 1, 1)   # tol_xy = 0, straight_reject
    eng.set_params(p)
    eng.set_grid(free)
    eng.rrt_begin([sx, sy, 0.0], [goal[0][0], goal[0][1], 0.0])
    eng.enable_timing(0 if os.environ.get("TR_BENCH_NO_EVENTS") else (2 if args.phases else 1))

    dev = torch.device("cuda", local)
    # two sets of sample/record buffers: batch b+1 is staged while batch b is in flight
    samp = [torch.empty(B * 16, dtype=torch.uint8, device=dev) for _ in range(2)]
    recs = [torch.empty(B * 80, dtype=torch.uint8, device=dev) for _ in range(2)]
    if world > 1:
        samp_all = [torch.empty(BT * 16, dtype=torch.uint8, device=dev) for _ in range(2)]
        recs_all = [torch.empty(BT * 80, dtype=torch.uint8, device=dev) for _ in range(2)]
    else:
        samp_all, recs_all = samp, recs
    rs = np.random.RandomState(args.seed)          # MT19937 legacy gaussians, as np.random uses
    state = {"nodes": 1}
    phase = np.zeros(5)
    hostp = np.zeros(3)
    nnp = np.zeros(3)
    enq = [0.0]                                       # host time spent enqueueing (s)
    counted = [0]
    eng.rrt_reserve(int(prefill * 1.3) + (args.warmup + args.steps + 4) * BT, BT)

    def gather(out, inp):
        """Rank-order all-gather (RCCL on the engine's stream; gloo rehearsal through the host)."""
        if args.backend == "nccl":
            dist.all_gather_into_tensor(out, inp)
        else:
            parts = [torch.empty_like(inp, device="cpu") for _ in range(world)]
            dist.all_gather(parts, inp.cpu())
            out.copy_(torch.cat(parts).to(out.device))

    def sl(g):
        return g[3 * B * rank: 3 * B * (rank + 1)]

    # Pipelined batch loop (include/thetarrt.h): the tree and its dedupe live on the GPU, so
    # batch b+1 is enqueued while the host replays batch b, and batch b+1 is expanded against the
    # tree before batch b's append on a side stream beside batch b (pipe_stage), then corrected for
    # batch b's nodes; results equal the sequential loop's.
    def run_batches(gauss_rows, timed=False):
        n = state["nodes"]
        for i, g in enumerate(gauss_rows):
            k = i & 1
            te = time.perf_counter()
            eng.pipe_expand(sl(g).data_ptr(), B, samp[k].data_ptr(), recs[k].data_ptr())
            if args.stage and i + 1 < len(gauss_rows):
                eng.pipe_stage(sl(gauss_rows[i + 1]).data_ptr(), B, samp[k ^ 1].data_ptr(),
                               recs[k ^ 1].data_ptr())
            if DEBUG:
                print("rank %d batch %d expanded, pending %d" % (rank, i, eng.pending()),
                      file=sys.stderr, flush=True)
            if world > 1:
                gather(samp_all[k], samp[k])
                gather(recs_all[k], recs[k])
                if DEBUG:                           # ranks must see the same gathered batch
                    cs = torch.stack([recs_all[k].view(torch.int64).sum(),
                                      samp_all[k].view(torch.int64).sum()]).cpu()
                    ref = cs.clone()
                    dist.broadcast(ref, 0)
                    if not torch.equal(cs, ref):
                        print("rank %d batch %d: gathered batch differs from rank 0" % (rank, i),
                              file=sys.stderr, flush=True)
            eng.pipe_dedupe(samp_all[k].data_ptr(), recs_all[k].data_ptr(), BT)
            if timed:
                enq[0] += time.perf_counter() - te
            if eng.pending() > args.lag:
                n, _ = eng.pipe_commit()
                if timed:
                    acc()
        while eng.pending():
            n, _ = eng.pipe_commit()
            if timed:
                acc()
        state["nodes"] = n

    def acc():
        phase[:] += np.array(eng.last_timings())
        hostp[:] += np.array(eng.last_host_timings())
        nnp[:] += np.array(eng.last_nn_timings())
        counted[0] += 1

    # The same pipeline driven by the native loop (tr_rrt_run), no per-batch Python; with N > 1 the
    # engine all-gathers the records over its own RCCL communicator on the engine stream.
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
        samp_all2 = torch.empty(2 * BT * 16, dtype=torch.uint8, device=dev)
        recs_all2 = torch.empty(2 * BT * 80, dtype=torch.uint8, device=dev)

    def run_native(gauss_block, timed=False):
        te = time.perf_counter()
        n, _ = eng.run(gauss_block.data_ptr(), B, gauss_block.shape[0], samp2.data_ptr(),
                       recs2.data_ptr(), lag=args.lag, stage=args.stage,
                       d_samples_all=samp_all2.data_ptr() if use_comm else 0,
                       d_records_all=recs_all2.data_ptr() if use_comm else 0)
        state["nodes"] = n
        if timed:
            st, commits = eng.last_run_stats()
            phase[:] = st[0:5]
            nnp[:] = st[5:8]
            hostp[:] = np.array(st[8:11]) * gauss_block.shape[0]
            counted[0] = 1
            enq[0] = st[10] * 1e-6 * gauss_block.shape[0]   # host enqueue time (native loop)

    # untimed prefill: the engine grows its own tree to the benchmark's size
    t_pre = time.perf_counter()
    n_pre = 0
    while state["nodes"] < prefill:
        rows = torch.from_numpy(rs.standard_normal((4, 3 * BT))).to(dev)
        if native:
            run_native(rows)
        else:
            run_batches([rows[i] for i in range(4)])
        n_pre += len(rows)
    log(rank, "prefill: %d steps -> %d nodes in %.1fs" % (n_pre, state["nodes"], time.perf_counter() - t_pre))

    total = args.warmup + args.steps
    gauss = torch.from_numpy(rs.standard_normal((total, 3 * BT))).to(dev)   # resident in HBM
    if native:
        run_native(gauss[:args.warmup])
    else:
        run_batches([gauss[i] for i in range(args.warmup)])
    n0 = state["nodes"]

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if native:
        run_native(gauss[args.warmup:total], timed=True)
    else:
        run_batches([gauss[i] for i in range(args.warmup, total)], timed=True)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    n1 = state["nodes"]

    K = args.steps
    value = K * BT / el
    avg = phase / max(1, counted[0])                  # per-batch microseconds (HIP events)
    nn_t = nnp / max(1, counted[0])                   # [staged sweep (side stream), NN on the path]
    n_mid = 0.5 * (n0 + n1)
    # Roofline of the dominant kernel, the nearest-node sweep k_nn_pass1: its fp32
    # screen is 2 FMA = 4 flop per (sample, node) pair, on the f32 matrix cores (one
    # v_mfma_f32_32x32x2_f32 per 32 x 32 pairs; TR_NN_VALU=1: the same screen on the VALU), against
    # the 157.3 TF FP32 peak (matrix = vector on gfx950).  The tree sits in L2: HBM does not bound it.
    # Its time is the mean HIP-event duration of every k_nn_pass1 launch of the timed run (side
    # stream).  A sweep staged `stage` batches ahead covers the tree `stage` batches back: N_mid
    # minus that many steps' appended nodes.
    grow = (n1 - n0) / max(1, K)
    if args.stage and nn_t[2] > 0:
        kern, t_us = "k_nn_pass1 (snapshot sweep, side stream)", nn_t[2]
        pairs = B * max(1.0, n_mid - args.stage * grow)
    else:
        kern, t_us = "k_nn_pass1+k_nn_resolve", avg[0]
        pairs = B * n_mid
    t_us = t_us if t_us > 0 else float("nan")        # timing events disabled
    bound = "valu" if os.environ.get("TR_NN_VALU") else "mfma"
    roof = {"kernel": kern, "bound": bound, "achieved": NN_FLOP_PER_PAIR * pairs / (t_us * 1e-6) / 1e12,
            "peak": FP32_PEAK_TF, "unit": "TFLOP/s", "traffic": pmc_traffic(kern),
            "launch_us": t_us, "pairs_per_launch": pairs}
    roof["frac"] = roof["achieved"] / roof["peak"]
    out = {
        "metric": METRIC, "value": value, "unit": "candidate-sample expansions/s", "n_gpus": world,
        "steps": K, "warmup": args.warmup, "ms_per_step": el / K * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "%s: %dx%d map2-style grid (8%% occupied), %d samples/GPU/step, tree grown "
                               "by the engine from %d to %d nodes over the timed steps"
                               % (args.config, n_grid, n_grid, B, n0, n1),
                   "global_batch": BT, "grid": [n_grid, n_grid], "tree_nodes": [n0, n1],
                   "parallelism": "sample-sharded x%d, replicated tree, RCCL all-gather of records"
                                  % world + ("" if native else " (Python loop)")},
        "phase_us_per_step": {"nn_staged_sweep": nn_t[0], "nn": avg[0], "expand": avg[1],
                              "arc": avg[2], "dedupe": avg[3],
                              "gpu_sum": avg[4], "host_commit_wait": hostp[0] / K,
                              "host_replay": hostp[1] / K, "host_enqueue": None if enq[0] is None else enq[0] / K * 1e6},
        "roofline": roof,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        nodes = eng.book().nodes()
        rate, n, dt = cpu_baseline(free, start, goal, nodes, args.cpu_budget, args.seed)
        out["cpu_baseline"] = {"value": rate, "unit": "candidate-sample expansions/s", "cores": 1,
                               "kind": "port",
                               "sample": "%d samples expanded one by one (pure-Python oracle, reference "
                                         "call pattern) against the final %d-node tree, %.1fs"
                                         % (n, len(nodes), dt)}
    if rank == 0:
        os.write(out_fd, (json.dumps(out) + "\n").encode())
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
