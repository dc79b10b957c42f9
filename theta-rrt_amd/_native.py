"""ctypes binding of libthetarrt.so (include/thetarrt.h).

The product has no CPU fallback: if the HIP library is missing or no GPU is visible, every compute
entry point raises.  Host-only pieces (the bookkeeping `tr_book_*`) work without a GPU.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# THETARRT_LIB: another build of the same library (the sanitizer variants, theta-rrt_amd/build.py)
LIB_PATH = os.environ.get("THETARRT_LIB") or os.path.join(HERE, "libthetarrt.so")

TR_OK, TR_E_ARG, TR_E_HIP, TR_E_STRAIGHT, TR_E_INDEX, TR_E_STATE, TR_E_VALUE = 0, -1, -2, -3, -4, -5, -6
ST_SKIP, ST_COLLISION, ST_OK, ST_STRAIGHT, ST_INDEX, ST_CONSTRAINT = 0, 2, 3, 4, 5, 7
FL_DROVE, FL_GOAL, FL_STRAIGHT, FL_INDEX_SAMPLE, FL_MEMBER, FL_SAME_NEAR = 1, 2, 4, 8, 16, 32


class tr_params(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("bikelength", "leftconstraint", "rightconstraint",
                                          "frontclearance", "maxdrivedist", "weightxy", "xystdv",
                                          "anglestdv", "tol_xy", "tol_ang")] + \
               [("forwardonly", C.c_int32), ("straight_reject", C.c_int32)]


SAMPLE_DTYPE = np.dtype([("x", np.int32), ("y", np.int32), ("th", np.float64)])
RECORD_DTYPE = np.dtype([("x", np.float64), ("y", np.float64), ("th", np.float64),
                         ("steer", np.float64), ("iccx", np.float64), ("iccy", np.float64),
                         ("rad", np.float64), ("dist", np.float64), ("near", np.int64),
                         ("status", np.int16), ("flags", np.int16), ("ex", np.int32)])
RESOLVED_DTYPE = np.dtype([("r", RECORD_DTYPE), ("idx", np.int64), ("flags", np.int32),
                           ("pad", np.int32)])
RS_MEMBER, RS_SAME_NEAR, RS_FIRST = 1, 2, 4
assert SAMPLE_DTYPE.itemsize == 16 and RECORD_DTYPE.itemsize == 80 and RESOLVED_DTYPE.itemsize == 96

P = C.c_void_p
I64 = C.c_int64
I64P = C.POINTER(C.c_int64)
DP = C.POINTER(C.c_double)

HOST_GATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64)

_SIGS = {
    "tr_last_error": (C.c_char_p, []),
    "tr_version": (C.c_int, []),
    "tr_create": (C.c_int, [C.c_int, C.POINTER(P)]),
    "tr_destroy": (C.c_int, [P]),
    "tr_set_stream": (C.c_int, [P, P]),
    "tr_sync": (C.c_int, [P]),
    "tr_set_params": (C.c_int, [P, C.POINTER(tr_params)]),
    "tr_set_grid": (C.c_int, [P, P, I64, I64]),
    "tr_tree_reset": (C.c_int, [P, I64]),
    "tr_tree_append": (C.c_int, [P, P, I64]),
    "tr_tree_size": (I64, [P]),
    "tr_nn_batch": (C.c_int, [P, P, I64, P, P]),
    "tr_set_option": (C.c_int, [P, C.c_char_p, I64]),
    "tr_get_option": (C.c_int, [P, C.c_char_p, I64P]),
    "tr_los_batch": (C.c_int, [P, P, I64, P]),
    "tr_los_batch_dev": (C.c_int, [P, P, I64, P]),
    "tr_steer_batch": (C.c_int, [P, P, I64, P]),
    "tr_drive_batch": (C.c_int, [P, P, I64, P, P]),
    "tr_body_clear_batch": (C.c_int, [P, P, I64, C.c_double, P]),
    "tr_arc_batch": (C.c_int, [P, P, I64, P]),
    "tr_bresenham": (C.c_int, [P, P, P, I64, I64P]),
    "tr_circle": (C.c_int, [P, C.c_double, C.c_double, C.c_double, P, I64, I64P]),
    "tr_arc_pixels": (C.c_int, [P, P, P, I64, I64P]),
    "tr_expand_dev": (C.c_int, [P, P, I64, P, P, P]),
    "tr_expand_dev_noalloc": (C.c_int, [P, P, I64, P, P, P]),
    "tr_book_create": (C.c_int, [C.POINTER(P)]),
    "tr_book_destroy": (C.c_int, [P]),
    "tr_book_reset": (C.c_int, [P, P]),
    "tr_book_ingest": (C.c_int, [P, P, P, I64, I64, I64P, I64P]),
    "tr_book_set_straight_reject": (C.c_int, [P, C.c_int]),
    "tr_book_replay": (C.c_int, [P, P, I64, I64P, I64P]),
    "tr_book_reserve": (C.c_int, [P, I64, I64]),
    "tr_book_size": (I64, [P]),
    "tr_book_edges": (I64, [P]),
    "tr_book_nodes": (C.c_int, [P, I64, I64, P]),
    "tr_book_export": (C.c_int, [P, P, P, P, P]),
    "tr_rrt_begin": (C.c_int, [P, P, P]),
    "tr_rrt_step": (C.c_int, [P, P, I64, C.c_int, I64P, I64P]),
    "tr_rrt_book": (P, [P]),
    "tr_last_timings": (C.c_int, [P, DP]),
    "tr_enable_timing": (C.c_int, [P, C.c_int]),
    "tr_last_host_timings": (C.c_int, [P, DP]),
    "tr_last_nn_timings": (C.c_int, [P, DP]),
    "tr_rrt_pipe_stage": (C.c_int, [P, P, I64, P, P]),
    "tr_rrt_run": (C.c_int, [P, P, I64, I64, P, P, P, P, C.c_int, C.c_int, C.POINTER(C.c_int64),
                             C.POINTER(C.c_int64)]),
    "tr_comm_unique_id": (C.c_int, [P]),
    "tr_comm_init": (C.c_int, [P, C.c_int, C.c_int, P]),
    "tr_last_run_stats": (C.c_int, [P, DP, C.POINTER(C.c_int64)]),
    "tr_rrt_reserve": (C.c_int, [P, I64, I64]),
    "tr_rrt_pipe_expand": (C.c_int, [P, P, I64, P, P]),
    "tr_rrt_pipe_dedupe": (C.c_int, [P, P, P, I64]),
    "tr_rrt_pipe_commit": (C.c_int, [P, I64P, I64P]),
    "tr_rrt_pending": (C.c_int, [P]),
    "tr_findnearest_batch": (C.c_int, [P, P, I64, P, P, I64, P, I64, P, P]),
    "tr_rrt_findnearest": (C.c_int, [P, P, I64, P, P]),
    "tr_astar": (C.c_int, [P, I64, I64, I64, I64, C.c_int, P, I64, I64P, P]),
    "tr_astar_batch": (C.c_int, [P, P, I64, C.c_int, P, I64, P, P]),
    "tr_rng_set_state": (C.c_int, [P, P, C.c_int32, C.c_int32, C.c_double]),
    "tr_rng_get_state": (C.c_int, [P, P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), DP]),
    "tr_rng_gauss_dev": (C.c_int, [P, I64, P]),
    "tr_last_run_kernel_us": (C.c_int, [P, DP, I64P]),
    "tr_comm_init_host": (C.c_int, [P, C.c_int, C.c_int, P, P]),
    "tr_lineofsight": (C.c_int, [P, P, P]),
}

_lib = None


def lib():
    """Load libthetarrt.so (fails loudly: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("theta-rrt_amd: %s is missing; build it with "
                              "`python theta-rrt_amd/build.py` (hipcc, gfx950)" % LIB_PATH)
        # torch bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's).  Whichever loads
        # first serves the whole process, and torch cannot initialise on a runtime it did not
        # ship with; load torch's first so torch tensors and this library share one HIP runtime.
        # (THETARRT_NO_TORCH=1: a process without torch, e.g. under a sanitizer runtime)
        if not os.environ.get("THETARRT_NO_TORCH"):
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
    return _lib


class NativeError(RuntimeError):
    pass


def check(rc):
    if rc == TR_OK:
        return
    msg = lib().tr_last_error().decode(errors="replace")
    if rc == TR_E_STRAIGHT:
        raise TypeError(msg)              # rrt.py:275 -> :71 in the reference
    if rc == TR_E_INDEX:
        raise IndexError(msg)             # search.py:30 in the reference (non-square maps)
    if rc == TR_E_VALUE:
        raise ValueError(msg)             # search.py:262 in the reference (np.argmin of [])
    raise NativeError("libthetarrt error %d: %s" % (rc, msg))


def ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Book:
    """Host bookkeeping (no GPU): the reference's G / cameFrom as append-only arrays."""

    def __init__(self, handle=None, owner=None):
        self._own = handle is None
        if handle is None:
            h = C.c_void_p()
            check(lib().tr_book_create(C.byref(h)))
            handle = h
        self._h = handle
        self._owner = owner          # the Engine whose context owns the book (kept alive)

    @property
    def h(self):
        if self._owner is not None and not self._owner.h:
            raise NativeError("the engine that owns this book is closed")
        return self._h

    @h.setter
    def h(self, v):
        self._h = v

    def close(self):
        if self._own and self._h:
            lib().tr_book_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_straight_reject(self, on):
        check(lib().tr_book_set_straight_reject(self.h, 1 if on else 0))

    def reset(self, start_xyt):
        check(lib().tr_book_reset(self.h, ptr(np.ascontiguousarray(start_xyt, np.float64))))

    def ingest(self, samples, records, n_snap):
        samples = np.ascontiguousarray(samples, SAMPLE_DTYPE)
        records = np.ascontiguousarray(records, RECORD_DTYPE)
        n_new, sol = C.c_int64(), C.c_int64()
        check(lib().tr_book_ingest(self.h, ptr(samples), ptr(records), len(records), n_snap,
                                   C.byref(n_new), C.byref(sol)))
        return n_new.value, sol.value

    def reserve(self, nodes, edges):
        check(lib().tr_book_reserve(self.h, int(nodes), int(edges)))

    def replay(self, resolved):
        rs = np.ascontiguousarray(resolved, RESOLVED_DTYPE)
        n_new, sol = C.c_int64(), C.c_int64()
        check(lib().tr_book_replay(self.h, ptr(rs), len(rs), C.byref(n_new), C.byref(sol)))
        return n_new.value, sol.value

    def size(self):
        return lib().tr_book_size(self.h)

    def nodes(self, a=0, b=None):
        b = self.size() if b is None else b
        out = np.empty((b - a, 3), np.float64)
        check(lib().tr_book_nodes(self.h, a, b, ptr(out)))
        return out

    def export(self):
        n, m = self.size(), lib().tr_book_edges(self.h)
        parent = np.empty(n, np.int64)
        u6 = np.empty((n, 6), np.float64)
        e_off = np.empty(n + 1, np.int64)
        e_child = np.empty(m, np.int64)
        check(lib().tr_book_export(self.h, ptr(parent), ptr(u6), ptr(e_off), ptr(e_child)))
        return dict(nodes=self.nodes(), parent=parent, u=u6, e_off=e_off, e_child=e_child)


def gpu_visible():
    n = C.c_int(0)
    try:
        hip = C.CDLL("libamdhip64.so")
        return hip.hipGetDeviceCount(C.byref(n)) == 0 and n.value > 0
    except OSError:
        return False


class Engine:
    """One tr_ctx bound to one GPU (one per process / rank)."""

    def __init__(self, device=None):
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        h = C.c_void_p()
        check(lib().tr_create(device, C.byref(h)))
        self.h = h
        self.device = device
        self._grid = None
        self._params = None

    def close(self):
        if self.h:
            lib().tr_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- state
    def set_params(self, p: tr_params):
        key = bytes(p)
        if key != self._params:
            check(lib().tr_set_params(self.h, C.byref(p)))
            self._params = key

    def set_grid(self, free):
        g = np.ascontiguousarray(np.asarray(free).astype(np.uint8, copy=False))
        if g.ndim != 2:
            raise ValueError("occupancy grid must be 2-D [y][x]")
        if self._grid is not None and self._grid.shape == g.shape and np.array_equal(self._grid, g):
            return
        check(lib().tr_set_grid(self.h, ptr(g), g.shape[0], g.shape[1]))
        self._grid = g.copy()
        self.grid_serial = getattr(self, "grid_serial", 0) + 1     # uploads so far (config.engine's key)

    def set_option(self, name, value):
        """Engine option (include/thetarrt.h tr_set_option), e.g. ("gate", 0)."""
        check(lib().tr_set_option(self.h, name.encode(), int(value)))

    def get_option(self, name):
        v = C.c_int64()
        check(lib().tr_get_option(self.h, name.encode(), C.byref(v)))
        return v.value

    def set_stream(self, stream_handle):
        check(lib().tr_set_stream(self.h, C.c_void_p(stream_handle)))

    def sync(self):
        check(lib().tr_sync(self.h))

    # -- tree
    def tree_reset(self, cap=1024):
        check(lib().tr_tree_reset(self.h, cap))

    def tree_append(self, xyt):
        xyt = np.ascontiguousarray(xyt, np.float64).reshape(-1, 3)
        check(lib().tr_tree_append(self.h, ptr(xyt), len(xyt)))

    def tree_size(self):
        return lib().tr_tree_size(self.h)

    # -- batches
    def nn(self, q_xy, d2=False):
        """rrt.py:155-158 for a batch of integer queries: node indices (and, d2=True, the winners'
        squared distances)."""
        q = np.ascontiguousarray(q_xy, np.int32).reshape(-1, 2)
        out = np.empty(len(q), np.int64)
        dd = np.empty(len(q), np.float64) if d2 else None
        check(lib().tr_nn_batch(self.h, ptr(q), len(q), ptr(out), ptr(dd)))
        return (out, dd) if d2 else out

    def los(self, seg4):
        s = np.ascontiguousarray(seg4, np.float64).reshape(-1, 4)
        out = np.empty(len(s), np.uint8)
        check(lib().tr_los_batch(self.h, ptr(s), len(s), ptr(out)))
        return out.astype(bool)

    def findnearest(self, xyt, e_par, e_child, goals3):
        """rrt.py:117-128 for every goal: (child node index or -1, distance) arrays."""
        xyt = np.ascontiguousarray(xyt, np.float64).reshape(-1, 3)
        ep = np.ascontiguousarray(e_par, np.int64).ravel()
        ec = np.ascontiguousarray(e_child, np.int64).ravel()
        if ep.shape != ec.shape:
            raise ValueError("e_par and e_child differ in length")
        g = np.ascontiguousarray(goals3, np.float64).reshape(-1, 3)
        node = np.empty(len(g), np.int64)
        dist = np.empty(len(g), np.float64)
        check(lib().tr_findnearest_batch(self.h, ptr(xyt), len(xyt), ptr(ep), ptr(ec), len(ec),
                                         ptr(g), len(g), ptr(node), ptr(dist)))
        return node, dist

    def rrt_findnearest(self, goals3):
        """findnearest over the session's tree (every batch committed)."""
        g = np.ascontiguousarray(goals3, np.float64).reshape(-1, 3)
        node = np.empty(len(g), np.int64)
        dist = np.empty(len(g), np.float64)
        check(lib().tr_rrt_findnearest(self.h, ptr(g), len(g), ptr(node), ptr(dist)))
        return node, dist

    def lineofsight(self, n1, n2):
        """search.py:35-41 for one segment, on the host (tr_lineofsight)."""
        seg = (C.c_double * 4)(float(n1[0]), float(n1[1]), float(n2[0]), float(n2[1]))
        out = C.c_uint8()
        check(lib().tr_lineofsight(self.h, seg, C.byref(out)))
        return bool(out.value)

    def astar(self, start, goal, thetastar=True):
        """search.py:221-307 for one query, on the host (tr_astar).  Returns (path int64 [n][2] or
        None, stats)."""
        st = np.zeros(4, np.int64)
        n = C.c_int64(0)
        cap = 1 << 16
        while True:
            out = np.empty((cap, 2), np.int64)
            rc = lib().tr_astar(self.h, int(start[0]), int(start[1]), int(goal[0]), int(goal[1]),
                                1 if thetastar else 0, ptr(out), cap, C.byref(n), ptr(st))
            if rc == TR_E_ARG and n.value > cap:
                cap = n.value
                continue
            check(rc)
            break
        stats = dict(expanded=int(st[0]), los_segments=int(st[2]), status=int(st[3]))
        return (out[:n.value].copy() if st[3] == 0 else None), stats

    def astar_batch(self, queries, thetastar=True, cap=4096):
        """search.py:221-307 for many (sx, sy, gx, gy) queries at once, each search resident on the
        GPU (tr_astar_batch).  Returns (list of int64 [n][2] paths or None, stats int64 [n][4] =
        expanded, queue entries consumed, pushes past the queue's buckets, status)."""
        q = np.ascontiguousarray(queries, np.int32).reshape(-1, 4)
        n = len(q)
        paths = np.empty((n, cap, 2), np.int64)
        plen = np.zeros(n, np.int64)
        stats = np.zeros((n, 4), np.int64)
        check(lib().tr_astar_batch(self.h, ptr(q), n, 1 if thetastar else 0, ptr(paths), cap,
                                   ptr(plen), ptr(stats)))
        out = [paths[i, :plen[i]].copy() if stats[i, 3] == 0 else None for i in range(n)]
        return out, stats

    def steer(self, in6):
        a = np.ascontiguousarray(in6, np.float64).reshape(-1, 6)
        out = np.empty((len(a), 9), np.float64)
        check(lib().tr_steer_batch(self.h, ptr(a), len(a), ptr(out)))
        return out

    def drive(self, in9):
        a = np.ascontiguousarray(in9, np.float64).reshape(-1, 9)
        out = np.empty((len(a), 3), np.float64)
        ok = np.empty(len(a), np.int32)
        check(lib().tr_drive_batch(self.h, ptr(a), len(a), ptr(out), ptr(ok)))
        return out, ok.astype(bool)

    def body_clear(self, xyt, mult):
        a = np.ascontiguousarray(xyt, np.float64).reshape(-1, 3)
        out = np.empty(len(a), np.uint8)
        check(lib().tr_body_clear_batch(self.h, ptr(a), len(a), float(mult), ptr(out)))
        return out.astype(bool)

    def arc_clear(self, in10):
        a = np.ascontiguousarray(in10, np.float64).reshape(-1, 10)
        out = np.empty(len(a), np.uint8)
        check(lib().tr_arc_batch(self.h, ptr(a), len(a), ptr(out)))
        return out.astype(bool)

    def expand_dev(self, d_gauss, B, goal3, d_samples, d_records, noalloc=False):
        """rrt.py:144-176 for B samples against the device tree (tr_expand_dev); noalloc=True: the
        entry point that uses the static scratch and allocates nothing."""
        fn = lib().tr_expand_dev_noalloc if noalloc else lib().tr_expand_dev
        check(fn(self.h, C.c_void_p(d_gauss), int(B), ptr(np.ascontiguousarray(goal3, np.float64)),
                 C.c_void_p(d_samples), C.c_void_p(d_records)))

    def _list(self, fn, *args):
        cap = 4096
        while True:
            out = np.empty((cap, 2), np.int64)
            n = C.c_int64()
            check(fn(self.h, *args, ptr(out), cap, C.byref(n)))
            if n.value <= cap:
                return out[: n.value]
            cap = int(n.value)

    def bresenham(self, seg4):
        s = np.ascontiguousarray(seg4, np.float64)
        return self._list(lib().tr_bresenham, ptr(s))

    def circle(self, cx, cy, r):
        return self._list(lib().tr_circle, C.c_double(cx), C.c_double(cy), C.c_double(r))

    def arc_pixels(self, in10):
        a = np.ascontiguousarray(in10, np.float64)
        return self._list(lib().tr_arc_pixels, ptr(a))

    # -- RRT session
    def rrt_begin(self, start3, goal3):
        check(lib().tr_rrt_begin(self.h, ptr(np.asarray(start3, np.float64)),
                                 ptr(np.asarray(goal3, np.float64))))

    def rrt_step(self, gauss=None, B=None, dev_ptr=None):
        n, sol = C.c_int64(), C.c_int64()
        if dev_ptr is not None:
            check(lib().tr_rrt_step(self.h, C.c_void_p(dev_ptr), B, 1, C.byref(n), C.byref(sol)))
        else:
            g = np.ascontiguousarray(gauss, np.float64)
            check(lib().tr_rrt_step(self.h, ptr(g), len(g) // 3, 0, C.byref(n), C.byref(sol)))
        return n.value, sol.value

    # -- pipelined session (include/thetarrt.h): expand -> [all-gather] -> dedupe -> commit(b-1)
    def rrt_reserve(self, nodes, batch):
        check(lib().tr_rrt_reserve(self.h, int(nodes), int(batch)))

    def pipe_expand(self, d_gauss, B, d_samples, d_records):
        check(lib().tr_rrt_pipe_expand(self.h, C.c_void_p(d_gauss), B, C.c_void_p(d_samples),
                                       C.c_void_p(d_records)))

    def pipe_stage(self, d_gauss, B, d_samples, d_records):
        """Look-ahead expansion of a future batch on the side stream (include/thetarrt.h)."""
        check(lib().tr_rrt_pipe_stage(self.h, C.c_void_p(d_gauss), B, C.c_void_p(d_samples),
                                      C.c_void_p(d_records)))

    # -- the np.random gaussian stream on the device (rand_conf's draws, rrt.py:58,66)
    def rng_set_state(self, state):
        """Seed the device stream from a numpy RandomState state tuple (np.random.get_state())."""
        name, key, pos, has, gauss = state[:5]
        if name != "MT19937":
            raise ValueError("only MT19937 states")
        k = np.ascontiguousarray(key, np.uint32)
        if k.shape != (624,):
            raise ValueError("MT19937 key must have 624 words")
        check(lib().tr_rng_set_state(self.h, ptr(k), int(pos), int(has), float(gauss)))

    def rng_get_state(self):
        """The device stream's position as numpy's state tuple (np.random.set_state accepts it)."""
        k = np.empty(624, np.uint32)
        pos, has, g = C.c_int32(), C.c_int32(), C.c_double()
        check(lib().tr_rng_get_state(self.h, ptr(k), C.byref(pos), C.byref(has), C.byref(g)))
        return ("MT19937", k, pos.value, has.value, g.value)

    def rng_gauss_dev(self, n, d_out):
        """RandomState.standard_normal(n) into device memory (async on the engine stream)."""
        check(lib().tr_rng_gauss_dev(self.h, int(n), C.c_void_p(d_out)))

    def run(self, d_gauss, B, rows, d_samples, d_records, lag=4, stage=True, d_samples_all=0,
            d_records_all=0):
        """Native pipelined loop over `rows` batches (include/thetarrt.h tr_rrt_run); `stage` = the
        look-ahead depth (True = 1), d_samples / d_records hold max(2, stage + 1) sets of B.
        d_gauss = None: the engine draws the gaussians from its stream (rng_set_state)."""
        nn, sol = C.c_int64(), C.c_int64()
        check(lib().tr_rrt_run(self.h, C.c_void_p(d_gauss), B, rows, C.c_void_p(d_samples),
                               C.c_void_p(d_records), C.c_void_p(d_samples_all or None),
                               C.c_void_p(d_records_all or None), int(lag), int(stage),
                               C.byref(nn), C.byref(sol)))
        return nn.value, sol.value

    @staticmethod
    def comm_unique_id():
        buf = (C.c_uint8 * 128)()
        check(lib().tr_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, rank, world, uid):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        check(lib().tr_comm_init(self.h, int(rank), int(world), buf))

    def comm_init_host(self, rank, world, gather):
        """Sharded session with the exchange through the host: gather(send: bytes) -> bytes of
        every rank in rank order (e.g. a gloo all_gather).  tr_comm_init_host."""
        def cb(user, send, recv, nbytes):
            try:
                out = gather(C.string_at(send, nbytes))
                if len(out) != world * nbytes:
                    return 2
                C.memmove(recv, out, len(out))
                return 0
            except Exception:                                # noqa: BLE001 (status to the engine)
                import traceback
                traceback.print_exc()
                return 1
        self._gather_cb = HOST_GATHER_FN(cb)                 # kept alive with the engine
        check(lib().tr_comm_init_host(self.h, int(rank), int(world),
                                      C.cast(self._gather_cb, C.c_void_p), None))

    def last_run_stats(self):
        a = (C.c_double * 11)()
        n = C.c_int64()
        check(lib().tr_last_run_stats(self.h, a, C.byref(n)))
        return list(a), n.value

    def last_run_kernel_us(self):
        """Mean HIP-event us over the last run's sampled batches: dict per kernel + sample counts."""
        a = (C.c_double * 5)()
        n = (C.c_int64 * 2)()
        check(lib().tr_last_run_kernel_us(self.h, a, n))
        keys = ("k_nn_pass1", "k_nn_resolve", "k_nn_delta", "k_expand_arc", "dedupe")
        return dict(zip(keys, list(a))), (n[0], n[1])

    def pipe_dedupe(self, d_samples, d_records, n):
        check(lib().tr_rrt_pipe_dedupe(self.h, C.c_void_p(d_samples), C.c_void_p(d_records), n))

    def pipe_commit(self):
        nn, sol = C.c_int64(), C.c_int64()
        check(lib().tr_rrt_pipe_commit(self.h, C.byref(nn), C.byref(sol)))
        return nn.value, sol.value

    def pending(self):
        return lib().tr_rrt_pending(self.h)

    def book(self):
        return Book(lib().tr_rrt_book(self.h), owner=self)

    def enable_timing(self, level=1):
        """1: HIP-event time of the nearest-node kernels; 2: every phase (adds GPU gaps)."""
        check(lib().tr_enable_timing(self.h, int(level)))

    def last_host_timings(self):
        a = (C.c_double * 3)()
        check(lib().tr_last_host_timings(self.h, a))
        return list(a)

    def last_nn_timings(self):
        """NN us of the last committed batch: staged sweep (side stream), NN on the batch's path."""
        a = (C.c_double * 3)()
        check(lib().tr_last_nn_timings(self.h, a))
        return list(a)

    def last_timings(self):
        """GPU us of the last committed batch: nn, steer/drive, arc, bookkeeping, sum."""
        a = (C.c_double * 5)()
        check(lib().tr_last_timings(self.h, a))
        return list(a)


_engine = None


def engine():
    """Process-wide engine on LOCAL_RANK's GPU (created lazily)."""
    global _engine
    if _engine is None:
        _engine = Engine()
    return _engine
