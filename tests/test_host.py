"""CPU-only tests: the C-ABI library loads and exports every declared symbol, the host bookkeeping
(tr_book_*) follows the reference's dict semantics, and host-side invariants the kernels rely on."""
import math
import os
import re

import numpy as np
import pytest

from conftest import ROOT
import pkgload

pkgload.load()
from theta_rrt_amd import _native  # noqa: E402

HEADER = os.path.join(ROOT, "include", "thetarrt.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\*]+\s*\*?\s*(tr_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    lib = _native.lib()
    names = declared_symbols()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), n
    assert set(_native._SIGS) <= set(names) | {"tr_last_error", "tr_version"}
    assert lib.tr_version() == 3


def _rec(x, y, th, near, status=_native.ST_OK, flags=0):
    r = np.zeros(1, _native.RECORD_DTYPE)
    r["x"], r["y"], r["th"], r["near"], r["status"], r["flags"] = x, y, th, near, status, flags
    r["steer"], r["iccx"], r["iccy"], r["rad"], r["dist"] = 10.0, 1.0, 2.0, 3.0, 4.0
    return r


def _samp(x, y, th):
    s = np.zeros(1, _native.SAMPLE_DTYPE)
    s["x"], s["y"], s["th"] = x, y, th
    return s


def test_book_semantics_match_reference_bookkeeping():
    """rrt.py:179-188: vertex dedupe by exact value (-0.0 == 0.0), edge always appended, cameFrom
    overwritten for re-reached nodes, not set when qnew == qnear; rrt.py:151 membership skip."""
    b = _native.Book()
    b.reset([5.0, 5.0, 0.0])
    recs = np.concatenate([
        _rec(10.0, 5.0, 1.0, 0),                       # new node 1
        _rec(10.0, 5.0, 1.0, 0),                       # duplicate of 1: edge only
        _rec(5.0, 5.0, -0.0, 0),                       # == start (qnew == qnear): edge, no cameFrom
        _rec(12.0, 7.0, 2.0, 1),                       # new node 2 from 1
        _rec(99.0, 99.0, 9.0, 0, _native.ST_COLLISION),  # rejected
        _rec(10.0, 5.0, 1.0, 2),                       # re-reach 1 from 2: cameFrom[1] overwritten
    ])
    samps = np.concatenate([_samp(1, 1, 0.5)] * len(recs))
    n_new, sol = b.ingest(samps, recs, n_snap=1)
    assert (n_new, sol) == (2, -1)
    ex = b.export()
    assert ex["nodes"].tolist() == [[5, 5, 0], [10, 5, 1], [12, 7, 2]]
    assert ex["parent"].tolist() == [-1, 2, 1]
    assert ex["e_off"].tolist() == [0, 3, 4, 5]
    assert ex["e_child"].tolist() == [1, 1, 0, 2, 1]
    # membership: a sample equal to a snapshot node is skipped before anything else
    n_new, sol = b.ingest(_samp(12, 7, 2.0), _rec(50.0, 50.0, 0.0, 0, _native.ST_STRAIGHT), n_snap=3)
    assert (n_new, sol) == (0, -1)
    with pytest.raises(TypeError):
        b.ingest(_samp(13, 7, 2.0), _rec(50.0, 50.0, 0.0, 0, _native.ST_STRAIGHT), n_snap=3)
    # goal stops the batch (rrt.py:198-201)
    recs = np.concatenate([_rec(20.0, 20.0, 0.0, 0), _rec(21.0, 21.0, 0.0, 0, flags=_native.FL_GOAL),
                           _rec(22.0, 22.0, 0.0, 0)])
    n_new, sol = b.ingest(np.concatenate([_samp(2, 2, 0.1)] * 3), recs, n_snap=b.size())
    assert (n_new, sol) == (2, 4)


def test_midpoint_circle_closed_form():
    """The arc kernel enumerates getCircle's octant in closed form (geom.hpp circle_x)."""
    def cx(r, k):
        T = r * r - k * k
        if T <= 0:
            return 0
        x = int((math.sqrt(4.0 * T + 1.0) - 1.0) * 0.5)
        while x * (x + 1) < T:
            x += 1
        while x > 0 and (x - 1) * x >= T:
            x -= 1
        return x
    for r in list(range(0, 700)) + [20000, 123457]:
        x, y, d, pts = r, 0, 1 - r, []
        while x > y:
            pts.append(x)
            y += 1
            if d < 0:
                d += 2 * y + 1
            else:
                x -= 1
                d += 2 * (y - x) + 1
        assert [cx(r, k) for k in range(len(pts))] == pts
        assert cx(r, len(pts)) <= len(pts)


def test_right_angle_rotation_constants_are_host_libm_values():
    """geom.hpp's zquat short-cuts (rotations by +-90 / +-180 deg) must be exactly the values the
    reference's scipy/numpy stack computes for sin / cos of deg * (pi/180) / 2."""
    src = open(os.path.join(ROOT, "theta-rrt_amd", "csrc", "geom.hpp")).read()
    consts = dict(re.findall(r"(kS45|kC45|kC90) = (0x[0-9a-fp.+-]+)", src))
    k_deg = 0.017453292519943295
    assert float.fromhex(consts["kS45"]) == math.sin(90 * k_deg / 2)
    assert float.fromhex(consts["kC45"]) == math.cos(90 * k_deg / 2)
    assert float.fromhex(consts["kC90"]) == math.cos(180 * k_deg / 2)
    assert 1.0 == math.sin(180 * k_deg / 2)
    assert np.sin(np.float64(90 * k_deg / 2)) == math.sin(90 * k_deg / 2)


def test_bresenham_closed_form():
    """los_wave (kernels.hip) gives pixel k of a Bresenham line the y-step count
    floor((2 dy k + dx - 1) / (2 dx)) instead of running the err recurrence of search.py:71-92;
    exhaustive check of that identity over every octant-normalised (dx, dy) with dx < 300."""
    for dx in range(1, 300):
        for dy in range(0, dx + 1):
            err, n = 2 * dy - dx, 0
            for k in range(dx + 1):
                assert (2 * dy * k + dx - 1) // (2 * dx) == n, (dx, dy, k)
                if err > 0:
                    n += 1
                    err -= 2 * dx
                err += 2 * dy


def test_arc_keep_cross_products_equal_the_angle_test(tmp_path):
    """geom.hpp's arc_keeps decides getArc's per-pixel keep test (search.py:161-181) from cross
    products and takes the reference's angle comparisons only inside a narrow band around the
    begin / land rays: a host build of both over 9.6M (arc, pixel) pairs, including integral centres
    with pixels exactly on the rays, must agree everywhere."""
    import subprocess
    exe = str(tmp_path / "arc_keep_check")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950",
                    "-I" + os.path.join(ROOT, "theta-rrt_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "arc_keep_check.hip"), "-o", exe],
                   check=True, stderr=subprocess.DEVNULL)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert "mismatches 0" in r.stdout
