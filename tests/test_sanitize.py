"""Sanitizer builds of the host library: the host code of libthetarrt (bookkeeping,
commit ring, replay worker, A*, C-ABI glue) instrumented, the device code unchanged
(theta-rrt_amd/build.py variants; every -fsanitize= follows -Xarch_host).

* ASan + UBSan (CPU): the host-book, API and sharded-bookkeeping tests run against the instrumented
  library with the clang runtime preloaded; any report fails the run (halt_on_error).
* TSan (GPU): pipelined sessions (native loop with its replay worker thread, pipe_* calls with
  interleaved commits) under ThreadSanitizer, from the prebuilt libthetarrt_tsan.so.
"""
import importlib.util
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _build_mod():
    spec = importlib.util.spec_from_file_location("_tr_build", os.path.join(ROOT, "theta-rrt_amd", "build.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _run(variant, argv, timeout):
    b = _build_mod()
    lib = b.lib_path(variant)
    rt = b.sanitizer_runtime(variant)
    if rt is None:
        pytest.skip("no clang %s runtime in this ROCm" % variant)
    env = dict(os.environ, LD_PRELOAD=rt, THETARRT_LIB=lib,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1:suppressions=" +
               os.path.join(ROOT, "tests", "native", "tsan.supp"))
    probe = ("import pkgload; pkgload.load(); from theta_rrt_amd import _native; _native.lib(); "
             "m = open('/proc/self/maps').read(); print(%r in m, 'libclang_rt' in m)" % os.path.basename(lib))
    r = subprocess.run([sys.executable, "-c", probe], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.stdout.split() == ["True", "True"], (r.stdout, r.stderr[-2000:])
    r = subprocess.run(argv, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    for bad in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer"):
        assert bad not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    return out


def test_host_library_asan_ubsan():
    _build_mod().build(variant="asan")          # ~25 s when stale; __graft_entry__.build() prebuilds
    _run("asan", [sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                  "tests/test_host.py", "tests/test_api_host.py", "tests/test_sharded.py"], 600)


@pytest.mark.gpu
def test_replay_worker_tsan():
    b = _build_mod()
    assert os.path.exists(b.lib_path("tsan")), "libthetarrt_tsan.so missing: run __graft_entry__.build()"
    # The HIP runtime itself must come up under the TSan runtime (its address-space layout): on
    # boxes where a bare hipGetDeviceCount fails there, nothing of this library has run yet.
    rt = b.sanitizer_runtime("tsan")
    if rt is None:
        pytest.skip("no clang tsan runtime in this ROCm")
    probe = ("import ctypes as C; h = C.CDLL('libamdhip64.so'); n = C.c_int(); "
             "print(h.hipGetDeviceCount(C.byref(n)), n.value)")
    r = subprocess.run([sys.executable, "-c", probe], env=dict(os.environ, LD_PRELOAD=rt),
                       capture_output=True, text=True, timeout=120)
    if r.stdout.split()[:1] != ["0"]:
        pytest.skip("the HIP runtime does not initialise under the TSan runtime on this box "
                    "(hipGetDeviceCount -> %s)" % (r.stdout.strip() or r.stderr.strip()[-200:]))
    os.environ["THETARRT_NO_TORCH"] = "1"
    try:
        out = _run("tsan", [sys.executable, "tests/native/tsan_session.py"], 240)
    finally:
        os.environ.pop("THETARRT_NO_TORCH")
    assert "pipe:" in out
