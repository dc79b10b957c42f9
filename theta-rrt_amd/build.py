"""Build libthetarrt.so (gfx950) in-tree with hipcc.

`python theta-rrt_amd/build.py [--force] [--variant asan|tsan|phases|ddphases]`

Variants instrument the HOST code only (every -fsanitize= follows -Xarch_host; the device code is
the product build's): `asan` = AddressSanitizer + UndefinedBehaviorSanitizer, `tsan` =
ThreadSanitizer (the replay worker thread and the commit ring).  They run with the clang runtime
preloaded (sanitizer_runtime()) and THETARRT_LIB pointing at them (tests/test_sanitize.py).
"""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libthetarrt.so")
SOURCES = ["kernels.hip", "nn.hip", "nn_grid.hip", "dedupe.hip", "findnearest.hip", "astar.hip", "astar_dev.hip", "rng.hip", "capi.hip"]
HEADERS = ["geom.hpp", "thetarrt_internal.hpp", "legacy_gauss.hpp", "legacy_log.hpp", "lanegroup.hpp", "mt_jump.hpp", "diaglog.hpp", os.path.join("..", "..", "include", "thetarrt.h")]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-fno-fast-math", "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops", "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]
_H = "-Xarch_host"
VARIANTS = {   # (compile flags, link flags)
    "asan": ([_H, "-fsanitize=address", _H, "-fsanitize=undefined", _H, "-fno-sanitize-recover=undefined",
              _H, "-fno-omit-frame-pointer", _H, "-g"],
             ["-fno-gpu-sanitize", "-fsanitize=address,undefined", "-shared-libasan"]),
    "tsan": ([_H, "-fsanitize=thread", _H, "-fno-omit-frame-pointer", _H, "-g"],
             ["-fno-gpu-sanitize", "-fsanitize=thread"]),
    # diagnosis builds (device code differs from the product's): wall-clock stamps between the
    # phases of k_expand_arc / k_dd, printed every 40 launches
    "phases": (["-DTR_DIAG_PHASES"], []),
    "ddphases": (["-DTR_DIAG_DD"], []),
    "nobins": (["-DTR_DIAG_NOBINS"], []),
    "nohostdelta": (["-DTR_DIAG_NOHOSTDELTA"], []),   # k_dd without its writes to the pinned commit slot
    "rs16": (["-DTR_RS=16"], []),
    "c256": (["-DTR_P1_CAP=256"], []), "c384": (["-DTR_P1_CAP=384"], []),
}


def lib_path(variant=None):
    return LIB if not variant else os.path.join(HERE, "libthetarrt_%s.so" % variant)


def sanitizer_runtime(variant):
    """The clang runtime to LD_PRELOAD for a sanitizer variant (None if absent)."""
    name = {"asan": "libclang_rt.asan-x86_64.so", "tsan": "libclang_rt.tsan-x86_64.so"}[variant]
    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/" + name))
    return hits[-1] if hits else None


def stale(variant=None):
    out = lib_path(variant)
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False, variant=None):
    out = lib_path(variant)
    if not force and not stale(variant):
        return out
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cflags, lflags = [], []
    for v in (variant.split("+") if variant else []):      # "phases+rs8": the flags of both
        cflags += VARIANTS[v][0]
        lflags += VARIANTS[v][1]
    tag = "." + variant if variant else ""
    def compile_one(src):
        obj = os.path.join(CSRC, src.replace(".hip", tag + ".o"))
        cmd = [hipcc, *FLAGS, *cflags, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        # hipcc's host pass does not know the device feature and says so once per function
        r = subprocess.run(cmd, stderr=subprocess.PIPE, text=True)
        sys.stderr.write("".join(l for l in r.stderr.splitlines(True) if "packed-fp32-ops" not in l))
        if r.returncode:
            raise subprocess.CalledProcessError(r.returncode, cmd)
        return obj
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 1, 8)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    cmd = [hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", *lflags, *objs, "-o", out + ".tmp"]
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    for o in objs:
        os.remove(o)
    return out


if __name__ == "__main__":
    v = sys.argv[sys.argv.index("--variant") + 1] if "--variant" in sys.argv else None
    print(build(force="--force" in sys.argv, verbose=True, variant=v))
