"""Build compile-time variants of libthetarrt.so for A/B runs on the GPU box (not shipped).

    python tools/build_variants.py NAME -DMACRO=VALUE ...  -> theta-rrt_amd/variants/libthetarrt_NAME.so

A GPU script copies a variant over theta-rrt_amd/libthetarrt.so before each run.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "theta-rrt_amd"))
import build  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
out = os.path.join(ROOT, "theta-rrt_amd", "variants")
os.makedirs(out, exist_ok=True)
build.FLAGS = build.FLAGS + defs
build.LIB = os.path.join(out, "libthetarrt_%s.so" % name)
print(build.build(force=True))
