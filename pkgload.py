"""Import helper: the package directory is `theta-rrt_amd/` (not a Python identifier), so it is
registered as the module `theta_rrt_amd`.  After `pkgload.load()`, `import theta_rrt_amd.rrt` works."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "theta-rrt_amd")
NAME = "theta_rrt_amd"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(NAME, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
