"""The reference's parameter block and map input (main.py:14-42).

Parameters live on `builtins` under the reference's names so existing callers keep working; the
engine reads them at every call.  `ensure_defaults()` sets only the names a caller has not set.
"""
import builtins

import numpy as np

from . import _native

DEFAULTS = dict(THETASTAR=True, bikelength=5, FORWARDONLY=True, LEFTCONSTRAINT=-65,
                RIGHTCONSTRAINT=65, frontclearance=2, K=300, showtree=False, maxdrivedist=30,
                tol_xy=10, tol_ang=45, weightxy=.6, xystdv=0.4, anglestdv=100)


def ensure_defaults():
    for k, v in DEFAULTS.items():
        if not hasattr(builtins, k):
            setattr(builtins, k, v)


def get(name):
    ensure_defaults()
    return getattr(builtins, name)


def native_params():
    ensure_defaults()
    b = builtins
    return _native.tr_params(float(b.bikelength), float(b.LEFTCONSTRAINT), float(b.RIGHTCONSTRAINT),
                             float(b.frontclearance), float(b.maxdrivedist), float(b.weightxy),
                             float(b.xystdv), float(b.anglestdv), float(b.tol_xy), float(b.tol_ang),
                             1 if b.FORWARDONLY else 0,
                             1 if getattr(b, "rrt_straight", "raise") == "reject" else 0)


def load_map(path):
    """main.py:37-42: PNG -> convert('1') -> bool array on builtins.imarray (True = free)."""
    from PIL import Image
    builtins.imarray = np.array(Image.open(path).convert('1'))
    return builtins.imarray


def imarray():
    a = getattr(builtins, "imarray", None)
    if a is None:
        raise NameError("name 'imarray' is not defined (set builtins.imarray, main.py:42)")
    return a


# (identity of the uploaded map, version), the version counter, the uploaded array itself (the
# reference keeps it alive, so no later array can take its id() and buffer address and pass for it)
# and the engine's upload count after that upload (a set_grid made on the engine directly since
# then means the engine no longer holds this map)
_grid_key = [None, 0, None, -1]


def grid_changed():
    """Mark builtins.imarray as modified in place (getCircle(draw=True) does; so must any caller
    that writes into the array): the next engine() call uploads it again."""
    _grid_key[1] += 1


def engine():
    """The process engine with the current builtins map and parameters uploaded.  The map is
    uploaded when builtins.imarray is a different array (object, buffer, shape) or has been marked
    changed: per-call cost is a key comparison, not a copy of the map."""
    e = _native.engine()
    e.set_params(native_params())
    a = imarray()
    key = (id(a), a.__array_interface__["data"][0], a.shape, a.strides, _grid_key[1], id(e))
    if key != _grid_key[0] or getattr(e, "grid_serial", 0) != _grid_key[3]:
        e.set_grid(a)
        _grid_key[0] = key
        _grid_key[2] = a
        _grid_key[3] = getattr(e, "grid_serial", 0)
    return e
