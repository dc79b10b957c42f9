"""theta-rrt on MI355X: batched RRT expansion + Theta* line of sight behind the reference's API.

Modules mirror eshira/theta-rrt: `search` (grid primitives, Bresenham, circle/arc, A*/Theta*) and
`rrt` (bicycle kinematics, sampler, RRT).  The per-iteration hot loop runs in hand-written HIP
kernels (libthetarrt.so, C-ABI in include/thetarrt.h) reached through ctypes.
"""
from . import config  # noqa: F401

__all__ = ["config", "search", "rrt", "engine"]
