"""Grid primitives, line of sight, circle/arc rasters and A*/lazy Theta* (reference: search.py).

Same names, arguments and return shapes as eshira/theta-rrt search.py.  The raster and ray
functions run on the GPU through libthetarrt.so; `valid`/`freespace`/`L2norm` are one-line scalar
helpers kept in Python.  The map is `builtins.imarray` (bool [y][x], True = free), as in the
reference (main.py:42).
"""
import builtins
import itertools
import math

import numpy as np

from . import _native, config


def heuristic(node, goal):
    """search.py:9-11."""
    return L2norm(node, goal)


def L2norm(node0, node1):
    """search.py:13-15."""
    return math.sqrt(pow((node1[0] - node0[0]), 2) + pow((node1[1] - node0[1]), 2))


def valid(node):
    """search.py:17-24 (x is bounded by shape[0], y by shape[1], as in the reference)."""
    a = config.imarray()
    x, y = int(node[0]), int(node[1])
    return 0 <= x < a.shape[0] and 0 <= y < a.shape[1]


def freespace(node):
    """search.py:26-33."""
    if not valid(node):
        return False
    return bool(config.imarray()[int(node[1])][int(node[0])])


def lineofsight(node1, node2):
    """search.py:35-41 — one segment, on the host (tr_lineofsight: a single ray costs less than a
    GPU round trip).  Batches go to the GPU: lineofsight_batch."""
    return config.engine().lineofsight(node1, node2)


def lineofsight_batch(segments):
    """Batched lineofsight for (n, 4) endpoints (x0, y0, x1, y1) -> bool[n] (Theta* LOS batches)."""
    return config.engine().los(np.asarray(segments, np.float64).reshape(-1, 4))


def bresenham(node1, node2):
    """search.py:43-56 — pixel list in the reference's order (endpoints truncated by int())."""
    x0, y0, x1, y1 = int(node1[0]), int(node1[1]), int(node2[0]), int(node2[1])
    if abs(y1 - y0) < abs(x1 - x0):
        return plotLineLow(x1, y1, x0, y0) if x0 > x1 else plotLineLow(x0, y0, x1, y1)
    return plotLineHigh(x1, y1, x0, y0) if y0 > y1 else plotLineHigh(x0, y0, x1, y1)


def plotLineLow(x0, y0, x1, y1):
    """search.py:58-75."""
    pixels = []
    dx, dy, sy = x1 - x0, y1 - y0, 1
    if dy < 0:
        sy, dy = -1, -dy
    D, y = 2 * dy - dx, y0
    for x in range(x0, x1 + 1):
        pixels.append((x, y))
        if D > 0:
            y, D = y + sy, D - 2 * dx
        D = D + 2 * dy
    return pixels


def plotLineHigh(x0, y0, x1, y1):
    """search.py:77-94."""
    return [(x, y) for (y, x) in plotLineLow(y0, x0, y1, x1)]


def getCirclePoints(xc, yc, p, q):
    """search.py:96-105."""
    out = []
    for v1 in (-p, p, -q, q):
        for v2 in (-p, p, -q, q):
            if abs(v1) != abs(v2) and valid((xc + v1, yc + v2)):
                out.append((xc + v1, yc + v2))
    return out


def getCircle(center, r, draw=False):
    """search.py:107-142 — midpoint circle (+ diagonal patch) on the GPU.  draw=True blanks the
    pixels in builtins.imarray like the reference."""
    pix = [tuple(p) for p in config.engine().circle(float(center[0]), float(center[1]), float(r)).tolist()]
    if draw:
        for x, y in pix:
            builtins.imarray[y, x] = 0
        config.grid_changed()
    return pix


def getArc(begin, land, u):
    """search.py:144-182 — circle pixels inside the begin->land window (Bresenham if straight)."""
    if u[1] is None:
        return bresenham(begin, land)
    row = np.array([begin[0], begin[1], land[0], land[1], u[0], u[1][0], u[1][1], u[2], u[3], 0.0])
    return [tuple(p) for p in config.engine().arc_pixels(row).tolist()]


def getneighbors(node):
    """search.py:184-194."""
    out = []
    for d in itertools.product([-1, 0, 1], repeat=2):
        if d != (0, 0):
            c = (int(node[0] - d[0]), int(node[1] - d[1]))
            if valid(c) and freespace(c):
                out.append(c)
    return out


def reconstruct(node, pathmap):
    """search.py:196-204."""
    path = [node]
    while path[-1] in pathmap:
        path.append(pathmap[path[-1]])
    return path[::-1]


def astar(start, goal):
    """search.py:221-307: 8-connected A* with lazy Theta* (builtins.THETASTAR).

    Returns the path (list of (x, y)) or False and prints like the reference.  One search runs in
    the engine on the host (tr_astar: the reference's queue order); astar_many runs batches of
    searches resident on the GPU."""
    path, st = config.engine().astar(start, goal, bool(config.get("THETASTAR")))
    if st["status"] == 1:
        print("Start or goal is not valid. Error.")
        return False
    if st["status"] == 2:
        print("Start or goal is inside an obstacle. Error.")
        return False
    if path is None:
        return False
    print("Expanded nodes:", st["expanded"])
    return [(int(x), int(y)) for x, y in path]


def astar_many(pairs):
    """search.py:221-307 for many (start, goal) pairs at once, each search resident on the GPU
    (tr_astar_batch, one wave per query): a list with what astar(start, goal) returns for each pair,
    without the prints.  Raises where the reference raises (IndexError / ValueError)."""
    q = [[s[0], s[1], g[0], g[1]] for s, g in pairs]
    paths, st = config.engine().astar_batch(q, bool(config.get("THETASTAR")))
    out = []
    for p, row in zip(paths, st):
        if row[3] == 4:
            raise IndexError("index is out of bounds (imarray[y][x], search.py:30)")
        if row[3] == 5:
            raise ValueError("attempt to get argmin of an empty sequence (search.py:262)")
        if row[3] >= 6:
            raise _native.NativeError("astar_many: device queue capacity (status %d)" % row[3])
        out.append(False if p is None else [(int(x), int(y)) for x, y in p])
    return out


def drawpath(mainpath):
    """search.py:206-219 (matplotlib, host only: draw.py); pixels from the GPU bresenham."""
    from . import draw
    return draw.search_drawpath(mainpath, bresenham)
