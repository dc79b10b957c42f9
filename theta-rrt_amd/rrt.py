"""Bicycle kinematics, sampler and RRT (reference: rrt.py), with the hot loop on the GPU.

Same names, arguments and return shapes as eshira/theta-rrt rrt.py.  `rrt()` runs the whole
expansion loop in libthetarrt.so: per batch of B samples one fused GPU pass (NN argmin, steer,
body rays, drive, arc check) and the reference's bookkeeping in C++ on the host.  B=1 (the default)
is the reference loop exactly; B>1 uses snapshot-batch semantics (every sample of a batch sees the tree as it stood when the batch began; accepted nodes are appended in sample order).

Parameters are the reference's `builtins` names (main.py:14-32); `builtins.rrt_batch` sets the
default batch size.
"""
import builtins
import math

import numpy as np

from . import config, search

_DEG = math.pi / 180.0
_RAD = 180.0 / math.pi


def standardangle(angle):
    """rrt.py:9-14."""
    while angle > 180:
        angle = angle - 360
    while angle <= -180:
        angle = angle + 360
    return angle


def linefrompoints(p, q):
    """rrt.py:42-46."""
    a = q[1] - p[1]
    b = p[0] - q[0]
    return a, b, a * p[0] + b * p[1]


def angle_to_arclength(radius, angle):
    """rrt.py:48-51."""
    while angle < 0:
        angle = angle + 360
    return (np.pi * 2 * radius) * angle / 360


def arclength_to_angle(radius, arclength):
    """rrt.py:70-71."""
    return arclength * 360 / (np.pi * 2 * radius)


def anglebetween(vec1, vec2):
    """rrt.py:73-77."""
    dot = np.dot(vec1[:2], vec2)
    det = vec2[0] * vec1[1] - vec1[0] * vec2[1]
    return standardangle(np.rad2deg(np.arctan2(det, dot)))


def anglediff(angle1, angle2):
    """rrt.py:108-115: z angle of Rz(a1)^-1 Rz(a2) in degrees (scipy Rotation arithmetic)."""
    h1, h2 = angle1 * _DEG / 2, angle2 * _DEG / 2
    pz, pw = -math.sin(h1), math.cos(h1)
    qz, qw = math.sin(h2), math.cos(h2)
    px = py = -0.0
    qx = qy = 0.0
    r0 = pw * qx + qw * px + (py * qz - pz * qy)
    r1 = pw * qy + qw * py + (pz * qx - px * qz)
    r2 = pw * qz + qw * pz + (px * qy - py * qx)
    r3 = pw * qw - (px * qx + py * qy + pz * qz)
    n = math.sqrt(r0 * r0 + r1 * r1 + r2 * r2 + r3 * r3)
    x, y, z, w = r0 / n, r1 / n, r2 / n, r3 / n
    a = math.atan2(x + z, w - y) + math.atan2(z - x, y + w)
    if a < -math.pi:
        a += 2 * math.pi
    elif a > math.pi:
        a -= 2 * math.pi
    return np.float64(a * _RAD)


def rand_conf(mean):
    """rrt.py:53-68: goal-biased pose from the global np.random stream (3 legacy gaussians)."""
    a = config.imarray()
    xs, ys = config.get("xystdv") * a.shape[0], config.get("xystdv") * a.shape[1]
    randx, randy = np.random.normal(mean[0], [xs, ys], 2)
    clipped = np.array([randx, randy])
    np.clip([randx, randy], [0, 0], [a.shape[0] - 1, a.shape[1] - 1], out=clipped)
    t = standardangle(np.random.normal(standardangle(mean[1]), config.get("anglestdv"), 1)[0])
    return ((int(clipped[0]), int(clipped[1])), t)


def _u_from_row(o):
    if o[8]:
        return (0, None, None, 1)
    return (o[3], np.array([o[4], o[5]]), o[6], o[7])


def steer(bikeorigin, theta, bikegoal, thetagoal, plot=False):
    """rrt.py:306-541 on the GPU.  Returns ((goal_point, final_angle), u)."""
    o = config.engine().steer(np.array([[bikeorigin[0], bikeorigin[1], theta, bikegoal[0],
                                         bikegoal[1], thetagoal]], np.float64))[0]
    if o[8]:
        moved = (o[0], o[1]) != (float(bikegoal[0]), float(bikegoal[1]))
        goal = np.array([o[0], o[1]]) if moved else bikegoal
        return (goal, theta), (0, None, None, 1)
    return (np.array([o[0], o[1]]), o[2]), _u_from_row(o)


def drive(bikeorigin, u):
    """rrt.py:272-304 on the GPU.  A straight control raises TypeError, as in the reference."""
    if u[1] is None or u[2] is None:
        raise TypeError("unsupported operand type(s) for *: 'float' and 'NoneType'")
    row = np.array([[bikeorigin[0][0], bikeorigin[0][1], bikeorigin[1], u[0], u[1][0], u[1][1],
                     u[2], u[3], 0.0]], np.float64)
    out, ok = config.engine().drive(row)
    return ((out[0, 0], out[0, 1]), out[0, 2]), u


def bike_clear(bike):
    """rrt.py:208-213."""
    return bool(config.engine().body_clear(np.array([[bike[0][0], bike[0][1], bike[1]]]), 1.0)[0])


def front_of_bike_clear(bike, plot=False):
    """rrt.py:215-222."""
    m = float(config.get("frontclearance"))
    return bool(config.engine().body_clear(np.array([[bike[0][0], bike[0][1], bike[1]]]), m)[0])


def findnearest(tree, goal):
    """rrt.py:117-128: the child (first in `for parent in G.keys(): for child in G[parent]` order)
    with the smallest weightxy * L2norm + (1 - weightxy) * |anglediff| to `goal`, on the GPU.
    Returns (child, distance), or (None, None) for a tree without edges, like the reference."""
    keys = list(tree.keys())
    index = {k: i for i, k in enumerate(keys)}
    e_par, e_child = [], []
    for i, parent in enumerate(keys):
        for child in tree[parent]:
            e_par.append(i)
            e_child.append(index[child])
    if not e_child:
        return (None, None)
    xyt = np.array([[k[0][0], k[0][1], k[1]] for k in keys], np.float64)
    node, dist = config.engine().findnearest(xyt, e_par, e_child, [[goal[0][0], goal[0][1], goal[1]]])
    return (keys[int(node[0])], float(dist[0]))


def _pose(row):
    return ((float(row[0]), float(row[1])), float(row[2]))


def tree_views(ex):
    """Rebuild the reference's dict views (G, cameFrom) from exported arrays."""
    keys = [_pose(r) for r in ex["nodes"]]
    G = {}
    for i, k in enumerate(keys):
        G[k] = [keys[c] for c in ex["e_child"][ex["e_off"][i]:ex["e_off"][i + 1]]]
    cameFrom = {keys[0]: None}
    for i, p in enumerate(ex["parent"]):
        if p >= 0:
            u = ex["u"][i]
            uu = (u[0], None, None, u[4]) if u[5] else (u[0], np.array([u[1], u[2]]), u[3], u[4])
            cameFrom[keys[i]] = (keys[p], uu)
    return keys, G, cameFrom


def run(start, goal, batch=1, gauss_source=None, debug=False, engine=None):
    """Run the batched RRT and return (sol_index | -1, exported arrays).  `gauss_source(n)` returns
    the next n legacy gaussians; by default they are the global np.random stream rand_conf draws
    (rrt.py:58,66): for batch > 1 the engine draws that stream itself on the GPU (seeded from
    np.random.get_state(), written back after the run, so np.random continues exactly as if the
    host had drawn the batches used) and runs the full batches in its native pipelined loop."""
    eng = engine or config.engine()
    start = (start[0], standardangle(start[1]))
    goal = (goal[0], standardangle(goal[1]))
    eng.rrt_begin([start[0][0], start[0][1], start[1]], [goal[0][0], goal[0][1], goal[1]])
    total, done, sol = int(config.get("K")) - 1, 0, -1
    rows = total // int(batch) if (gauss_source is None and int(batch) > 1 and not debug) else 0
    if rows:
        eng.rng_set_state(np.random.get_state())
        # look-ahead for batches up to 8192 samples (the correction scans the last batch's nodes;
        # larger batches sweep on their own stream)
        try:
            _, sol = eng.run(None, int(batch), rows, 0, 0, stage=1 if int(batch) <= 8192 else 0)
        finally:
            # also where the reference raises (TypeError / IndexError): the engine has rewound its
            # stream to the end of the raising batch, as the host-drawn loop leaves np.random
            np.random.set_state(eng.rng_get_state())
        done = rows * int(batch)
    while done < total and sol < 0:
        b = min(int(batch), total - done)
        if debug:
            print(done + 1 if b == 1 else "%d-%d" % (done + 1, done + b))
        done += b
        g = gauss_source(3 * b) if gauss_source else np.random.standard_normal(3 * b)
        _, sol = eng.rrt_step(g)
    return sol, eng.book().export()


def rrt(start, goal, debug=False, batch=None):
    """rrt.py:130-206.  Returns (sol | None, G, cameFrom) like the reference."""
    if batch is None:
        batch = getattr(builtins, "rrt_batch", 1)
    sol, ex = run(start, goal, batch=batch, debug=debug)
    keys, G, cameFrom = tree_views(ex)
    if sol >= 0:
        print('Found goal!')
    print("Nodes in tree: ", len(keys))
    return (keys[sol] if sol >= 0 else None), G, cameFrom


def draw_bicycle(bike_loc, theta, alpha, color='blue'):
    """rrt.py:16-40 (matplotlib, host only: draw.py)."""
    from . import draw
    return draw.draw_bicycle(bike_loc, theta, alpha, color=color)


def draw_path_segment(bike1, bike2, u, colors=None, bikes=True):
    """rrt.py:224-270 (matplotlib, host only: draw.py)."""
    from . import draw
    return draw.draw_path_segment(bike1, bike2, u, colors=colors, bikes=bikes)


def drawpath(solution, camefrom):
    """rrt.py:79-98 (matplotlib, host only: draw.py)."""
    from . import draw
    return draw.drawpath(solution, camefrom)


def drawtree(begin, graph, camefrom):
    """rrt.py:100-106 (matplotlib, host only: draw.py)."""
    from . import draw
    return draw.drawtree(begin, graph, camefrom)
