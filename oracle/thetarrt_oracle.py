"""CPU oracle for the theta-rrt hot path — TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this module,
and only as the checker / the timed CPU baseline.  The product (`theta-rrt_amd/`) never imports it.

What it is: a restatement, in plain Python + numpy, of the eshira/theta-rrt algorithm on the
north-star path (rand_conf through the loop bookkeeping, and the Theta* line of sight).  Every function cites the reference file:line it
follows.  Where the reference calls third-party arithmetic the oracle does this:

* numpy primitives the reference calls (`np.arctan2`, `np.dot`, `np.linalg.solve/cond/norm`,
  `np.clip`, `np.random` legacy normal) are called here the same way, so the oracle inherits the
  same machine behaviour as the reference would have on the same host;
* scipy `Rotation` (scipy 1.15.3, compiled only) is restated: quaternion from a z-Euler angle,
  rotation-matrix apply, quaternion compose + normalise and the `as_euler('xyz')` extraction.  The
  restatement was checked bit-for-bit against scipy 1.15.3 on 20k random inputs each
  (tests/test_oracle.py re-checks it against the installed scipy and against the golden vectors).

Pinning: tests/golden/*.npz were captured by importing the reference itself in the build container
(tests/golden/make_golden.py); tests/test_oracle.py checks this oracle against every one of them.

Batch semantics (new; the reference is strictly sequential, rrt.py:141): see `rrt_batched`.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

# ----------------------------------------------------------------------------- parameters
@dataclass
class Params:
    """The `builtins.*` parameter block of main.py:14-32 (same names, same defaults)."""
    THETASTAR: bool = True
    bikelength: float = 5
    FORWARDONLY: bool = True
    LEFTCONSTRAINT: float = -65
    RIGHTCONSTRAINT: float = 65
    frontclearance: float = 2
    K: int = 300
    maxdrivedist: float = 30
    tol_xy: float = 10
    tol_ang: float = 45
    weightxy: float = .6
    xystdv: float = 0.4
    anglestdv: float = 100


DEG = math.pi / 180.0          # np.deg2rad multiplier
RAD = 180.0 / math.pi          # np.rad2deg multiplier


# ----------------------------------------------------------------------------- angles
def wrap180(a):
    """standardangle, rrt.py:9-14: repeated +-360 until a in (-180, 180]."""
    while a > 180:
        a = a - 360
    while a <= -180:
        a = a + 360
    return a


def _zquat(deg):
    """Rotation.from_euler('z', deg, degrees=True) quaternion (x, y, z, w)."""
    h = deg * DEG / 2
    return (0.0, 0.0, math.sin(h), math.cos(h))


def _zrot(deg, v):
    """Rotation.from_euler('z', deg, degrees=True).apply(v) for a 3-vector v (scipy matrix path)."""
    x, y, z, w = _zquat(deg)
    x2, y2, z2, w2 = x * x, y * y, z * z, w * w
    xy, zw, xz, yw, yz, xw = x * y, z * w, x * z, y * w, y * z, x * w
    m = ((x2 - y2 - z2 + w2, 2 * (xy - zw), 2 * (xz + yw)),
         (2 * (xy + zw), -x2 + y2 - z2 + w2, 2 * (yz - xw)),
         (2 * (xz - yw), 2 * (yz + xw), -x2 - y2 + z2 + w2))
    v0, v1, v2 = float(v[0]), float(v[1]), float(v[2])
    return np.array([m[i][0] * v0 + m[i][1] * v1 + m[i][2] * v2 for i in range(3)])


def angle_diff(a1, a2):
    """anglediff, rrt.py:108-115: z angle of Rz(a1)^-1 * Rz(a2), scipy arithmetic restated."""
    p = _zquat(a1)
    p = (-p[0], -p[1], -p[2], p[3])                      # inv()
    q = _zquat(a2)
    cr = (p[1] * q[2] - p[2] * q[1], p[2] * q[0] - p[0] * q[2], p[0] * q[1] - p[1] * q[0])
    r = [p[3] * q[k] + q[3] * p[k] + cr[k] for k in range(3)]
    r.append(p[3] * q[3] - (p[0] * q[0] + p[1] * q[1] + p[2] * q[2]))
    n = math.sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3])
    x, y, z, w = (c / n for c in r)
    # as_euler('xyz') third angle: half_sum + half_diff (Tait-Bryan, extrinsic, sign +1)
    ang = math.atan2(x + z, w - y) + math.atan2(z - x, y + w)
    if ang < -math.pi:
        ang += 2 * math.pi
    elif ang > math.pi:
        ang -= 2 * math.pi
    return ang * RAD


def angle_between(v1, v2):
    """anglebetween, rrt.py:73-77 (numpy dot / arctan2 exactly as the reference calls them)."""
    dot = np.dot(v1[:2], v2)
    det = v2[0] * v1[1] - v1[0] * v2[1]
    return wrap180(np.rad2deg(np.arctan2(det, dot)))


def heading(v):
    """anglebetween([1,0], v): the image-frame angle of v."""
    return angle_between([1, 0], v)


def _line(p, q):
    """linefrompoints, rrt.py:42-46."""
    a = q[1] - p[1]
    b = p[0] - q[0]
    return a, b, a * p[0] + b * p[1]


def arc_len(radius, angle):
    """angle_to_arclength, rrt.py:48-51."""
    while angle < 0:
        angle = angle + 360
    return (np.pi * 2 * radius) * angle / 360


def arc_angle(radius, length):
    """arclength_to_angle, rrt.py:70-71 (TypeError when radius is None, as in the reference)."""
    return length * 360 / (np.pi * 2 * radius)


# ----------------------------------------------------------------------------- grid (search.py:13-94)
class Grid:
    """Occupancy grid `imarray` (bool, [y][x], True = free) and its queries."""

    def __init__(self, free):
        self.free = np.asarray(free, dtype=bool)

    def valid(self, node):
        """search.py:17-24 — note x is checked against shape[0] and y against shape[1]."""
        x, y = int(node[0]), int(node[1])
        return 0 <= x < self.free.shape[0] and 0 <= y < self.free.shape[1]

    def freespace(self, node):
        """search.py:26-33."""
        return self.valid(node) and bool(self.free[int(node[1])][int(node[0])])

    def los(self, n1, n2):
        """lineofsight, search.py:35-41."""
        return all(self.freespace(p) for p in bresenham(n1, n2))


def l2(a, b):
    """L2norm, search.py:13-15."""
    return math.sqrt(pow((b[0] - a[0]), 2) + pow((b[1] - a[1]), 2))


def bresenham(n1, n2):
    """search.py:43-94: integer Bresenham, iterating along the increasing major axis."""
    x0, y0, x1, y1 = int(n1[0]), int(n1[1]), int(n2[0]), int(n2[1])
    steep = not (abs(y1 - y0) < abs(x1 - x0))
    if steep:   # plotLineHigh: swap roles of x and y
        x0, y0, x1, y1 = y0, x0, y1, x1
    if x0 > x1:
        x0, y0, x1, y1 = x1, y1, x0, y0
    dx, dy = x1 - x0, y1 - y0
    step = 1
    if dy < 0:
        step, dy = -1, -dy
    err = 2 * dy - dx
    out = []
    y = y0
    for x in range(x0, x1 + 1):
        out.append((y, x) if steep else (x, y))
        if err > 0:
            y += step
            err -= 2 * dx
        err += 2 * dy
    return out


# ----------------------------------------------------------------------------- circle / arc (search.py:96-182)
def circle_pixels(grid, center, r):
    """getCircle, search.py:107-142 (midpoint circle + optional diagonal patch), valid-filtered."""
    xc, yc, r = int(center[0]), int(center[1]), int(r)
    x, y, d = r, 0, 1 - r
    pix = []
    while x > y:
        vals = (-x, x, -y, y)
        for v1 in vals:
            for v2 in vals:
                if abs(v1) != abs(v2):
                    p = (xc + v1, yc + v2)
                    if grid.valid(p):
                        pix.append(p)
        y += 1
        if d < 0:
            d += 2 * y + 1
        else:
            x -= 1
            d += 2 * (y - x) + 1
    s = r * 0.5 * math.sqrt(2)
    t = (xc + int(round(s)), yc + int(round(s)))
    members = set(pix)
    if not any(q in members for q in ((t[0] + 1, t[1]), (t[0] - 1, t[1]), (t[0], t[1] + 1), (t[0], t[1] - 1))):
        k = round(s)
        for p in ((xc + k, yc + k), (xc - k, yc - k), (xc + k, yc - k), (xc - k, yc + k)):
            if grid.valid(p):
                pix.append(p)
    return pix


def _ad_vec(a1, a2):
    """angle_diff over arrays: closed form away from the 0/+-180 branch points, exact restatement
    inside a 1e-9 deg band (the closed form differs from scipy by < 1e-11 deg, so every sign and
    `< 180` decision taken outside the band equals scipy's)."""
    d = a2 - a1
    d = np.where(d > 180, d - 360, d)
    d = np.where(d <= -180, d + 360, d)
    band = (np.abs(d) < 1e-9) | (np.abs(d) > 180 - 1e-9)
    for i in np.nonzero(band)[0]:
        d[i] = angle_diff(float(np.broadcast_to(a1, d.shape)[i]), float(np.broadcast_to(a2, d.shape)[i]))
    return d


def arc_pixels(grid, begin, land, u):
    """getArc, search.py:144-182: circle pixels kept by the begin->land angular window."""
    if u[1] is None:
        return bresenham(begin, land)
    pix = circle_pixels(grid, u[1], u[2])
    icc = u[1]
    b_ang = heading(np.subtract(begin, icc))
    e_ang = heading(np.subtract(land, icc))
    diff = angle_diff(b_ang, e_ang) if u[0] < 0 else angle_diff(e_ang, b_ang)
    if diff < 0:
        diff = 360 + diff
    if not pix:
        return []
    P = np.array(pix, dtype=np.float64)
    v = P - np.asarray(icc, dtype=np.float64)
    # heading() of every pixel, vectorised with the same numpy ufuncs
    ang = np.rad2deg(np.arctan2(v[:, 0] * 0 - 1 * v[:, 1], v[:, 0]))
    ang = np.where(ang > 180, ang - 360, ang)
    ang = np.where(ang <= -180, ang + 360, ang)
    if u[0] > 0:
        fwd, bwd = _ad_vec(ang, b_ang), _ad_vec(e_ang, ang)
    else:
        fwd, bwd = _ad_vec(b_ang, ang), _ad_vec(ang, e_ang)
    keep = ((fwd >= 0) & (bwd >= 0)) if diff < 180 else ((fwd >= 0) | (bwd >= 0))
    return [p for p, k in zip(pix, keep) if k]


# ----------------------------------------------------------------------------- kinematics (rrt.py:208-541)
class StraightDrive(TypeError):
    """The reference's latent TypeError: drive() on a straight control (rrt.py:275 -> :71)."""


def body_clear(grid, P, bike, mult=1.0):
    """bike_clear (mult=1, rrt.py:208-213) / front_of_bike_clear (mult=frontclearance, :215-222)."""
    f = _zrot(bike[1], [P.bikelength * mult, 0, 0])
    pv = np.add(f[:2], bike[0])
    return grid.los(bike[0], (int(pv[0]), int(pv[1])))


def drive(P, origin, u):
    """drive, rrt.py:272-304: rotate the bike frame about the ICC by u[3] of arc length."""
    if u[1] is None:
        raise StraightDrive("unsupported operand type(s) for *: 'float' and 'NoneType'")
    ang = arc_angle(u[2], u[3])
    front = _zrot(origin[1], [P.bikelength, 0, 0])
    back = _zrot(180, front)
    o3 = [origin[0][0], origin[0][1], 0]
    c3 = [u[1][0], u[1][1], 0]
    front = np.add(np.subtract(o3, c3), front)
    back = np.add(np.subtract(o3, c3), back)
    rot = -ang if u[0] < 0 else ang
    front, back = _zrot(rot, front), _zrot(rot, back)
    front = np.add(c3[:2], front[:2])
    back = np.add(c3[:2], back[:2])
    mid = 0.5 * np.add(back, front)
    theta = -heading(np.subtract(front[:2], mid))
    return ((mid[0], mid[1]), theta), u


def _solve_icc(a, b):
    """np.linalg.solve + the cond > 1e6 test of rrt.py:347-350 / :388-391 (None = singular)."""
    try:
        x = np.linalg.solve(a, b)
    except np.linalg.LinAlgError:
        return None
    if np.linalg.cond(a) > 1000000:
        return None
    return x


def steer(P, origin, theta, goal, theta_goal):
    """steer, rrt.py:306-541.  Returns ((point, angle), u) with u = (steer, ICC, rad, dist) or the
    straight control (0, None, None, 1)."""
    mid = np.array([0.5 * (origin[0] + goal[0]), 0.5 * (origin[1] + goal[1])])
    bis = np.subtract(origin, goal)
    frame = _zrot(theta, [P.bikelength, 0, 0])
    normal = _zrot(90, frame)
    perp = _zrot(90, [bis[0], bis[1], 0])
    a1, b1, c1 = _line(mid, np.add(mid, perp[:2]))
    a2, b2, c2 = _line(origin, np.add(origin, normal[:2]))
    icc = _solve_icc(np.array([[a1, b1], [a2, b2]]), np.array([c1, c2]))
    if icc is None:
        return _straight(P, origin, theta, goal)
    rad = np.linalg.norm(np.subtract(origin, icc))
    pivot = np.add(frame[:2], origin)
    sv = np.subtract(pivot, icc)
    sv = _zrot(90, [sv[0], sv[1], 0])[:2]
    steer_a = wrap180(-angle_between(frame[:2], sv))
    if P.FORWARDONLY and (steer_a > 90 or steer_a < -90):
        steer_a = wrap180(steer_a + 180)
    limited = False
    if steer_a < P.LEFTCONSTRAINT or steer_a > P.RIGHTCONSTRAINT:
        steer_a = P.LEFTCONSTRAINT if steer_a < P.LEFTCONSTRAINT else P.RIGHTCONSTRAINT
        fnorm = _zrot(steer_a, normal)
        a1, b1, c1 = _line(pivot, np.add(pivot, fnorm[:2]))
        a2, b2, c2 = _line(origin, np.add(origin, normal[:2]))
        icc = _solve_icc(np.array([[a1, b1], [a2, b2]]), np.array([c1, c2]))
        if icc is None:
            return _straight(P, origin, theta, goal)
        rad = np.linalg.norm(np.subtract(origin, icc))
        limited = True
    ccw = -90 if ((0 <= steer_a < 90) or (-180 < steer_a <= -90)) else 90

    def tangent_heading(pt):
        fv = np.subtract(pt, icc)
        return -heading(_zrot(-ccw, [fv[0], fv[1], 0])[:2])

    final = tangent_heading(goal)
    mix = P.weightxy * wrap180(final) + (1 - P.weightxy) * wrap180(theta_goal)
    if limited:
        mix = heading(np.subtract(goal, origin))
    t2 = mix + ccw
    goal_ang = heading(np.subtract(goal, icc))
    cands = []
    for t in (t2, t2 + 180):
        mp = _zrot(t, [1, 0, 0])[:2]
        mp = rad * mp / np.linalg.norm(mp)
        mp = np.add(icc, mp)
        cands.append((mp, angle_diff(heading(np.subtract(mp, icc)), goal_ang)))
    final = mix
    if abs(cands[0][1]) < abs(cands[1][1]):
        gp = cands[0][0]
    else:
        gp = cands[1][0]
        final = wrap180(final - 180)
    if limited:
        gp = cands[0][0]
        final = tangent_heading(gp)
    to_origin = np.subtract(origin, icc)
    arc = angle_diff(heading(np.subtract(gp, icc)), heading(to_origin))
    if steer_a > 0:
        if arc < 0:
            arc = 360 + arc
    elif arc > 0:
        arc = 360 - arc
    dist = arc_len(rad, abs(arc))
    if dist > P.maxdrivedist:
        dist = P.maxdrivedist
        turn = arc_angle(rad, P.maxdrivedist)
        gp = _zrot(-turn if steer_a < 0 else turn, [to_origin[0], to_origin[1], 0])
        gp = np.add(gp[:2], icc)
        final = tangent_heading(gp)
    return (gp, final), (steer_a, icc, rad, dist)


def _straight(P, origin, theta, goal):
    """The LinAlgError branch of steer, rrt.py:526-541."""
    v = np.subtract(goal, origin)
    if np.linalg.norm(v) > 0.000001:
        step = P.maxdrivedist * v / np.linalg.norm(v)
        if not (np.linalg.norm(step) > np.linalg.norm(v)):
            goal = np.add(origin, step)
    return (goal, theta), (0, None, None, 1)


def rand_conf(P, shape, goal):
    """rand_conf, rrt.py:53-68 — consumes 3 legacy gaussians of the global np.random stream."""
    rx, ry = np.random.normal(goal[0], [P.xystdv * shape[0], P.xystdv * shape[1]], 2)
    c = np.array([rx, ry])
    np.clip([rx, ry], [0, 0], [shape[0] - 1, shape[1] - 1], out=c)
    t = wrap180(np.random.normal(wrap180(goal[1]), P.anglestdv, 1)[0])
    return ((int(c[0]), int(c[1])), t)


def samples_from_gauss(P, shape, goal, g):
    """rand_conf batched: row j of g (shape (B,3), the next 3B legacy gaussians) -> sample j.

    Bit-identical to B successive rand_conf calls (normal = loc + scale * gauss)."""
    g = np.asarray(g, np.float64).reshape(-1, 3)
    sx, sy = P.xystdv * shape[0], P.xystdv * shape[1]
    x = np.clip(goal[0][0] + sx * g[:, 0], 0, shape[0] - 1)
    y = np.clip(goal[0][1] + sy * g[:, 1], 0, shape[1] - 1)
    t = [wrap180(wrap180(goal[1]) + P.anglestdv * float(v)) for v in g[:, 2]]
    return [((int(a), int(b)), wrap180(c)) for a, b, c in zip(x.tolist(), y.tolist(), t)]


# ----------------------------------------------------------------------------- nearest neighbour (rrt.py:155-158)
def nn_loop(tree_xy, q):
    """The reference's inline argmin (rrt.py:156-157), pure Python: first index of min L2norm."""
    best, bi = None, -1
    for i, p in enumerate(tree_xy):
        d = l2(p, q)
        if best is None or d < best:
            best, bi = d, i
    return bi


def nn_numpy(tx, ty, qx, qy):
    """Vectorised restatement of the same arithmetic (pow(.,2) == x*x correctly rounded; the sum and
    sqrt are single IEEE ops), np.argmin -> first index on ties.  tx/ty fp64 (N,), qx/qy (B,)."""
    out = np.empty(len(qx), np.int64)
    tx = np.asarray(tx, np.float64)
    ty = np.asarray(ty, np.float64)
    step = max(1, (1 << 24) // max(1, len(tx)))
    for s in range(0, len(qx), step):
        dx = np.asarray(qx[s:s + step], np.float64)[:, None] - tx[None, :]
        dy = np.asarray(qy[s:s + step], np.float64)[:, None] - ty[None, :]
        out[s:s + step] = np.argmin(np.sqrt(dx * dx + dy * dy), axis=1)
    return out


# ----------------------------------------------------------------------------- findnearest (rrt.py:117-128)
def findnearest(P, nodes, e_par, e_child, goal):
    """rrt.findnearest over edges (e_par[k], e_child[k]) listed in the reference's traversal order
    (`for parent in G.keys(): for child in G[parent]`): the first child with the smallest
    weightxy * L2norm(child, goal) + (1 - weightxy) * |anglediff(child, goal)| (strict <, rrt.py:126).
    nodes: [n][3] poses; goal: ((x, y), theta).  Returns (node index | -1, distance | None)."""
    best, bi = None, -1
    for c in e_child:
        x, y, t = nodes[c]
        d = P.weightxy * l2((x, y), goal[0]) + (1 - P.weightxy) * abs(angle_diff(t, goal[1]))
        if best is None or d < best:
            best, bi = d, int(c)
    return bi, best


# ----------------------------------------------------------------------------- one expansion (rrt.py:144-188)
@dataclass
class Expansion:
    status: str                     # 'blocked_sample' | 'dup_sample' | 'collision' | 'ok' | 'straight_drive'
    qrand: tuple = None
    near: int = -1
    qnew: tuple = None
    u: tuple = None
    drove: bool = False


def expand_one(P, grid, nodes, qrand, nn=None):
    """The per-sample body of rrt.py:144-176 against a frozen node list `nodes` (poses)."""
    if not grid.freespace(qrand[0]):
        return Expansion("blocked_sample", qrand)
    if nn is None:
        nn = nn_loop([n[0] for n in nodes], qrand[0])
    qnear = nodes[nn]
    (gp, th), u = steer(P, qnear[0], qnear[1], qrand[0], qrand[1])
    qnew = ((gp[0], gp[1]), th)
    drove = False
    if not grid.valid(qnew[0]) or not body_clear(grid, P, qnew) or not body_clear(grid, P, qnew, P.frontclearance):
        u = (u[0], u[1], u[2], u[3] / 3)
        drove = True
        try:
            qnew, u = drive(P, qnear, u)
        except StraightDrive:
            return Expansion("straight_drive", qrand, nn, None, u, True)
    # rrt.py:173-174: `False in [freespace(px) for px in pixels]` tests every pixel first (eager
    # list), so on a non-square map a pixel after a blocked one still raises IndexError
    if False in [grid.freespace(p) for p in arc_pixels(grid, qnear[0], qnew[0], u)]:
        return Expansion("collision", qrand, nn, qnew, u, drove)
    return Expansion("ok", qrand, nn, qnew, u, drove)


def _key(pose):
    return (float(pose[0][0]), float(pose[0][1]), float(pose[1]))


@dataclass
class Tree:
    """Insertion-ordered tree = the reference's dict G + cameFrom (rrt.py:134-138, 179-188)."""
    nodes: list = field(default_factory=list)       # poses in insertion order (= G.keys() order)
    index: dict = field(default_factory=dict)       # exact-value key -> node index
    children: list = field(default_factory=list)    # G[node] edge lists (duplicates allowed)
    parent: list = field(default_factory=list)      # cameFrom parent index (-1 = None / unset)
    u: list = field(default_factory=list)           # cameFrom control

    def add(self, pose):
        k = _key(pose)
        if k in self.index:
            return self.index[k], False
        self.index[k] = len(self.nodes)
        self.nodes.append(pose)
        self.children.append([])
        self.parent.append(-1)
        self.u.append(None)
        return len(self.nodes) - 1, True


def rrt_batched(P, grid, start, goal, B=1, gauss_source=None, nn_fn=None, on_batch=None,
                straight="raise"):
    """rrt, rrt.py:130-206, in snapshot-batch form.  B=1 is the reference loop exactly.

    Batch semantics: the K-1 iterations are taken B at a time.  Every per-sample decision
    that reads the tree (membership of qrand, nearest node) reads the tree as it stood when the batch
    began; samples whose expansion succeeds are then appended in sample order with the reference's
    bookkeeping (duplicate vertices merged, edge always added, cameFrom only if qnew != qnear), and
    the batch stops at the first node within tolerance of the goal.  Raises StraightDrive where the
    reference raises TypeError (straight="reject" discards that candidate instead: engine option).
    """
    start = (start[0], wrap180(start[1]))
    goal = (goal[0], wrap180(goal[1]))
    T = Tree()
    T.add(start)
    shape = grid.free.shape
    total, done, sol = P.K - 1, 0, None
    while done < total and sol is None:
        b = min(B, total - done)
        done += b
        g = gauss_source(3 * b) if gauss_source else np.random.standard_normal(3 * b)
        qs = samples_from_gauss(P, shape, goal, g)
        snap = list(T.nodes)
        n_snap = len(snap)
        txy = np.array([[float(n[0][0]), float(n[0][1])] for n in snap])
        live = [j for j, q in enumerate(qs) if grid.freespace(q[0]) and
                not (_key(q) in T.index and T.index[_key(q)] < n_snap)]
        if nn_fn is None:
            near = nn_numpy(txy[:, 0], txy[:, 1], [qs[j][0][0] for j in live], [qs[j][0][1] for j in live])
        else:
            near = nn_fn(txy, [qs[j][0] for j in live])
        recs = []
        for j, nn in zip(live, near):
            e = expand_one(P, grid, snap, qs[j], int(nn))
            if e.status == "straight_drive" and straight == "raise":
                raise StraightDrive("unsupported operand type(s) for *: 'float' and 'NoneType'")
            if e.status == "ok":
                recs.append(e)
        for e in recs:
            i_new, _ = T.add(e.qnew)
            T.children[e.near].append(i_new)
            if _key(e.qnew) != _key(snap[e.near]):
                T.parent[i_new] = e.near
                T.u[i_new] = e.u
            if l2(e.qnew[0], goal[0]) < P.tol_xy and abs(angle_diff(e.qnew[1], goal[1])) < P.tol_ang:
                sol = i_new
                break
        if on_batch:
            on_batch(T, qs, recs)
    return sol, T


# ----------------------------------------------------------------------------- Theta* (search.py:184-307)
def astar(P, grid, start, goal, los_fn=None):
    """astar with lazy Theta*, search.py:221-307.  Returns (path | False, expanded, los_calls).

    `los_fn(a, b)` defaults to grid.los; the reference's PriorityQueue ordering of (f, node) tuples is
    reproduced with heapq on the same tuples."""
    import heapq
    import itertools
    los_fn = los_fn or grid.los
    if not grid.valid(start) or not grid.valid(goal):
        return False, 0, 0
    if not grid.freespace(start) or not grid.freespace(goal):
        return False, 0, 0

    def nbrs(n):
        out = []
        for d in itertools.product([-1, 0, 1], repeat=2):
            if d != (0, 0):
                c = (int(n[0] - d[0]), int(n[1] - d[1]))
                if grid.valid(c) and grid.freespace(c):
                    out.append(c)
        return out

    closed, openset, came, g = set(), set(), {}, {start: 0}
    pq = []
    for n in nbrs(start):
        g[n] = l2(start, n)
        came[n] = start
        openset.add(n)
        heapq.heappush(pq, (g[n] + l2(n, goal), n))
    closed.add(start)
    los_calls = 0
    while pq:
        cur = heapq.heappop(pq)[1]
        if cur in closed:
            continue
        if P.THETASTAR:
            los_calls += 1
            if not los_fn(cur, came[cur]):
                cand = [n for n in nbrs(cur) if n in closed]
                vals = [g[n] + l2(n, cur) for n in cand]
                k = int(np.argmin(vals))
                came[cur], g[cur] = cand[k], vals[k]
        openset.remove(cur)
        closed.add(cur)
        if cur == goal:
            path = [cur]
            while path[-1] in came:
                path.append(came[path[-1]])
            return path[::-1], len(closed), los_calls
        for nb in nbrs(cur):
            if nb in closed:
                continue
            gg = g[cur] + l2(nb, cur)
            if nb not in openset:
                g[nb] = gg
                heapq.heappush(pq, (gg + l2(nb, goal), nb))
                openset.add(nb)
                came[nb] = cur
            elif gg < g[nb]:
                g[nb] = gg
                came[nb] = cur
                heapq.heappush(pq, (gg + l2(nb, goal), nb))
            if P.THETASTAR:
                par = came[cur]
                gg = g[par] + l2(par, nb)
                if gg < g[nb]:
                    came[nb] = par
                    g[nb] = gg
                    heapq.heappush(pq, (gg + l2(nb, goal), nb))
    return False, len(closed), los_calls
