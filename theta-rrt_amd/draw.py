"""Plotting of trees, paths and bicycles (reference: rrt.py:16-40,79-106,224-270, search.py:206-219).

Host-side matplotlib only, off the hot path: the same function names,
arguments, colours and z-order as the reference, drawing onto `builtins.ax` when main.py has set
it (main.py:44) or onto the current axes otherwise.  Rotations are the closed-form z rotations the
reference builds with scipy `Rotation.from_euler('z', deg)`; a drawing has no parity bar beyond
placing the same primitives at the same coordinates.  matplotlib is imported on first use.
"""
import builtins
import math

import numpy as np

from . import config


def _plt():
    import matplotlib.pyplot as plt
    return plt


def _ax():
    a = getattr(builtins, "ax", None)
    return a if a is not None else _plt().gca()


def _rot(deg, v):
    """Rotation.from_euler('z', deg, degrees=True).apply([x, y, 0])[:2]."""
    c, s = math.cos(math.radians(deg)), math.sin(math.radians(deg))
    return np.array([c * v[0] - s * v[1], s * v[0] + c * v[1]])


def _standardangle(a):
    while a > 180:
        a -= 360
    while a <= -180:
        a += 360
    return a


def _anglebetween(v1, v2):
    """rrt.py:73-77."""
    dot = v1[0] * v2[0] + v1[1] * v2[1]
    det = v2[0] * v1[1] - v1[0] * v2[1]
    return _standardangle(math.degrees(math.atan2(det, dot)))


def draw_bicycle(bike_loc, theta, alpha, color='blue'):
    """rrt.py:16-40: body line, heading arrow, front wheel (alpha) and its normal."""
    plt = _plt()
    L = float(config.get("bikelength"))
    frame = _rot(theta, [L, 0])
    x, y = bike_loc[0], bike_loc[1]
    plt.plot([x, frame[0] + x], [y, frame[1] + y], color=color, linewidth=5)
    arrow = dict(edgecolor='black', linewidth=0.5, headwidth=2.5, zorder=10, angles='xy',
                 scale_units='xy', scale=1)
    plt.quiver(x, y, frame[0] / 2, frame[1] / 2, facecolor='red', **arrow)
    pivot = (frame[0] + x, frame[1] + y)
    for off, fc in ((0, 'yellow'), (90, 'cyan')):
        wheel = _rot(theta, _rot(alpha + off, [L / 2, 0]))
        plt.quiver(pivot[0], pivot[1], wheel[0], wheel[1], facecolor=fc, **arrow)


def draw_path_segment(bike1, bike2, u, colors=None, bikes=True):
    """rrt.py:224-270: the arc about the ICC (dashed, left/right coloured) or the straight
    segment, and the bicycle at bike1 steered by u[0]."""
    import matplotlib.patches as patches
    colors = colors or {"left": "magenta", "right": "dodgerblue", "straight": "red",
                        "bike": "dodgerblue"}
    icc = u[1]
    if icc is not None:
        rad = u[2]
        to2 = np.subtract(bike2[0], icc)
        to1 = np.subtract(bike1[0], icc)
        angle = _anglebetween([1, 0], to2)
        angle2 = _anglebetween([1, 0], to1)
        angle3 = _anglebetween(to2, to1)
        frame = _rot(bike1[1], [float(config.get("bikelength")), 0])
        pivot = np.add(frame, bike1[0])
        sv = _rot(90, np.subtract(pivot, icc))
        steerangle = _standardangle(-_anglebetween(frame, sv))
        flip = bool(config.get("FORWARDONLY")) and (steerangle > 90 or steerangle < -90)
        color = colors["right"] if u[0] < 0 else colors["left"]
        if u[0] < 0 or flip:
            arc = patches.Arc(icc, rad * 2, rad * 2, angle=-angle, theta1=0, theta2=-angle3,
                              edgecolor=color, linestyle='--', zorder=10)
        else:
            arc = patches.Arc(icc, rad * 2, rad * 2, angle=-angle2, theta1=0, theta2=angle3,
                              edgecolor=color, linestyle='--', zorder=10)
        _ax().add_patch(arc)
    else:
        _plt().plot([bike1[0][0], bike2[0][0]], [bike1[0][1], bike2[0][1]], linestyle='--',
                    color=colors["straight"])
    if bikes:
        draw_bicycle(bike1[0], bike1[1], u[0], color=colors["bike"])


def drawpath(solution, camefrom):
    """rrt.py:79-98: the branch from `solution` back to the root (cameFrom[root] is None)."""
    if solution is None or camefrom.get(solution) is None:
        return
    draw_bicycle(solution[0], solution[1], 0, color='green')
    a = solution
    b, u = camefrom[a]
    while b is not None:
        draw_path_segment(b, a, u)
        a = b
        if camefrom[b] is None:
            break
        b, u = camefrom[b]


def drawtree(begin, graph, camefrom):
    """rrt.py:100-106: every edge in light grey, a bicycle at every leaf."""
    grey = {"left": "lightgray", "right": "silver", "straight": "silver", "bike": "darkgray"}
    for parent in graph.keys():
        for child in graph[parent]:
            _, u = camefrom[child]
            draw_path_segment(parent, child, u, colors=grey, bikes=False)
        if not graph[parent]:
            draw_bicycle(parent[0], parent[1], 0, color='darkgray')


def search_drawpath(mainpath, bresenham):
    """search.py:206-219: the Bresenham pixels of an A*/Theta* path, coloured by order."""
    path = []
    for first, second in zip(mainpath, mainpath[1:]):
        path = path + list(bresenham(first, second))
    if path:
        print("Found path")
        _plt().scatter([p[0] for p in path], [p[1] for p in path], s=10, c=range(len(path)),
                       cmap="winter")
