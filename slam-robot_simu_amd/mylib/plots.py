"""Drawing helpers shared by the animation front-ends (particle_filter.animate,
extended_kalman_filter.animate, graph_based_slam.Robot.draw).

The reference draws the same few primitives in each of its demos
(particle_filter.py:248-327, extended_kalman_filter.py:219-274,
graph_based_slam.py:717-897): a trajectory line with the current point, a
heading stroke, the landmark stars, robot-to-landmark sight lines and error
ellipses.  They are collected here so every front-end renders them the same
way.  Nothing here computes estimates: the front-ends draw what the GPU
filters return.
"""
from __future__ import annotations

import numpy as np
from matplotlib import patches


def trajectory(ax, history, color, label=None, marker=True):
    """Polyline through a list of (3,1)/(2,1) poses, the last one marked."""
    if not len(history):
        return None
    xy = np.array([[p[0, 0], p[1, 0]] for p in history])
    (line,) = ax.plot(xy[:, 0], xy[:, 1], c=color, linewidth=1.0, linestyle="-", label=label)
    if marker:
        ax.scatter(xy[-1, 0], xy[-1, 1], c=color, marker="o", alpha=0.5)
    return line


def headings(ax, xs, ys, yaws, color, arrow=False, gain=1.0):
    """Heading of each pose: a headless stroke (PF / EKF demos) or an arrow
    in data units (graph SLAM demo)."""
    u, v = gain * np.cos(yaws), gain * np.sin(yaws)
    if arrow:
        return ax.quiver(xs, ys, u, v, color=color, angles="xy", scale_units="xy", scale=1)
    return ax.quiver(xs, ys, u, v, color=color, units="inches", scale=6.0, width=0.01,
                     headwidth=0.0, headlength=0.0, headaxislength=0.0)


def landmark_stars(ax, xs, ys, face="yellow", edge="orange", label=None):
    return ax.scatter(xs, ys, s=100, c=face, marker="*", alpha=0.5, linewidths=2,
                      edgecolors=edge, label=label)


def sight_lines(ax, origin_xy, targets_xy, color="green"):
    for tx, ty in targets_xy:
        ax.plot([origin_xy[0], tx], [origin_xy[1], ty], "--", c=color)


def error_ellipse(ax, center, ellipse, cov2, label=""):
    """The ErrorEllipse's axes / angle of a 2x2 covariance, as a patch."""
    w, h, ang = ellipse.calc_error_ellipse(cov2)
    e = patches.Ellipse(center, w, h, angle=np.rad2deg(ang), linewidth=2, alpha=0.2,
                        facecolor="yellow", edgecolor="black", label=label)
    ax.add_patch(e)
    return e


def finish(ax, title, legend=True):
    ax.set_xlabel("x [m]")
    ax.set_ylabel("y [m]")
    ax.set_title(title)
    ax.grid()
    if legend:
        ax.legend(fontsize=10)
