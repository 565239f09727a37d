"""The reference's callers on top of the GPU estimators (SURVEY 8(f)4 and the
graph driver, graph_based_slam.py:584-975): the Robot drop-in reproduces the
reference's 18-frame demo (tests/golden/graph.npz, recorded from the
reference's own Robot under seed 0), and the animation callbacks of the three
demos render headless frames of what the filters return.

Robot tolerance: every frame re-linearises at the poses the previous frames
produced, so the per-iteration differences of test_gpu_graph (H^-1's
conditioning x 1e-16 relative to the step) accumulate over the frames; the
bar is 1e-10 m / rad on every pose after every frame (measured: 3.9e-14),
with the same gate decisions (is_calc) and iteration counts as the
reference.
"""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _agg():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    yield
    plt.close("all")


def _frames(g):
    """log entries per frame: a frame's updateEstPose calls all see the same
    number of poses (the initial pose + one per move)."""
    out = {}
    for i in range(int(g["demo_n"])):
        out.setdefault(g[f"demo{i}_poses_before"].shape[0], []).append(i)
    return [out[k] for k in sorted(out)]


def test_robot_demo_matches_reference():
    import matplotlib.pyplot as plt
    import graph_based_slam as gs
    g = golden("graph")
    np.random.seed(int(g["seed"]))                    # the reference seeds, then builds its robot
    rbt = gs.make_demo_robot()
    frames = _frames(g)
    worst = 0.0
    for f, entries in enumerate(frames):
        rbt.move(gs.VEL_mps, gs.OMEGA_rps)
        st = rbt.estimateOpticalTrajectory()
        assert len(st) == len(entries), (f, len(st), len(entries))
        for row, i in zip(st, entries):
            assert bool(row[0]) == bool(g[f"demo{i}_stats"][0]), (f, i)
        est = np.array([p[:, 0] for p in rbt._est._poses])
        ref = g[f"demo{entries[-1]}_poses_after"]
        assert est.shape == ref.shape
        err = np.abs(est - ref).max()
        worst = max(worst, err)
        assert err <= 1e-10, (f, err)
        if f % 6 == 5:                                 # the frame draws (headless)
            fig = plt.figure(figsize=(12, 6))
            ax1, ax2 = fig.add_subplot(1, 2, 1), fig.add_subplot(1, 2, 2)
            rbt.draw(ax1, ax2)
            fig.canvas.draw()
            plt.close(fig)
    print(f"robot demo: {len(frames)} frames, worst pose difference {worst:.3g}")


def test_graph_demo_callback():
    import matplotlib.pyplot as plt
    import graph_based_slam as gs
    np.random.seed(0)
    gs.gRbt, gs.time_s = None, 0.0
    fig = plt.figure(figsize=(12, 6))
    for i in range(3):
        ax1, ax2 = gs.graph_based_slam(i, gs.PERIOD_ms)
    fig.canvas.draw()
    assert gs.gRbt.loop_cnt >= 1 and len(gs.gRbt.getActualPoses()) == 4
    assert ax1.get_title() == "World System" and ax2.get_title() == "Robot System"
    gs.gRbt = None


def test_pf_animation_frames():
    import matplotlib.pyplot as plt
    from particle_filter import PFAnimation, ParticleFilter
    np.random.seed(1)
    pf = ParticleFilter(100, n_particles=2000)
    anim = PFAnimation(pf, 100)
    fig = plt.figure(figsize=(12, 6))
    for i in range(4):
        axes = anim(i)
    fig.canvas.draw()
    line = [ln for ln in axes[0].get_lines() if ln.get_label() == "Estimation"][0]
    np.testing.assert_array_equal(line.get_xdata(), [p[0, 0] for p in anim.est])
    np.testing.assert_array_equal(line.get_ydata(), [p[1, 0] for p in anim.est])
    assert len(anim.truth) == 4


def test_ekf_animation_frames():
    import matplotlib.pyplot as plt
    from extended_kalman_filter import EKFAnimation, ExtendedKalmanFilter
    np.random.seed(2)
    ekf = ExtendedKalmanFilter(100)
    anim = EKFAnimation(ekf, 100)
    fig = plt.figure(figsize=(8, 6))
    for i in range(4):
        (ax,) = anim(i)
    fig.canvas.draw()
    line = [ln for ln in ax.get_lines() if ln.get_label() == "Predicted"][0]
    np.testing.assert_array_equal(line.get_ydata(), [p[1, 0] for p in anim.pred])
    assert len(ax.patches) == 1                        # the error ellipse of P
