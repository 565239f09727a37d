"""Drop-in ParticleFilter backed by the MI355X kernels (libslam_hip.so).

Same constructor and ``main_pf()`` contract as the reference
(particle_filter.py:21 / :86-119), plus ``step(control, observations)`` that
returns the estimate and the weighted particle covariance.  The estimator
(resample -> predict -> likelihood -> normalise -> argmax) runs on the GPU;
this module only simulates the ground truth and the landmark observation, as
the reference does on its side of main_pf (:100, :110).

Noise streams
  noise="numpy" (default): the host draws from NumPy's global RNG in the
      reference's order -- [rand() if resampling] -> mvn(0, Q, NP) ->
      observation noise -- so a seeded run reproduces the reference's
      trajectory (tests/test_gpu_pf.py).
  noise="mt19937": the same NumPy stream, drawn on the GPU: the device holds
      np.random's MT19937 state and draws rand() / mvn(0, Q, NP) / mvn(0, R,
      NL) itself, observing the landmarks from the true pose there; only the
      2.5 KB state crosses the boundary (taken from np.random before a step
      when the host changed it, handed back after), so the global stream
      continues exactly as the reference's would.
  noise="device": Philox-4x32-10 on the GPU (no per-step host->device
      noise traffic); statistically equivalent, not stream-identical.
"""
from __future__ import annotations

import numpy as np

from mylib import limit
from mylib import transform as tf
from slamhip.pf import DeviceParticleFilter

DEFAULT_LANDMARKS = np.array([[5.0, 5.0], [2.0, -3.0], [-3.0, 4.0], [-5.0, -1.0], [0.0, 0.0]])


class ParticleFilter(object):
    """Monte-Carlo localisation against a known landmark map (GPU)."""

    def __init__(self, period_ms, *, n_particles=1000, landmarks=None, noise="numpy",
                 motion="linear", likelihood="product", alphas=(0.1,) * 6, seed=0, device=0):
        self.period_ms = period_ms
        self.dt = period_ms / 1000                                 # :30
        self.n_particles = int(n_particles)                        # :31
        self.lm = DEFAULT_LANDMARKS.copy() if landmarks is None else np.asarray(landmarks, float)
        self.radius = 10.0                                         # :46
        self.yaw_rate = np.deg2rad(10.0)                           # :47
        self.vel = self.radius * self.yaw_rate                     # :48
        self.Q = np.diag([0.03, 0.03, np.deg2rad(2.0)]) ** 2        # :62-65
        self.R = np.diag([0.3, 0.3]) ** 2                          # :68-70
        self.x_true = np.array([[self.radius], [0.0], [np.deg2rad(90.0)]])   # :74-79
        if noise not in ("numpy", "mt19937", "device"):
            raise ValueError("noise must be 'numpy', 'mt19937' or 'device'")
        self.noise = noise
        self.motion = motion
        self.alphas = tuple(alphas)
        self.dev = DeviceParticleFilter(
            self.n_particles, self.lm, dt=self.dt, q=self.Q, r=self.R, x0=self.x_true[:, 0],
            motion=motion, likelihood=likelihood, alphas=alphas, seed=seed, device=device)
        self._rng_seen = None

    # ------------------------------------------------------------- world
    def _truth_step(self, x):
        """Ground-truth motion: particle_filter.py:121-142 for one column
        (linear model) or motion_model.py:64-86 (velocity model)."""
        yaw = x[2, 0]
        if self.motion == "linear":
            a = self.dt * np.cos(yaw)
            b = self.dt * np.sin(yaw)
            return np.array([[x[0, 0] + self.vel * a], [x[1, 0] + self.vel * b],
                             [limit.limit_angle(yaw + self.yaw_rate * self.dt)]])
        r = self.vel / self.yaw_rate
        turn = limit.limit_angle(self.yaw_rate * self.dt)
        yaw2 = limit.limit_angle(yaw + turn)
        return np.array([[x[0, 0] + r * (-np.sin(yaw) + np.sin(yaw2))],
                         [x[1, 0] + r * (np.cos(yaw) - np.cos(yaw2))], [yaw2]])

    def _observe(self, x_true):
        """particle_filter.py:144-154: landmarks in the robot frame + N(0, R)."""
        z = tf.world2robot(x_true, self.lm)
        return z + np.random.multivariate_normal([0.0, 0.0], self.R, z.shape[0])

    def _draw_noise(self):
        n = self.n_particles
        if self.motion == "linear":
            return np.random.multivariate_normal([0.0, 0.0, 0.0], self.Q, n)   # :165
        return np.random.standard_normal(3 * n).reshape(n, 3)                 # motion_model.py:46-48

    # --------------------------------------------------------- interface
    def step(self, control, observations, noise=None, u_resample=float("nan")):
        """One estimator step -> (pose (3,1), covariance (3,3))."""
        out = self.dev.step(control, observations, noise, u_resample)
        return out["x_est"].reshape(3, 1), out["cov"]

    def _rng_to_device(self):
        """np.random's state -> the device stream, unless it is the one the
        device handed back last step (nothing drew from np.random since)."""
        cur = np.random.get_state()
        seen = self._rng_seen
        if (seen is None or cur[2:] != seen[2:] or not np.array_equal(cur[1], seen[1])):
            self.dev.use_numpy_stream(cur)

    def _rng_from_device(self):
        st = self.dev.rng_state()
        np.random.set_state(st)
        self._rng_seen = st

    def main_pf(self):
        """particle_filter.py:86-119 -> (LM, x_true, x_est, px, Q, max_idx, max_val)."""
        self.x_true = self._truth_step(self.x_true)
        if self.noise == "mt19937":
            self._rng_to_device()
            out = self.dev.step_truth((self.vel, self.yaw_rate), self.x_true)
            self._rng_from_device()
            x, y, th, _ = self.dev.get_state()
            return (self.lm, self.x_true, out["x_est"].reshape(3, 1), np.vstack([x, y, th]),
                    self.Q, out["max_idx"], out["max_val"])
        if self.noise == "numpy":
            u = np.random.rand() if self.dev.resample_next else float("nan")
            noise = self._draw_noise()
        else:
            u, noise = float("nan"), None
        z = self._observe(self.x_true)
        out = self.dev.step((self.vel, self.yaw_rate), z, noise, u)
        x, y, th, _ = self.dev.get_state()
        px = np.vstack([x, y, th])
        return (self.lm, self.x_true, out["x_est"].reshape(3, 1), px, self.Q,
                out["max_idx"], out["max_val"])

    @property
    def weights(self):
        return self.dev.get_state()[3]


# ---------------------------------------------------------------- animation
class PFAnimation:
    """The reference's demo frame (particle_filter.py:248-327) over this
    filter: landmarks with sight lines from the estimate, the particle cloud
    with headings, true and estimated tracks, the maximum-likelihood label,
    and a zoom panel sized by the chi-square radius of Q."""

    def __init__(self, pf, period_ms, confidence=99.0):
        from mylib.error_ellipse import ErrorEllipse
        self.pf = pf
        self.period_ms = period_ms
        self.confidence = confidence
        self.ellipse = ErrorEllipse(confidence)
        self.truth, self.est = [], []
        self.time_s = 0.0

    def __call__(self, i):
        import matplotlib.pyplot as plt
        from mylib import plots
        self.time_s += self.period_ms / 1000
        lm, x_true, x_est, px, Q, w_idx, w_val = self.pf.main_pf()
        self.truth.append(x_true[0:2, :].copy())
        self.est.append(x_est[0:2, :].copy())
        plt.cla()
        axes = (plt.subplot2grid((1, 2), (0, 0)), plt.subplot2grid((1, 2), (0, 1)))
        for k, ax in enumerate(axes):
            plots.landmark_stars(ax, lm[:, 0], lm[:, 1], label="Land Mark" if k == 0 else None)
            plots.sight_lines(ax, x_est[0:2, 0], lm)
            ax.scatter(px[0], px[1], c="cyan", marker="o", alpha=0.5)
            plots.trajectory(ax, self.truth, "red", "Ground Truth" if k == 0 else None)
            plots.trajectory(ax, self.est, "blue", "Estimation" if k == 0 else None)
        zoom = axes[1]
        plots.headings(zoom, px[0], px[1], px[2], "cyan")
        plots.headings(zoom, x_true[0], x_true[1], x_true[2], "red")
        plots.headings(zoom, x_est[0], x_est[1], x_est[2], "blue")
        zoom.annotate("Maximuim Likelihood Estimate:\n[Index]:{0}\n[Weight]:{1:.3f}".format(w_idx, w_val),
                      xy=(x_est[0, 0], x_est[1, 0]), xycoords="data", xytext=(0.55, 0.9),
                      textcoords="axes fraction",
                      bbox=dict(boxstyle="round,pad=0.5", fc=(1.0, 0.7, 0.7)),
                      arrowprops=dict(arrowstyle="->", color="black", connectionstyle="arc3,rad=0"))
        axes[0].set_aspect("equal", adjustable="datalim")
        plots.finish(axes[0], "Localization by PF")
        half = self.ellipse.calc_chi(self.confidence, Q[0:2, 0:2]) * 3
        zoom.set_xlim(x_true[0][0] - half, x_true[0][0] + half)
        zoom.set_ylim(x_true[1][0] - half, x_true[1][0] + half)
        plots.finish(zoom, "Zoom")
        print("time:{0:.3f}[s]".format(self.time_s))
        return axes


_animations = {}


def animate(i, pf, period_ms):
    """FuncAnimation callback with the reference's signature (:248)."""
    key = id(pf)
    if key not in _animations:
        _animations[key] = PFAnimation(pf, period_ms)
    return _animations[key](i)


if __name__ == "__main__":
    import matplotlib.animation as animation
    import matplotlib.pyplot as plt

    period_ms = 100
    frame_cnt = int(36 * 1000 / period_ms)
    fig = plt.figure(figsize=(18, 9))
    pf = ParticleFilter(period_ms)
    ani = animation.FuncAnimation(fig, animate, frames=frame_cnt, fargs=(pf, period_ms), blit=False,
                                  interval=period_ms, repeat=False)
    plt.show()
