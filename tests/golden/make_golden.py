"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only in the build container, where takuyani/SLAM-Robot_Simu is mounted
read-only at /root/reference.  The reference is imported (never copied); its
private methods are called through their name-mangled attributes and a few
global functions are wrapped to observe values the reference keeps internal.
Only data (inputs and outputs) is written.

    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/make_golden.py

One harness addition is unavoidable: particle_filter.py:191 calls
``matplotlib.mlab.bivariate_normal``, removed in matplotlib 3.1.  The published
formula is injected into ``matplotlib.mlab`` before the first step (nothing
under /root/reference is modified).
"""
import os
import sys
import contextlib
import io

import numpy as np

REF = os.environ.get("SLAM_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
os.environ.setdefault("MPLBACKEND", "Agg")
sys.path.insert(0, REF)

import matplotlib  # noqa: E402
from matplotlib import mlab  # noqa: E402


def _bivariate_normal(X, Y, sigmax=1.0, sigmay=1.0, mux=0.0, muy=0.0, sigmaxy=0.0):
    xm, ym = X - mux, Y - muy
    rho = sigmaxy / (sigmax * sigmay)
    q = xm ** 2 / sigmax ** 2 + ym ** 2 / sigmay ** 2 - 2 * rho * xm * ym / (sigmax * sigmay)
    den = 2 * np.pi * sigmax * sigmay * np.sqrt(1 - rho ** 2)
    return np.exp(-q / (2 * (1 - rho ** 2))) / den


mlab.bivariate_normal = _bivariate_normal


def _quiet():
    return contextlib.redirect_stdout(io.StringIO())


# --------------------------------------------------------------- primitives
def heavy_weights(rs, n, zero_frac=0.0):
    """Deterministic heavy-tailed positive weights built with multiplications
    only (bit-identical on every IEEE machine, so large inputs are stored as a
    seed instead of as data)."""
    u = rs.random_sample(n)
    v = rs.random_sample(n)
    w = u * u
    w = w * w
    w = w * w
    w = w * w * v            # ~u**16 * v : spans many decades
    if zero_frac > 0:
        w[rs.random_sample(n) < zero_frac] = 0.0
    return w


def gen_units():
    from mylib import limit, transform
    rs = np.random.RandomState(1234)
    ang = np.concatenate([
        np.array([0.0, -0.0, np.pi, -np.pi, 3 * np.pi, -3 * np.pi, np.pi + 1e-12,
                  -np.pi - 1e-12, 2 * np.pi, -2 * np.pi, 7.5, -7.5, 100.0, -100.0,
                  1e-300, -1e-300, np.nextafter(np.pi, 10), np.nextafter(-np.pi, -10)]),
        rs.uniform(-20, 20, 500)])
    wrapped = np.array([limit.limit_angle(a) for a in ang])

    poses = np.stack([rs.uniform(-20, 20, 64), rs.uniform(-20, 20, 64),
                      rs.uniform(-4, 4, 64)], axis=1)
    pts = rs.uniform(-15, 15, (64, 7, 2))
    w2r = np.stack([transform.world2robot(p.reshape(3, 1), q) for p, q in zip(poses, pts)])
    r2w = np.stack([transform.robot2world(p.reshape(3, 1), q) for p, q in zip(poses, pts)])

    dx = np.concatenate([rs.normal(size=300) * 0.5, rs.normal(size=100) * 30, [0.0, 40.0, 1e3]])
    dy = np.concatenate([rs.normal(size=300) * 0.5, rs.normal(size=100) * 30, [0.0, -40.0, 1e3]])
    gauss = _bivariate_normal(dx, dy, 0.3, 0.3, 0.0, 0.0, 0.0)

    sums = {}
    for n in [1, 7, 8, 100, 128, 129, 500, 1000, 8192, 8193, 20000, 100003, 1 << 20]:
        a = heavy_weights(np.random.RandomState(n), n)
        sums[n] = float(np.sum(a.reshape(1, n)))
    np.savez_compressed(
        os.path.join(OUT, "units.npz"),
        ang_in=ang, ang_out=wrapped, poses=poses, pts=pts, w2r=w2r, r2w=r2w,
        gdx=dx, gdy=dy, gauss=gauss,
        sum_sizes=np.array(list(sums)), sum_out=np.array([sums[n] for n in sums]))


# ------------------------------------------------------- particle filter
def _make_pf(pfm, n, lm):
    with _quiet():
        pf = pfm.ParticleFilter(100)
    pf._ParticleFilter__NP = n
    pf._ParticleFilter__NP_RECIP = 1 / n
    pf._ParticleFilter__ESS_TH = n / 100.0
    pf._ParticleFilter__LM = lm
    x0 = pf._ParticleFilter__x_true
    pf._ParticleFilter__px = np.tile(x0, (1, n))
    pf._ParticleFilter__pw_ini = np.full((1, n), 1 / n)
    pf._ParticleFilter__pw = np.full((1, n), 1 / n)
    return pf


class _RandRecorder:
    def __init__(self):
        self.real = np.random.rand
        self.last = None

    def __call__(self, *a):
        v = self.real(*a)
        self.last = v
        return v


def resample_tags(pfm, pf, pw, u, fn=None):
    """Indices chosen by the reference __resampling for weights pw and rand()=u.
    ``fn``: the unwrapped bound method when the instance attribute is wrapped."""
    fn = fn or pf._ParticleFilter__resampling
    n = pw.size
    tags = np.tile(np.arange(n, dtype=np.float64), (3, 1))
    saved, th = np.random.rand, pf._ParticleFilter__ESS_TH
    np.random.rand = lambda *a: u
    pf._ParticleFilter__ESS_TH = np.inf          # force the resampling branch
    try:
        px, _ = fn(tags, pw.reshape(1, n).copy())
    finally:
        np.random.rand = saved
        pf._ParticleFilter__ESS_TH = th
    return px[0].astype(np.int64)


def gen_pf_c1(seed=0, n=500, nl=20, steps=1000):
    """BASELINE config 1: 500 particles x 20 landmarks x 1000 steps, seed 0."""
    import particle_filter as pfm
    lm = np.random.RandomState(seed + 1).uniform(-10.0, 10.0, (nl, 2))
    np.random.seed(seed)
    pf = _make_pf(pfm, n, lm)
    rec = _RandRecorder()
    obs_log, res_log = [], []
    orig_obs = pf._ParticleFilter__observation
    orig_res = pf._ParticleFilter__resampling

    def obs_wrap(x):
        z = orig_obs(x)
        obs_log.append(z.copy())
        return z

    def res_wrap(px, pw):
        ess = float(np.reciprocal(pw @ pw.T)[0, 0])
        rec.last = None
        np.random.rand = rec
        try:
            px2, pw2 = orig_res(px, pw)
        finally:
            np.random.rand = rec.real
        res_log.append((ess, rec.last, pw.copy()))
        return px2, pw2

    pf._ParticleFilter__observation = obs_wrap
    pf._ParticleFilter__resampling = res_wrap
    keep = set(range(20)) | set(range(49, steps, 50))
    cols = {k: [] for k in ["x_true", "x_est", "max_idx", "max_val", "ess", "resampled", "u"]}
    px_keep, pw_keep, keep_steps = [], [], []
    idx_keep, idx_steps = [], []
    for k in range(steps):
        with _quiet():
            _, xt, xe, px, _, mi, mv = pf.main_pf()
        ess, u, pw_prev = res_log[-1]
        cols["x_true"].append(xt[:, 0].copy())
        cols["x_est"].append(xe[:, 0].copy())
        cols["max_idx"].append(int(mi))
        cols["max_val"].append(float(mv))
        cols["ess"].append(ess)
        cols["resampled"].append(u is not None)
        cols["u"].append(np.nan if u is None else float(u))
        if u is not None and len(idx_keep) < 12:
            idx_keep.append(resample_tags(pfm, pf, pw_prev[0], u, fn=orig_res))
            idx_steps.append(k)
        if k in keep:
            px_keep.append(px.copy())
            pw_keep.append(pf._ParticleFilter__pw[0].copy())
            keep_steps.append(k)
    np.savez_compressed(
        os.path.join(OUT, "pf_c1.npz"), seed=seed, n=n, lm=lm,
        z=np.array(obs_log), **{k: np.array(v) for k, v in cols.items()},
        px_keep=np.array(px_keep), pw_keep=np.array(pw_keep), keep_steps=np.array(keep_steps),
        idx_keep=np.array(idx_keep), idx_steps=np.array(idx_steps))


def gen_pf_stages(seed=7):
    """Kernel-level vectors: __likelihood / __resampling / __predict of the
    reference on synthetic particle sets (including underflowing weights)."""
    import particle_filter as pfm
    rs = np.random.RandomState(seed)
    out = {}
    for tag, n, nl, spread in [("a", 2000, 100, 0.6), ("b", 777, 20, 2.0), ("c", 4096, 5, 0.3)]:
        lm = rs.uniform(-10.0, 10.0, (nl, 2))
        pf = _make_pf(pfm, n, lm)
        px = np.vstack([10 + rs.normal(size=n) * spread, rs.normal(size=n) * spread,
                        np.pi / 2 + rs.normal(size=n) * spread * 0.3])
        pw = rs.random_sample(n)
        pw /= np.sum(pw)
        if tag == "b":       # inconsistent observations: every product underflows
            z = rs.uniform(-12, 12, (nl, 2))
        else:                # observations of a pose inside the cloud
            from mylib import transform
            z = transform.world2robot(np.array([[10.1], [-0.1], [np.pi / 2 + 0.05]]), lm)
            z = z + rs.normal(size=z.shape) * 0.3
        lik = pf._ParticleFilter__likelihood(px.copy(), pw.reshape(1, n).copy(), z)
        out.update({f"lik_{tag}_lm": lm, f"lik_{tag}_px": px, f"lik_{tag}_pw": pw,
                    f"lik_{tag}_z": z, f"lik_{tag}_out": lik[0]})
        # predict: reseed so the noise can be regenerated by the checker
        np.random.seed(seed + 100)
        pred = pf._ParticleFilter__predict(px.copy())
        out.update({f"pred_{tag}_in": px, f"pred_{tag}_out": pred,
                    f"pred_{tag}_seed": np.array(seed + 100)})
    # resampling index sets on concentrated / flat / zero-heavy weights
    for tag, n in [("r500", 500), ("r1000", 1000), ("r8193", 8193), ("r65536", 65536),
                   ("r1m", 1 << 20)]:
        pf = _make_pf(pfm, n, np.zeros((1, 2)))
        wseed = 1000 + n
        w = heavy_weights(np.random.RandomState(wseed), n,
                          zero_frac=0.5 if tag in ("r8193", "r1m") else 0.0)
        if tag in ("r8193", "r1m"):
            w[:64] = 0.0
        w = w / np.sum(w.reshape(1, n))
        u = float(rs.random_sample())
        idx = resample_tags(pfm, pf, w, u)
        # indices are monotone: store them run-length encoded (exact)
        vals, counts = np.unique(idx, return_counts=True)
        out.update({f"{tag}_wseed": np.array(wseed), f"{tag}_u": np.array(u),
                    f"{tag}_idx_vals": vals.astype(np.int32),
                    f"{tag}_idx_counts": counts.astype(np.int32)})
    np.savez_compressed(os.path.join(OUT, "pf_stages.npz"), **out)


# ------------------------------------------------------------ motion model
def gen_motion(seed=11):
    import motion_model as mm
    rs = np.random.RandomState(seed)
    poses = np.stack([rs.uniform(-10, 10, 300), rs.uniform(-10, 10, 300),
                      rs.uniform(-3, 3, 300)], axis=1)
    cases = [(1.0, 0.05, 0.05, 0.01, 0.01, 0.01, 0.01, np.pi / 2, np.deg2rad(90.0)),
             (0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 10 * np.deg2rad(10.0), np.deg2rad(10.0)),
             (2.0, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 10 * np.deg2rad(10.0), np.deg2rad(10.0))]
    out = {"poses": poses}
    for c, (dt, a1, a2, a3, a4, a5, a6, v, w) in enumerate(cases):
        m = mm.MotionModel(dt, a1, a2, a3, a4, a5, a6)
        np.random.seed(seed + c)
        noisy = np.stack([m.moveWithNoise(p.reshape(3, 1), v, w)[:, 0] for p in poses])
        clean = np.stack([m.moveWithoutNoise(p.reshape(3, 1), v, w)[:, 0] for p in poses])
        out.update({f"case{c}": np.array([dt, a1, a2, a3, a4, a5, a6, v, w]),
                    f"noisy{c}": noisy, f"clean{c}": clean, f"seed{c}": np.array(seed + c)})
    np.savez_compressed(os.path.join(OUT, "motion.npz"), **out)


# -------------------------------------------------------------------- EKF
def gen_ekf(seed=3, steps=360):
    import extended_kalman_filter as ekfm
    np.random.seed(seed)
    with _quiet():
        ekf = ekfm.ExtendedKalmanFilter(100)
    rows = {k: [] for k in ["x_true", "x_dr", "z", "x_hat_m", "P", "x_hat"]}
    for _ in range(steps):
        xt, xdr, z, xm, P = ekf.main_ekf()
        rows["x_true"].append(xt[:, 0].copy())
        rows["x_dr"].append(xdr[:, 0].copy())
        rows["z"].append(z[:, 0].copy())
        rows["x_hat_m"].append(xm[:, 0].copy())
        rows["P"].append(P.copy())
        rows["x_hat"].append(ekf._ExtendedKalmanFilter__x_hat[:, 0].copy())
    np.savez_compressed(os.path.join(OUT, "ekf.npz"), seed=seed,
                        **{k: np.array(v) for k, v in rows.items()})


# -------------------------------------------------------------- graph SLAM
def _pair_row(h1, h2):
    o1, o2 = h1.getObs(), h2.getObs()
    return [h1.getTime(), h1.getRobotPoseId(), o1.getLandMarkId(), o1.getDist(), o1.getDir(),
            o1.getOrient(), h2.getTime(), h2.getRobotPoseId(), o2.getLandMarkId(), o2.getDist(),
            o2.getDir(), o2.getOrient()]


def gen_graph(seed=0, demo_frames=18, big_steps=300):
    """graph_based_slam.py: the 18-frame demo (module-level robot, every
    Gauss-Newton iteration) and a T=300 run paired once at the end.  The
    reference's setPairObs / updateEstPose are wrapped to record their inputs
    (half-edge pairs, pose estimates) and outputs (edge blocks, H, b, det,
    cond, updated poses)."""
    np.random.seed(seed)                         # the module draws at import
    with _quiet():
        import graph_based_slam as gs
    TE = gs.TrajectoryEstimator
    orig_pair, orig_upd = TE.setPairObs, TE.updateEstPose
    log, cur = [], {"pairs": []}

    def pair(self, h1, h2):
        cur["pairs"].append(_pair_row(h1, h2))
        return orig_pair(self, h1, h2)

    def upd(self):
        poses_b = np.array([p[:, 0] for p in self._TrajectoryEstimator__mPosesEst])
        edges = [np.concatenate([e.mMatH_BfrBfr.ravel(), e.mMatH_BfrAft.ravel(),
                                 e.mMatH_AftBfr.ravel(), e.mMatH_AftAft.ravel(),
                                 e.mVecB_Bfr.ravel(), e.mVecB_Aft.ravel()])
                 for e in self._TrajectoryEstimator__mEdge]
        times = sorted(self._TrajectoryEstimator__KeepLandMarkTime)
        r = orig_upd(self)
        rec = dict(pairs=np.array(cur["pairs"], dtype=np.float64).reshape(-1, 12),
                   poses_before=poses_b, edges=np.array(edges).reshape(-1, 42),
                   times=np.array(times, dtype=np.int64),
                   H=self._TrajectoryEstimator__mMatH.copy(),
                   b=self._TrajectoryEstimator__mVecB[:, 0].copy(),
                   stats=np.array([float(r[0]), r[1], r[2], r[3]]),
                   poses_after=np.array([p[:, 0] for p in self._TrajectoryEstimator__mPosesEst]))
        log.append(rec)
        cur["pairs"] = []
        return r

    TE.setPairObs, TE.updateEstPose = pair, upd
    try:
        out = {"seed": np.array(seed)}
        with _quiet():
            for _ in range(demo_frames):
                gs.gRbt.move(gs.VEL_mps, gs.OMEGA_rps)
                gs.gRbt.estimateOpticalTrajectory()
        demo = list(log)
        out["demo_n"] = np.array(len(demo))
        for i, r in enumerate(demo):
            for k, v in r.items():
                out[f"demo{i}_{k}"] = v
        # T = 300: one robot, all moves first, then one trajectory estimate
        log.clear()
        x0 = np.array([[10.0], [0.0], [np.deg2rad(90.0)]])
        with _quiet():
            rbt = gs.Robot(x0, gs.PERIOD_ms / 1000, gs.SCN_SENS_RANGE_m, gs.SCN_SENS_ANGLE_rps,
                           gs.LAND_MARKS)
            for _ in range(big_steps):
                rbt.move(gs.VEL_mps, gs.OMEGA_rps)
            halves = [[h.getTime(), h.getRobotPoseId(), h.getObs().getLandMarkId(),
                       h.getObs().getDist(), h.getObs().getDir(), h.getObs().getOrient()]
                      for h in rbt._Robot__mHalfEdges]
            rbt.estimateOpticalTrajectory()
        out["big_halves"] = np.array(halves)
        out["big_n"] = np.array(len(log))
        for i, r in enumerate(log):
            out[f"big{i}_poses_before"] = r["poses_before"]
            out[f"big{i}_poses_after"] = r["poses_after"]
            out[f"big{i}_times"] = r["times"]
            out[f"big{i}_b"] = r["b"]
            out[f"big{i}_stats"] = r["stats"]
            out[f"big{i}_n_edges"] = np.array(len(r["edges"]))
            out[f"big{i}_edges_head"] = r["edges"][:64]
            out[f"big{i}_edges_colsum"] = r["edges"].sum(axis=0)
            H = r["H"]
            out[f"big{i}_H_diag3"] = np.array([H[j:j + 3, j:j + 3] for j in range(0, len(H), 3)])
            out[f"big{i}_H_colsum"] = H.sum(axis=0)
            out[f"big{i}_H_sample"] = H[::7, ::11]
    finally:
        TE.setPairObs, TE.updateEstPose = orig_pair, orig_upd
    np.savez_compressed(os.path.join(OUT, "graph.npz"), **out)


# ------------------------------------------------------- error ellipse
def gen_ellipse(seed=5):
    """mylib/error_ellipse.py: chi-squared lookup at table knots, between
    knots and at the ends; ellipse parameters of random and degenerate 2x2
    covariances; calc_chi."""
    from mylib import error_ellipse
    rs = np.random.RandomState(seed)
    ps = np.concatenate([[99.0, 99.9, 0.0, 50.0, 95.0, 2.5, 97.3, 12.34, 0.25, 99.95 - 0.05],
                         rs.uniform(0.0, 99.9, 40)])
    chi = np.array([float(error_ellipse.ErrorEllipse(p)._ErrorEllipse__chi) for p in ps])
    A = rs.normal(size=(200, 2, 2)) * rs.uniform(0.01, 10.0, (200, 1, 1))
    covs = A @ A.transpose(0, 2, 1)
    extra = np.array([[[16.0, 5.48], [5.48, 9.0]], [[1.0, 0.0], [0.0, 1.0]],
                      [[2.0, 0.0], [0.0, 1.0]], [[1.0, 0.0], [0.0, 2.0]],
                      [[1.0, -0.9], [-0.9, 1.0]], [[1e-8, 0.0], [0.0, 1e4]],
                      [[3.0, 3.0], [3.0, 3.0]], [[0.0, 0.0], [0.0, 0.0]]])
    covs = np.concatenate([extra, covs])
    ee = error_ellipse.ErrorEllipse(99.0)
    out = np.array([ee.calc_error_ellipse(c) for c in covs], dtype=np.float64)
    ee95 = error_ellipse.ErrorEllipse(95.0)
    out95 = np.array([ee95.calc_error_ellipse(c) for c in covs], dtype=np.float64)
    chi_l = np.array([ee.calc_chi(p, c) for p, c in zip(ps, covs)])
    np.savez_compressed(os.path.join(OUT, "ellipse.npz"), ps=ps, chi=chi, covs=covs,
                        out99=out, out95=out95, chi_l=chi_l)


# ------------------------------------------------------------- scan sensor
def gen_scan(seed=13, n_poses=40, n_lm=300):
    """graph_based_slam.py:78-172 ScanSensor.scan: random poses among random
    landmarks (the demo's 15 m / +-80 deg fan and noise setting, :899-902 /
    :604), one scan per pose from a seeded global stream; per pose the
    detected ids and the noise-free and noisy (dist, dir, orient)."""
    np.random.seed(seed)                         # the module draws at import
    with _quiet():
        import graph_based_slam as gs
    rs = np.random.RandomState(seed)
    lm = rs.uniform(-20.0, 20.0, (n_lm, 2))
    poses = np.column_stack([rs.uniform(-10, 10, n_poses), rs.uniform(-10, 10, n_poses),
                             rs.uniform(-np.pi, np.pi, n_poses)])
    sensor = gs.ScanSensor(15.0, np.deg2rad(80.0), lm)
    sensor.setNoiseParam(5, 2, 2)
    np.random.seed(seed + 1)
    ids, clean, noisy, npp = [], [], [], []
    for p in poses:
        wn, wo = sensor.scan(p.reshape(3, 1))
        npp.append(len(wn))
        for a, b in zip(wn, wo):
            ids.append(a.getLandMarkId())
            noisy.append([a.getDist(), a.getDir(), a.getOrient()])
            clean.append([b.getDist(), b.getDir(), b.getOrient()])
    np.savez_compressed(os.path.join(OUT, "scan.npz"), seed=seed, lm=lm, poses=poses,
                        n_per_pose=np.array(npp), ids=np.array(ids, dtype=np.int64),
                        clean=np.array(clean).reshape(-1, 3), noisy=np.array(noisy).reshape(-1, 3))


if __name__ == "__main__":
    which = sys.argv[1:] or ["units", "pf_c1", "pf_stages", "motion", "ekf", "graph", "ellipse",
                             "scan"]
    for w in which:
        print("generating", w, flush=True)
        globals()["gen_" + w]()
