"""Drop-in TrajectoryEstimator backed by the MI355X kernels (libslam_hip.so).

Same surface as the reference's estimator (graph_based_slam.py:330-514):
``TrajectoryEstimator(aPose)`` with ``addPose``, ``setPairObs``,
``updateEstPose`` and ``getEstTrajPose``, plus the Observation / HalfEdge
records its callers build (:20-75, :259-300).  ``setPairObs`` only records the
ordered pair; ``updateEstPose`` linearises every pair at the current pose
estimates, assembles H and b, applies the reference's gate and solves on the
GPU (csrc/graph_kernels.inl), then writes the updated poses back into the
caller's (3,1) arrays in place -- the reference mutates them in place too
(:499-502), and its Robot relies on that aliasing.

``ScanSensor`` (:78-213) is the sensor simulator: ``scan(pose)`` (and
``scan_batch(poses)`` for many poses at once) computes the noise-free
observations and the field-of-view test of every landmark on the GPU
(csrc/sensor_api.hip) and adds the reference's noise from NumPy's global
stream in the reference's draw order.

``estimate_trajectory(halves, n_landmarks)`` is Robot.estimateOpticalTrajectory
(:685-715): all 2-combinations of each landmark's half-edges, then
Gauss-Newton until sum(delta^2) < 0.01, with the poses resident on the GPU
between iterations.

``Robot`` (:584-897) is the reference's driver: ``move(v, w)`` (motion with
and without noise through the MotionModel drop-in, a scan of the noisy pose,
the odometry pose handed to the estimator), ``estimateOpticalTrajectory()``
and ``draw(ax1, ax2)``; ``graph_based_slam(i, period_ms)`` is the demo's
animation callback (:931-975) with the demo's constants (:899-925).
"""
from __future__ import annotations


import ctypes as C
from copy import deepcopy

import numpy as np

from slamhip import _lib
from slamhip._lib import check, dptr
from slamhip.graph import DeviceGraph, edge_array, pair_halves

BASE_ANG = np.pi / 2.0       # mylib/transform.py:12

DELTA_SUM_TH = 0.01          # graph_based_slam.py:662


class Observation:
    """graph_based_slam.py:20-75."""

    def __init__(self, aLandMarkId, aDist_m, aDir_rad, aOrient_rad):
        self._id, self._d, self._dir, self._or = aLandMarkId, aDist_m, aDir_rad, aOrient_rad

    def getLandMarkId(self):
        return self._id

    def getDist(self):
        return self._d

    def getDir(self):
        return self._dir

    def getOrient(self):
        return self._or


class ScanSensor(object):
    """graph_based_slam.py:78-213: a fan-shaped scan sensor.  The noise
    parameters are class-wide, as in the reference (setNoiseParam writes the
    class attributes)."""

    _R_Dist = 10 / 100                      # :85-87 defaults
    _R_DirSigma = np.deg2rad(3.0)
    _R_OrientSigma = np.deg2rad(3.0)

    def __init__(self, aRange_m, aAngle_rad, aLandMarks, device=0):
        self._range = aRange_m
        self._angle = aAngle_rad
        self._resl = int(np.rad2deg(aAngle_rad))
        self._lm = np.ascontiguousarray(aLandMarks, dtype=np.float64).reshape(-1, 2)
        self._device = int(device)
        self._tan = float(np.tan(BASE_ANG - aAngle_rad))          # :154
        ang = np.rad2deg(aAngle_rad)                               # :99-112 (the drawn fan)
        ofs = np.rad2deg(BASE_ANG)
        xs = np.arange(-ang + ofs, ang + ofs + 1.0, 1.0)
        p0 = [aRange_m * np.cos(np.deg2rad(x)) for x in xs] + [0.0]
        p1 = [aRange_m * np.sin(np.deg2rad(x)) for x in xs] + [0.0]
        p0.append(p0[0])
        p1.append(p1[0])
        self.local = np.array([p0, p1])

    def setNoiseParam(self, aDist, aDirSigma, aOrientSigma):
        """:115-126 (percent, degrees, degrees)."""
        ScanSensor._R_Dist = aDist / 100
        ScanSensor._R_DirSigma = np.deg2rad(aDirSigma)
        ScanSensor._R_OrientSigma = np.deg2rad(aOrientSigma)

    def _detect(self, poses):
        poses = np.ascontiguousarray(poses, dtype=np.float64).reshape(-1, 3)
        yaw = BASE_ANG - poses[:, 2]                               # transform.py:31, :152
        cs = np.ascontiguousarray(np.column_stack([np.cos(yaw), np.sin(yaw), yaw]))
        P, L = len(poses), len(self._lm)
        det = np.zeros((P, L), dtype=np.int32)
        obs = np.zeros((P, L, 3))
        lib = _lib.load()
        check(lib.slam_scan_detect(P, dptr(poses), dptr(cs), L, dptr(self._lm), float(self._range),
                                   self._tan, det.ctypes.data_as(C.POINTER(C.c_int32)), dptr(obs),
                                   self._device), "slam_scan_detect")
        return det.astype(bool), obs

    def _noisy(self, clean):
        """:163-165 for the detected observations, in order: three draws each."""
        n = len(clean)
        if np.any(clean[:, 0] * ScanSensor._R_Dist < 0) or ScanSensor._R_DirSigma < 0 or \
                ScanSensor._R_OrientSigma < 0:
            raise ValueError("scale < 0")                          # np.random.normal's check
        g = np.random.standard_normal(3 * n)                       # = 3n np.random.normal calls
        out = np.zeros((n, 3))
        if n:
            clean = np.ascontiguousarray(clean)
            check(_lib.load().slam_scan_noise(n, dptr(clean), dptr(g), float(ScanSensor._R_Dist),
                                              float(ScanSensor._R_DirSigma),
                                              float(ScanSensor._R_OrientSigma), dptr(out),
                                              self._device), "slam_scan_noise")
        return out

    def scan(self, aRobotPose):
        """:128-172: (obsWithNoise, obsWithoutNoise), lists of Observation."""
        return self.scan_batch(np.asarray(aRobotPose, dtype=np.float64).reshape(1, 3))[0]

    def scan_batch(self, poses):
        """scan() of every pose in order (the noise stream as consecutive calls)."""
        det, obs = self._detect(poses)
        p_idx, l_idx = np.nonzero(det)                             # pose-major, landmark order
        clean = obs[p_idx, l_idx]
        noisy = self._noisy(clean)
        out = [([], []) for _ in range(len(det))]
        for k, (p, i) in enumerate(zip(p_idx, l_idx)):
            out[p][0].append(Observation(int(i), noisy[k, 0], noisy[k, 1], noisy[k, 2]))
            out[p][1].append(Observation(int(i), clean[k, 0], clean[k, 1], clean[k, 2]))
        return out

    @classmethod
    def getLandMarkCovMatrixOnMeasurementSys(cls, aLandMarkDist):
        """:176-194."""
        dist = aLandMarkDist * ScanSensor._R_Dist
        dir_cov = (aLandMarkDist * np.sin(ScanSensor._R_DirSigma)) ** 2
        orient_cov = ScanSensor._R_DirSigma ** 2 + ScanSensor._R_OrientSigma ** 2
        return np.array([[dist ** 2, 0, 0], [0, dir_cov, 0], [0, 0, orient_cov]])

    @classmethod
    def tfMeasurement2World(cls, aCovMat, aLandMarkDir, aRobotDir):
        """:196-213."""
        ang = aLandMarkDir + aRobotDir - BASE_ANG
        c = np.cos(ang)
        s = np.sin(ang)
        rot = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])
        return rot @ aCovMat @ rot.T

    def tfMeasurement2Robot(self, aCovMat, aLandMarkDir):
        """:218-234: the measurement covariance in the robot frame."""
        c = np.cos(aLandMarkDir)
        s = np.sin(aLandMarkDir)
        rot = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])
        return rot @ aCovMat @ rot.T

    def draw(self, aAx, aColor, aPose):
        """:236-250: the scan fan at aPose and the true landmarks."""
        from mylib import plots
        from mylib import transform as tf
        world = tf.robot2world(aPose, self.local.T)
        aAx.plot(world.T[0], world.T[1], c=aColor, linewidth=1.0, linestyle="-")
        plots.landmark_stars(aAx, self._lm[:, 0], self._lm[:, 1], label="Land Mark(True)")

    def getLandMarkNum(self):
        """:252-259."""
        return len(self._lm)


class HalfEdge:
    """graph_based_slam.py:259-300."""

    def __init__(self, aTime, aObs, aRobotPoseId):
        self._t, self._obs, self._pid = aTime, aObs, aRobotPoseId

    def getTime(self):
        return self._t

    def getObs(self):
        return self._obs

    def getRobotPoseId(self):
        return self._pid


def _row(h_bfr, h_aft):
    ob, oa = h_bfr.getObs(), h_aft.getObs()
    return [h_bfr.getTime(), h_bfr.getRobotPoseId(), ob.getDist(), ob.getDir(), ob.getOrient(),
            h_aft.getTime(), h_aft.getRobotPoseId(), oa.getDist(), oa.getDir(), oa.getOrient()]


def _rec_row(r):
    """slam_graph_edge record -> setPairObs row (the form _row builds)."""
    return [int(r["time_bfr"]), int(r["pose_bfr"]), *r["obs_bfr"].tolist(),
            int(r["time_aft"]), int(r["pose_aft"]), *r["obs_aft"].tolist()]


class TrajectoryEstimator(object):
    """Pose-graph estimator (GPU linearise / assemble / solve)."""

    def __init__(self, aPose, *, solver="auto", device=0):
        self._poses = [aPose]
        self._is_obs = [True]
        self._rows = []
        self._lm_ids = []
        self._times = []
        self._device = device
        self._dev = DeviceGraph(solver=solver, device=device)

    def addPose(self, aPose, aIsObs):
        self._poses.append(aPose)
        self._is_obs.append(aIsObs)

    def setPairObs(self, aHalfEdge1, aHalfEdge2):
        """:362-439 (the blocks are formed on the device at updateEstPose)."""
        lm = aHalfEdge1.getObs().getLandMarkId()
        if aHalfEdge1.getTime() > aHalfEdge2.getTime():
            bfr, aft = aHalfEdge2, aHalfEdge1
        else:
            bfr, aft = aHalfEdge1, aHalfEdge2
        if lm not in self._lm_ids:
            self._lm_ids.append(lm)
        for t in (bfr.getTime(), aft.getTime()):
            if t not in self._times:
                self._times.append(t)
        self._rows.append(_row(bfr, aft))

    def getEstTrajPose(self):
        return [p for p, o in zip(self._poses, self._is_obs) if o]

    def _upload_poses(self):
        self._dev.set_poses(np.array([np.asarray(p, dtype=np.float64).reshape(3) for p in self._poses]))

    def _write_back(self, times):
        new = self._dev.get_poses()
        for t in times:
            self._poses[t][0, 0] = new[t, 0]
            self._poses[t][1, 0] = new[t, 1]
            self._poses[t][2, 0] = new[t, 2]

    def updateEstPose(self):
        """:452-514.  Returns (is_calc, delta_sum, det, cond)."""
        is_calc, delta_sum, det, cond = False, 0.0, 0.0, 0.0
        if len(self._times) * 3 > 3:
            self._upload_poses()
            self._dev.set_edges(self._rows)
            is_calc, delta_sum, det, cond = self._dev.update()
            if is_calc:
                self._write_back(sorted(self._times))
            else:
                print("can Not calculate trajectory!")
            self._rows, self._lm_ids, self._times = [], [], []
        return is_calc, delta_sum, det, cond

    def estimate_trajectory(self, halves, n_landmarks, max_iter=100):
        """Robot.estimateOpticalTrajectory (:685-715) for the HalfEdge list
        ``halves``: pairs every landmark's observations once, then iterates on
        the device.  Returns the per-iteration (is_calc, delta_sum, det, cond)."""
        rows = [[h.getTime(), h.getRobotPoseId(), h.getObs().getLandMarkId(),
                 h.getObs().getDist(), h.getObs().getDir(), h.getObs().getOrient()] for h in halves]
        paired = pair_halves(rows, n_landmarks, device=self._device)     # on the device

        def times_of(edges):
            return np.unique(np.concatenate([edges["time_bfr"], edges["time_aft"]])).tolist()

        pending = edge_array(self._rows) if len(self._rows) else None
        first = np.concatenate([pending, paired]) if pending is not None else paired
        seen = set(self._times)
        for t in times_of(first) if len(first) else []:
            if t not in seen:
                self._times.append(t)
        if len(self._times) * 3 <= 3:
            # updateEstPose's leng <= 3 branch (:469): nothing solved, and the
            # pairs of this iteration stay pending (the reference clears only
            # inside the branch, :509-512); the loop ends (delta_sum = 0)
            self._rows = [_rec_row(r) for r in first]
            return np.zeros((1, 4))
        self._upload_poses()
        # iteration 1 (:697-706): pairs set before this call -- linearised at
        # their setPairObs time, i.e. at these same poses -- plus this pairing
        self._dev.set_edges(first)
        st = [self._dev.update()]
        self._write_back(sorted(self._times))
        self._rows, self._lm_ids, self._times = [], [], []
        # later iterations: only the re-paired edges, re-linearised each time;
        # an iteration with is_calc = 0 returns delta_sum = 0 and ends the loop
        if DELTA_SUM_TH <= st[0][1] and max_iter > 1 and len(paired):
            if pending is not None:
                self._dev.set_edges(paired)
            st += list(self._dev.optimize(DELTA_SUM_TH, max_iter - 1))
            self._write_back(times_of(paired))
        return np.array(st, dtype=np.float64).reshape(-1, 4)


class Robot(object):
    """graph_based_slam.py:584-897: a robot that moves with the velocity motion
    model, scans the landmarks and estimates its trajectory by graph SLAM on
    the GPU.  The noise comes from NumPy's global stream in the reference's
    order (move: three normals; each scan: three per detected landmark)."""

    DELTA_SUM_TH = 0.01                                       # :630

    def __init__(self, aPose, aDt, aScanRng_m, aScanAng_rad, aLandMarks, *, device=0):
        from mylib.error_ellipse import ErrorEllipse
        from motion_model import MotionModel
        self._sensor = ScanSensor(aScanRng_m, aScanAng_rad, aLandMarks, device=device)
        self._sensor.setNoiseParam(5, 2, 2)                   # :604
        self._motion = MotionModel(aDt, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, device=device)
        self._est = TrajectoryEstimator(aPose, device=device)
        self._dt = aDt
        self._time = 0
        self._poses = [aPose]                                 # actual poses
        self._ctl = []
        self._obs_actu, self._obs_true, self._halves = [], [], []
        self._confidence = 99.0
        self._ellipse = ErrorEllipse(self._confidence)
        self._sensor.scan(aPose)                              # :625 (its draws are consumed)
        self._observe(aPose, len(self._poses) - 1, self._time)
        self.is_calc, self.loop_cnt, self.delta_sum, self.det, self.cond = False, 0, 0.0, 0.0, 0.0

    def move(self, aV, aW):
        """:638-656."""
        actual = self._motion.moveWithNoise(self._poses[-1], aV, aW)
        odometry = self._motion.moveWithoutNoise(self._poses[-1], aV, aW)
        self._ctl.append(np.array([aV, aW]))
        self._poses.append(actual)
        self._time += 1
        seen = self._observe(actual, len(self._poses) - 1, self._time)
        self._est.addPose(deepcopy(odometry), seen)

    def _observe(self, pose, pose_id, t):
        """:658-682: scan, keep a half-edge per observed landmark."""
        noisy, clean = self._sensor.scan(pose)
        self._halves.extend(HalfEdge(t, o, pose_id) for o in noisy)
        self._obs_actu.append(noisy)
        self._obs_true.append(clean)
        return len(noisy) > 0

    def estimateOpticalTrajectory(self):
        """:685-715 (pairing and Gauss-Newton on the device)."""
        st = self._est.estimate_trajectory(self._halves, self._sensor.getLandMarkNum())
        for k, (_, dsum, det, cond) in enumerate(st):
            print(" Loop({0}):sum(dx^2) = {1}, det(H) = {2}, cond(H) = {3}".format(k + 1, dsum, det, cond))
        last = st[-1]
        self.is_calc, self.loop_cnt = bool(last[0]), len(st)
        self.delta_sum, self.det, self.cond = float(last[1]), float(last[2]), float(last[3])
        return st

    def getActualPoses(self):
        return self._poses

    def getEstTrajPose(self):
        return self._est.getEstTrajPose()

    # ---------------------------------------------------------- drawing
    def draw(self, aAx1, aAx2):
        """:717-724: the world frame (ax1) and the robot frame (ax2)."""
        self._draw_world(aAx1)
        self._draw_robot_frame(aAx2)

    def _draw_track(self, ax, color, label, poses):
        from mylib import plots
        xs = [p[0, 0] for p in poses]
        ys = [p[1, 0] for p in poses]
        plots.headings(ax, xs, ys, [p[2, 0] for p in poses], color, arrow=True)
        ax.plot(xs, ys, c=color, linewidth=1.0, linestyle="-", label=label)

    def _draw_world(self, ax):
        """:726-828."""
        from mylib import plots
        pose = self._poses[-1]
        self._sensor.draw(ax, "green", pose)
        self._draw_track(ax, "red", "Actual Trajectory", self._poses)
        pts = []
        for k, o in enumerate(self._obs_actu[-1]):
            ang = o.getDir() + pose[2, 0] - BASE_ANG
            p = (o.getDist() * np.cos(ang) + pose[0, 0], o.getDist() * np.sin(ang) + pose[1, 0])
            cov = self._sensor.tfMeasurement2World(
                self._sensor.getLandMarkCovMatrixOnMeasurementSys(o.getDist()), o.getDir(), pose[2, 0])
            plots.error_ellipse(ax, p, self._ellipse, cov[0:2, 0:2],
                                label="Error Ellipse: %.2f[%%]" % self._confidence if k == 0 else "")
            pts.append(p)
        if pts:
            plots.sight_lines(ax, pose[0:2, 0], pts)
            pts = np.array(pts)
            plots.landmark_stars(ax, pts[:, 0], pts[:, 1], face="red", edge="red", label="Land Mark(Actual)")
        self._draw_track(ax, "blue", "Estimated Trajectory", self._est.getEstTrajPose())
        status = ("<Status>\n Calculated Propriety: %s\n Number of Iterations: %d\n"
                  " $\\sum_{} \\, \\Delta{x}^T \\Delta{x}$: %e\n $det(H)$:%e\n Condition Number:%e"
                  % ("OK" if self.is_calc else "NG", self.loop_cnt, self.delta_sum, self.det, self.cond))
        ax.text(0.01, 0.99, status, transform=ax.transAxes, fontsize=10, verticalalignment="top",
                bbox=dict(boxstyle="round", facecolor="wheat", alpha=0.5))

    def _draw_robot_frame(self, ax, gain=2):
        """:830-896: observations in the robot frame (true and noisy)."""
        from mylib import plots
        for obs, face, edge, label in ((self._obs_true[-1], "yellow", "orange", "Land Mark(True)"),
                                       (self._obs_actu[-1], "red", "red", "Land Mark(Actual)")):
            if not obs:
                continue
            xs = np.array([o.getDist() * np.cos(o.getDir()) for o in obs])
            ys = np.array([o.getDist() * np.sin(o.getDir()) for o in obs])
            plots.landmark_stars(ax, xs, ys, face=face, edge=edge, label=label)
            plots.headings(ax, xs, ys, np.array([o.getOrient() for o in obs]), edge, arrow=True, gain=gain)
        for k, o in enumerate(self._obs_actu[-1]):
            cov = self._sensor.tfMeasurement2Robot(
                self._sensor.getLandMarkCovMatrixOnMeasurementSys(o.getDist()), o.getDir())
            p = (o.getDist() * np.cos(o.getDir()), o.getDist() * np.sin(o.getDir()))
            plots.error_ellipse(ax, p, self._ellipse, cov[0:2, 0:2],
                                label="Error Ellipse: %.2f[%%]" % self._confidence if k == 0 else "")
            plots.sight_lines(ax, (0.0, 0.0), [p])
        ax.scatter(0, 0, s=100, c="blue", marker="o", alpha=0.5, label="Robot")
        ax.quiver(0, 0, 0, 1, color="blue", angles="xy", scale_units="xy", scale=1)


# ------------------------------------------------------------- the demo
SCN_SENS_RANGE_m = 15.0                                       # :899-925
SCN_SENS_ANGLE_rps = np.deg2rad(80.0)
RADIUS_m = 10.0
OMEGA_rps = np.deg2rad(10.0)
VEL_mps = RADIUS_m * OMEGA_rps
LAND_MARKS = np.array([[0.0, 0.0], [14.0, 1.0], [9.0, 9.0], [0.0, 15.0], [-11.0, 10.0],
                       [-14.0, 1.0], [-10.0, -9.0], [0.0, -16.0], [10.0, -11.0]])
PERIOD_ms = 2000


def make_demo_robot(device=0):
    """The demo's robot (the reference builds it at import, :927)."""
    x_base = np.array([[10.0], [0.0], [np.deg2rad(90.0)]])
    return Robot(x_base, PERIOD_ms / 1000, SCN_SENS_RANGE_m, SCN_SENS_ANGLE_rps, LAND_MARKS,
                 device=device)


gRbt = None
time_s = 0.0


def graph_based_slam(i, aPeriod_ms):
    """:931-975: move, estimate, draw both frames (the robot is made on the
    first call, not at import, so that importing needs no GPU)."""
    import matplotlib.pyplot as plt
    from mylib import plots
    global gRbt, time_s
    if gRbt is None:
        gRbt = make_demo_robot()
    print("TIME:{0:.3f}[s]".format(time_s))
    time_s += aPeriod_ms / 1000
    gRbt.move(VEL_mps, OMEGA_rps)
    gRbt.estimateOpticalTrajectory()
    plt.cla()
    ax1 = plt.subplot2grid((1, 2), (0, 0), aspect="equal")
    ax2 = plt.subplot2grid((1, 2), (0, 1), aspect="equal")
    gRbt.draw(ax1, ax2)
    ax1.set_aspect("equal", adjustable="datalim")
    plots.finish(ax1, "World System")
    rng = SCN_SENS_RANGE_m + 5.0
    ax2.axis([-rng, rng, -rng, rng])
    plots.finish(ax2, "Robot System")
    return ax1, ax2


if __name__ == "__main__":
    import matplotlib.animation as animation
    import matplotlib.pyplot as plt

    frame_cnt = int(36 * 1000 / PERIOD_ms)
    fig = plt.figure(figsize=(18, 9))
    ani = animation.FuncAnimation(fig, graph_based_slam, frames=frame_cnt, fargs=(PERIOD_ms,), blit=False,
                                  interval=PERIOD_ms, repeat=False)
    plt.show()
