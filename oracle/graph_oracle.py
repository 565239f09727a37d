"""ORACLE -- test infrastructure only.

CPU (NumPy) restatement of graph_based_slam.py's linearise-and-solve
(TrajectoryEstimator.setPairObs :362-439 with its helpers :517-581 and
ScanSensor's covariance model :175-215; updateEstPose :452-514; the pairing of
Robot.estimateOpticalTrajectory :685-715).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may use it.

Pinned: tests/golden/graph.npz (the reference's 18-frame demo, every
Gauss-Newton iteration, and a T=300 run) -- edge blocks, H, b, det, cond and
the updated poses reproduce bit for bit (test_oracle_golden.py).

Edge rows (the C-ABI's slam_graph_edge, also the fixture layout), one per
pair of half-edges of the same landmark, ordered as setPairObs orders them:
  [t_bfr, pose_bfr, d_bfr, dir_bfr, orient_bfr,
   t_aft, pose_aft, d_aft, dir_aft, orient_aft, landmark]
"""
from __future__ import annotations

import itertools

import numpy as np

from pf_oracle import HALF_PI, to_robot_frame, wrap_angle

# graph_based_slam.py:604 -- Robot sets ScanSensor.setNoiseParam(5, 2, 2)
R_DIST = 5 / 100
R_DIR = np.deg2rad(2.0)
R_ORIENT = np.deg2rad(2.0)

EDGE_FIELDS = 11


def order_pair(row12):
    """setPairObs :371-384: the later half-edge is 'aft' (ties: the second)."""
    t1, p1, lm, d1, a1, o1, t2, p2, _, d2, a2, o2 = row12
    if t1 > t2:
        return [t2, p2, d2, a2, o2, t1, p1, d1, a1, o1, lm]
    return [t1, p1, d1, a1, o1, t2, p2, d2, a2, o2, lm]


def edges_from_pairs(pairs12):
    """Fixture pair rows (12 columns, setPairObs argument order) -> edge rows."""
    return np.array([order_pair(r) for r in pairs12], dtype=np.float64).reshape(-1, EDGE_FIELDS)


def pairs_from_halves(halves, n_landmarks):
    """estimateOpticalTrajectory :697-703: for each landmark id in order, all
    2-combinations of its half-edges in recording order.  halves rows:
    [time, pose_id, landmark, dist, dir, orient]."""
    rows = []
    for lm in range(n_landmarks):
        hs = [h for h in halves if int(h[2]) == lm]
        for a, b in itertools.combinations(hs, 2):
            rows.append([a[0], a[1], a[2], a[3], a[4], a[5], b[0], b[1], b[2], b[3], b[4], b[5]])
    return np.array(rows, dtype=np.float64).reshape(-1, 12)


def measurement_cov(dist):
    """ScanSensor :175-194 (range, bearing, orientation variances)."""
    dd = dist * R_DIST
    return np.array([[dd ** 2, 0, 0],
                     [0, (dist * np.sin(R_DIR)) ** 2, 0],
                     [0, 0, R_DIR ** 2 + R_ORIENT ** 2]])


def cov_to_world(cov, bearing, yaw):
    """ScanSensor.tfMeasurement2World :196-215."""
    ang = bearing + yaw - HALF_PI
    c, s = np.cos(ang), np.sin(ang)
    rot = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])
    return rot @ cov @ rot.T


def landmark_frame(d, bearing, orient):
    """__tfRobot2LandMark :539-555: robot pose seen from the landmark."""
    return [d, wrap_angle(np.pi + bearing - orient), wrap_angle(HALF_PI - orient)]


def linearize_edge(edge, poses):
    """One setPairObs (:362-439) -> 42 values: BB, BA, AB, AA (row-major 3x3),
    b_B, b_A."""
    tb, pb, db, ab, ob, ta, pa, da, aa, oa, _ = edge
    xb = poses[int(pb)].reshape(3, 1)
    xa = poses[int(pa)].reshape(3, 1)
    rel = xa - xb                                              # :517-537
    rel[2, 0] = wrap_angle(rel[2, 0])
    la = landmark_frame(da, aa, oa)
    lb = landmark_frame(db, ab, ob)
    px = la[0] * np.cos(la[1]) - lb[0] * np.cos(lb[1])         # :557-581
    py = la[0] * np.sin(la[1]) - lb[0] * np.sin(lb[1])
    pt = wrap_angle(la[2] - lb[2])
    err = rel - np.array([[px], [py], [pt]])
    err[2, 0] = wrap_angle(err[2, 0])
    ca = cov_to_world(measurement_cov(da), aa, xa[2, 0])
    cb = cov_to_world(measurement_cov(db), ab, xb[2, 0])
    info = np.linalg.inv(ca + cb)
    th = wrap_angle(xb[2, 0] + ab)
    jb = np.array([[-1, 0, db * np.sin(th)], [0, -1, -db * np.cos(th)], [0, 0, -1]])
    th = wrap_angle(xa[2, 0] + aa)
    ja = np.array([[1, 0, -da * np.sin(th)], [0, 1, da * np.cos(th)], [0, 0, 1]])
    blocks = [jb.T @ info @ jb, jb.T @ info @ ja, ja.T @ info @ jb, ja.T @ info @ ja,
              jb.T @ info @ err, ja.T @ info @ err]
    return np.concatenate([m.ravel() for m in blocks])


def linearize(edges, poses):
    return np.array([linearize_edge(e, poses) for e in edges]).reshape(-1, 42)


def assemble(edges, blocks):
    """updateEstPose :467-492: dense H, b over the sorted unique times (edge
    order of accumulation; anchor 1e4 I on the first time)."""
    times = sorted(set(int(t) for t in edges[:, 0]) | set(int(t) for t in edges[:, 5]))
    n = 3 * len(times)
    H = np.zeros((n, n))
    b = np.zeros((n, 1))
    if n <= 3:
        return times, H, b
    H[0:3, 0:3] += np.identity(3) * (10 ** 4)
    pos = {t: 3 * i for i, t in enumerate(times)}
    for e, blk in zip(edges, blocks):
        i, j = pos[int(e[0])], pos[int(e[5])]
        H[i:i + 3, i:i + 3] += blk[0:9].reshape(3, 3)
        H[i:i + 3, j:j + 3] += blk[9:18].reshape(3, 3)
        H[j:j + 3, i:i + 3] += blk[18:27].reshape(3, 3)
        H[j:j + 3, j:j + 3] += blk[27:36].reshape(3, 3)
        b[i:i + 3, 0][:, np.newaxis] += blk[36:39].reshape(3, 1)
        b[j:j + 3, 0][:, np.newaxis] += blk[39:42].reshape(3, 1)
    return times, H, b


def update_est_pose(edges, poses):
    """updateEstPose :452-514 on a copy of ``poses`` (T,3).  Returns
    (stats (is_calc, delta_sum, det, cond), new poses, H, b, times)."""
    poses = np.array(poses, dtype=np.float64, copy=True)
    blocks = linearize(edges, poses)
    times, H, b = assemble(edges, blocks)
    if len(times) * 3 <= 3:
        return np.array([0.0, 0.0, 0.0, 0.0]), poses, H, b[:, 0], times
    det = np.linalg.det(H)
    cond = np.linalg.cond(H)
    if 0.1 < det and cond < 10 ** 15:
        delta = -np.linalg.inv(H) @ b
        for i, t in enumerate(times):
            poses[t, 0] += delta[i * 3, 0]
            poses[t, 1] += delta[i * 3 + 1, 0]
            poses[t, 2] = wrap_angle(poses[t, 2] + delta[i * 3 + 2, 0])
        return np.array([1.0, float((delta.T @ delta)[0, 0]), det, cond]), poses, H, b[:, 0], times
    return np.array([0.0, 0.0, det, cond]), poses, H, b[:, 0], times


def scan_sensor(pose, lm, scan_range, scan_angle, r_dist, r_dir, r_orient):
    """ScanSensor.scan (graph_based_slam.py:128-172) for one pose (3,): the
    detected landmark ids, the noise-free and the noisy (dist, dir, orient),
    drawing from NumPy's global stream in the reference's order (three
    np.random.normal calls per detected landmark, :163-165)."""
    pose = np.asarray(pose, dtype=np.float64).reshape(3)
    rl = to_robot_frame(pose, lm)                                  # :149
    dist = np.linalg.norm(rl, axis=1)                              # :150
    dirs = np.arctan2(rl[:, 1], rl[:, 0])                          # :151
    orient = np.ones(rl.shape[0]) * (HALF_PI - pose[2])            # :152
    scan_rad = HALF_PI - scan_angle                                # :155
    det = [i for i in range(len(rl))
           if dist[i] <= scan_range and rl[i, 1] >= np.absolute(rl[i, 0]) * np.tan(scan_rad)]
    ids, clean, noisy = [], [], []
    for i in det:
        d = np.random.normal(dist[i], dist[i] * r_dist)
        a = wrap_angle(np.random.normal(dirs[i], r_dir))
        o = wrap_angle(np.random.normal(orient[i], r_orient))
        ids.append(i)
        clean.append([dist[i], dirs[i], orient[i]])
        noisy.append([d, a, o])
    return (np.array(ids, dtype=np.int64), np.array(clean).reshape(-1, 3),
            np.array(noisy).reshape(-1, 3))
