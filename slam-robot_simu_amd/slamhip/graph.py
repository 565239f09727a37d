"""Device graph-based SLAM: a handle on libslam_hip's slam_graph_* entry
points (TrajectoryEstimator's linearise-and-solve, graph_based_slam.py
:362-514, and the Gauss-Newton loop :685-715)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import GRAPH_COND, GRAPH_SOLVER, GraphConfig, check, dptr

# slam_graph_edge, 80 bytes
EDGE_DTYPE = np.dtype([("time_bfr", "<i8"), ("pose_bfr", "<i8"), ("time_aft", "<i8"),
                       ("pose_aft", "<i8"), ("obs_bfr", "<f8", (3,)), ("obs_aft", "<f8", (3,))])


HALF_DTYPE = np.dtype([("time", "<i8"), ("pose", "<i8"), ("landmark", "<i8"), ("obs", "<f8", (3,))])


def pair_halves(halves, n_landmarks, device=0):
    """Robot.estimateOpticalTrajectory's pairing (graph_based_slam.py:697-703)
    on the device: ``halves`` rows [time, pose_id, landmark, dist, dir, orient]
    (or HALF_DTYPE records) in recording order -> slam_graph_edge records, in
    the reference's order (landmark, then itertools.combinations), each pair
    ordered as setPairObs orders it (:371-384)."""
    if not (isinstance(halves, np.ndarray) and halves.dtype == HALF_DTYPE):
        rows = np.asarray(halves, dtype=np.float64).reshape(-1, 6)
        rec = np.zeros(len(rows), dtype=HALF_DTYPE)
        rec["time"], rec["pose"], rec["landmark"] = rows[:, 0], rows[:, 1], rows[:, 2]
        rec["obs"] = rows[:, 3:6]
        halves = rec
    halves = np.ascontiguousarray(halves)
    lib = _lib.load()
    n = C.c_int64(0)
    check(lib.slam_graph_pair_halves(len(halves), halves.ctypes.data_as(C.c_void_p),
                                     int(n_landmarks), int(device), C.byref(n), None),
          "slam_graph_pair_halves")
    out = np.zeros(n.value, dtype=EDGE_DTYPE)
    if n.value:
        check(lib.slam_graph_pair_halves(len(halves), halves.ctypes.data_as(C.c_void_p),
                                         int(n_landmarks), int(device), C.byref(n),
                                         out.ctypes.data_as(C.c_void_p)),
              "slam_graph_pair_halves")
    return out


def edge_array(rows):
    """Edge rows [t_bfr, pose_bfr, d, dir, orient, t_aft, pose_aft, d, dir, orient, (lm)]
    -> slam_graph_edge records."""
    rows = np.asarray(rows, dtype=np.float64).reshape(len(rows), -1)
    out = np.zeros(len(rows), dtype=EDGE_DTYPE)
    out["time_bfr"] = rows[:, 0].astype(np.int64)
    out["pose_bfr"] = rows[:, 1].astype(np.int64)
    out["obs_bfr"] = rows[:, 2:5]
    out["time_aft"] = rows[:, 5].astype(np.int64)
    out["pose_aft"] = rows[:, 6].astype(np.int64)
    out["obs_aft"] = rows[:, 7:10]
    return out


class DeviceGraph:
    """Pose graph on one GPU.  Noise defaults = Robot's setNoiseParam(5, 2, 2)
    (graph_based_slam.py:604); anchor and gate = updateEstPose :475, :496."""

    def __init__(self, *, r_dist=0.05, r_dir=np.deg2rad(2.0), r_orient=np.deg2rad(2.0),
                 anchor=1e4, det_min=0.1, cond_max=1e15, solver="auto", pcg_tol=1e-10,
                 pcg_max_iter=20000, cond="margin", cond_tol=1e-5, cond_max_iter=3000, device=0):
        cfg = GraphConfig()
        cfg.r_dist, cfg.r_dir, cfg.r_orient = float(r_dist), float(r_dir), float(r_orient)
        cfg.anchor, cfg.det_min, cfg.cond_max = float(anchor), float(det_min), float(cond_max)
        cfg.pcg_tol, cfg.pcg_max_iter = float(pcg_tol), int(pcg_max_iter)
        cfg.solver = GRAPH_SOLVER[solver]
        cfg.cond_mode = GRAPH_COND[cond]
        cfg.cond_tol, cfg.cond_max_iter = float(cond_tol), int(cond_max_iter)
        self.cfg = cfg
        self._lib = _lib.load()
        h = C.c_void_p()
        check(self._lib.slam_graph_create(C.byref(cfg), int(device), C.byref(h)), "slam_graph_create")
        self._h = h
        self.n_poses = 0
        self.n_edges = 0

    def close(self):
        if getattr(self, "_h", None):
            self._lib.slam_graph_destroy(self._h)
            self._h = None

    __del__ = close

    def set_poses(self, poses):
        poses = np.ascontiguousarray(poses, dtype=np.float64).reshape(-1, 3)
        check(self._lib.slam_graph_set_poses(self._h, len(poses), dptr(poses)), "slam_graph_set_poses")
        self.n_poses = len(poses)

    def get_poses(self):
        out = np.empty((self.n_poses, 3))
        check(self._lib.slam_graph_get_poses(self._h, dptr(out)), "slam_graph_get_poses")
        return out

    def set_edges(self, edges):
        rec = edges if (isinstance(edges, np.ndarray) and edges.dtype == EDGE_DTYPE) else edge_array(edges)
        rec = np.ascontiguousarray(rec)
        check(self._lib.slam_graph_set_edges(self._h, len(rec), rec.ctypes.data_as(C.c_void_p)),
              "slam_graph_set_edges")
        self.n_edges = len(rec)

    def update(self):
        """updateEstPose: returns (is_calc, delta_sum, det, cond)."""
        st = np.zeros(4)
        check(self._lib.slam_graph_update(self._h, dptr(st)), "slam_graph_update")
        return bool(st[0]), float(st[1]), float(st[2]), float(st[3])

    def optimize(self, delta_sum_th=0.01, max_iter=100):
        st = np.zeros((max_iter, 4))
        n = C.c_int32(0)
        check(self._lib.slam_graph_optimize(self._h, float(delta_sum_th), int(max_iter), dptr(st),
                                            C.byref(n)), "slam_graph_optimize")
        return st[:n.value]

    def get_system(self, dense=True, blocks=False):
        nt = C.c_int64(0)
        check(self._lib.slam_graph_get_system(self._h, C.byref(nt), None, None, None, None),
              "slam_graph_get_system")
        n = 3 * nt.value
        times = np.empty(nt.value, dtype=np.int64)
        H = np.empty((n, n)) if dense else None
        b = np.empty(n)
        blk = np.empty((self.n_edges, 42)) if blocks else None
        check(self._lib.slam_graph_get_system(self._h, C.byref(nt),
                                              times.ctypes.data_as(C.POINTER(C.c_int64)),
                                              dptr(H), dptr(b), dptr(blk)), "slam_graph_get_system")
        return times, H, b, blk

    def get_bsr(self):
        """(rows, cols, vals (n_slots, 3, 3)) of the last assembled H."""
        ns = C.c_int64(0)
        check(self._lib.slam_graph_get_bsr(self._h, C.byref(ns), None, None, None), "slam_graph_get_bsr")
        rows = np.empty(ns.value, dtype=np.int64)
        cols = np.empty(ns.value, dtype=np.int64)
        vals = np.empty((ns.value, 3, 3))
        P64 = C.POINTER(C.c_int64)
        check(self._lib.slam_graph_get_bsr(self._h, C.byref(ns), rows.ctypes.data_as(P64),
                                           cols.ctypes.data_as(P64), dptr(vals)), "slam_graph_get_bsr")
        return rows, cols, vals

    def get_delta(self):
        nt = C.c_int64(0)
        check(self._lib.slam_graph_get_system(self._h, C.byref(nt), None, None, None, None),
              "slam_graph_get_system")
        out = np.empty(3 * nt.value)
        check(self._lib.slam_graph_get_delta(self._h, dptr(out)), "slam_graph_get_delta")
        return out

    def timing(self):
        out = np.zeros(5)
        check(self._lib.slam_graph_timing(self._h, dptr(out)), "slam_graph_timing")
        return dict(linearize_ms=out[0], assemble_ms=out[1], solve_ms=out[2], update_ms=out[3],
                    pcg_iterations=int(out[4]))

    def cond_info(self):
        """The last PCG-path update's condition estimate (slam_graph_cond_info)."""
        out = np.zeros(7)
        check(self._lib.slam_graph_cond_info(self._h, dptr(out)), "slam_graph_cond_info")
        return dict(iterations=int(out[0]), status=int(out[1]), lambda_min=out[2],
                    lambda_max=out[3], iterations_min=int(out[4]), iterations_max=int(out[5]),
                    ms=out[6])

    def gate_info(self):
        """The last PCG-path update's gate (cond="margin": an estimate with
        margins, not a certificate; slam_graph_gate_info): the log-det interval,
        the cond(H) the decision used, the Ritz values, each half's decision and
        the margins the decisions held (det_margin: the factor by which the Ritz
        lambda_min may over-estimate lambda_min(H) before the det lower end
        drops below ln det_min; cond_margin: cond_max / cond)."""
        out = np.zeros(14)
        check(self._lib.slam_graph_gate_info(self._h, dptr(out)), "slam_graph_gate_info")
        return dict(decided_by="bounds" if out[0] == 1 else "dense" if out[0] == 2 else "none",
                    det_decision=int(out[1]), det=GATE_DET.get(int(out[1]), "none"),
                    cond_decision=int(out[2]), logdet_lo=out[3], logdet_hi=out[4],
                    cond=out[5], lambda_min=out[6], lambda_max=out[7], trp2=out[8],
                    n=int(out[9]), estimate_iterations=int(out[10]), ms=out[11],
                    det_margin=out[12], cond_margin=out[13],
                    cond_decided=GATE_COND.get(int(out[2]), "none"))


GATE_DET = {1: "passed (log-det lower end, estimate with 1000x margin)",
            0: "rejected (log-det upper end, Fischer bound)", 3: "passed (dense LU det)",
            2: "rejected (dense LU det)", -1: "undecided"}
GATE_COND = {1: "passed (estimate with margin)", 0: "rejected (estimate: for certain)",
             5: "passed (converged estimate inside the margin band)",
             3: "passed (dense Lanczos cond)", 2: "rejected (dense Lanczos cond)", -1: "undecided"}


def circle_graph(n_poses, n_landmarks=64, loops_per_pose=3, seed=0, odom_noise=0.02):
    """Synthetic pose graph of the graph_based_slam.py form (BASELINE config 5):
    a robot circling at 10 m radius with a ScanSensor (15 m, +-80 deg,
    :899-902) among ``n_landmarks`` landmarks on a 14 m ring; one edge per
    consecutive pose pair sharing a landmark and ``loops_per_pose`` loop edges
    per pose between observations of the same landmark at other times.
    Returns (initial pose estimates (T,3), true poses (T,3), edge records)."""
    rs = np.random.RandomState(seed)
    step = np.deg2rad(10.0)
    ang = np.arange(n_poses) * step
    truth = np.column_stack([10 * np.cos(ang), 10 * np.sin(ang),
                             np.mod(ang + np.pi / 2 + np.pi, 2 * np.pi) - np.pi])
    la = np.linspace(0, 2 * np.pi, n_landmarks, endpoint=False)
    lm = np.column_stack([14 * np.cos(la), 14 * np.sin(la)])
    # visibility and noisy (distance, direction, orientation) per pose
    d = lm[None, :, :] - truth[:, None, :2]
    psi = np.pi / 2 - truth[:, 2]
    rx = np.cos(psi)[:, None] * d[..., 0] - np.sin(psi)[:, None] * d[..., 1]
    ry = np.sin(psi)[:, None] * d[..., 0] + np.cos(psi)[:, None] * d[..., 1]
    dist = np.hypot(rx, ry)
    vis = (dist <= 15.0) & (ry >= np.abs(rx) * np.tan(np.pi / 2 - np.deg2rad(80.0)))
    bearing = np.arctan2(ry, rx)
    orient = np.repeat((np.pi / 2 - truth[:, 2])[:, None], n_landmarks, 1)   # ScanSensor :153
    obs = np.stack([dist * (1 + 0.05 * rs.standard_normal(dist.shape)),
                    bearing + np.deg2rad(2.0) * rs.standard_normal(dist.shape),
                    orient + np.deg2rad(2.0) * rs.standard_normal(dist.shape)], -1)
    obs[..., 1:] = np.mod(obs[..., 1:] + np.pi, 2 * np.pi) - np.pi
    seen_by = [np.flatnonzero(vis[:, j]) for j in range(n_landmarks)]
    rows = []

    def add(t1, t2, j):
        a, b = (t1, t2) if t1 < t2 else (t2, t1)
        rows.append((a, a, *obs[a, j], b, b, *obs[b, j]))

    for t in range(1, n_poses):
        common = np.flatnonzero(vis[t - 1] & vis[t])
        if len(common):
            add(t - 1, t, int(common[rs.randint(len(common))]))
        vis_t = np.flatnonzero(vis[t])
        for _ in range(loops_per_pose if len(vis_t) else 0):
            j = int(vis_t[rs.randint(len(vis_t))])
            others = seen_by[j]
            o = int(others[rs.randint(len(others))])
            if o != t:
                add(o, t, j)
    rec = np.zeros(len(rows), dtype=EDGE_DTYPE)
    r = np.array(rows, dtype=np.float64)
    rec["time_bfr"] = r[:, 0].astype(np.int64)
    rec["pose_bfr"] = r[:, 1].astype(np.int64)
    rec["obs_bfr"] = r[:, 2:5]
    rec["time_aft"] = r[:, 5].astype(np.int64)
    rec["pose_aft"] = r[:, 6].astype(np.int64)
    rec["obs_aft"] = r[:, 7:10]
    init = truth + np.cumsum(odom_noise * rs.standard_normal(truth.shape), axis=0)
    init[:, 2] = np.mod(init[:, 2] + np.pi, 2 * np.pi) - np.pi
    return init, truth, rec
