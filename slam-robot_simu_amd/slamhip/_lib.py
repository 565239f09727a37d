"""ctypes binding of libslam_hip.so (include/slam_hip.h).

The shared library is built in-tree (``make -C slam-robot_simu_amd``) and is
the only compute path: there is no CPU fallback.  Loading fails loudly when the
library is missing, and every entry point raises on a non-zero return code.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SLAM_HIP_LIB: an alternative in-tree build (kernel variant experiments); the
# product path is always this library, and a missing library raises.
LIB_PATH = os.environ.get("SLAM_HIP_LIB", os.path.join(_HERE, "libslam_hip.so"))

SLAM_OK = 0
SLAM_ERR_ARG = -1
SLAM_ERR_HIP = -2
SLAM_ERR_INDEX = -3
SLAM_ERR_STATE = -4
SLAM_ERR_SOLVE = -5
SLAM_ERR_COMM = -6

MOTION = {"linear": 0, "velocity": 1}
LIKELIHOOD = {"product": 0, "logsum": 1}


class PFConfig(C.Structure):
    _fields_ = [("dt", C.c_double), ("ess_threshold", C.c_double), ("r_cov", C.c_double * 4),
                ("q_factor", C.c_double * 9), ("alphas", C.c_double * 6), ("x0", C.c_double * 3),
                ("seed", C.c_uint64), ("motion", C.c_int32), ("likelihood", C.c_int32)]


class PFResult(C.Structure):
    _fields_ = [("x_est", C.c_double * 3), ("cov", C.c_double * 9), ("max_val", C.c_double),
                ("ess", C.c_double), ("weight_sum", C.c_double), ("max_idx", C.c_int64),
                ("resampled", C.c_int32), ("resample_next", C.c_int32), ("status", C.c_int32),
                ("n_special", C.c_int32), ("ess_near", C.c_int32), ("dd_waves", C.c_int32)]


class EKFConfig(C.Structure):
    _fields_ = [("dt", C.c_double), ("vel", C.c_double), ("omega", C.c_double),
                ("q", C.c_double * 9), ("r", C.c_double * 4), ("x0", C.c_double * 3),
                ("p0", C.c_double * 9), ("motion", C.c_int32), ("pad0", C.c_int32),
                ("alphas", C.c_double * 6)]


class EKFSLAMConfig(C.Structure):
    _fields_ = [("dt", C.c_double), ("q_robot", C.c_double * 9), ("r_dist", C.c_double),
                ("r_dir", C.c_double), ("r_orient", C.c_double), ("motion", C.c_int32),
                ("pad0", C.c_int32), ("alphas", C.c_double * 6)]


class GraphEdge(C.Structure):
    _fields_ = [("time_bfr", C.c_int64), ("pose_bfr", C.c_int64), ("time_aft", C.c_int64),
                ("pose_aft", C.c_int64), ("obs_bfr", C.c_double * 3), ("obs_aft", C.c_double * 3)]


class GraphConfig(C.Structure):
    _fields_ = [("r_dist", C.c_double), ("r_dir", C.c_double), ("r_orient", C.c_double),
                ("anchor", C.c_double), ("det_min", C.c_double), ("cond_max", C.c_double),
                ("pcg_tol", C.c_double), ("pcg_max_iter", C.c_int32), ("solver", C.c_int32),
                ("cond_tol", C.c_double), ("cond_max_iter", C.c_int32), ("cond_mode", C.c_int32)]


GRAPH_SOLVER = {"auto": 0, "dense": 1, "pcg": 2}
GRAPH_COND = {"estimate": 0, "off": 1, "margin": 2, "certify": 2}   # "certify": the former name

_P = C.c_void_p
_D = C.POINTER(C.c_double)
_I64 = C.POINTER(C.c_int64)
_I32 = C.POINTER(C.c_int32)
_U32 = C.POINTER(C.c_uint32)

# name -> (restype, argtypes)
SIGNATURES = {
    "slam_version": (C.c_int, []),
    "slam_last_error": (C.c_char_p, []),
    "slam_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "slam_pf_create": (C.c_int, [C.POINTER(PFConfig), C.c_int64, C.c_int32, _D, C.c_int,
                                 C.POINTER(_P)]),
    "slam_pf_destroy": (C.c_int, [_P]),
    "slam_pf_set_landmarks": (C.c_int, [_P, _D]),
    "slam_pf_set_state": (C.c_int, [_P, _D, _D, _D, _D]),
    "slam_pf_get_state": (C.c_int, [_P, _D, _D, _D, _D]),
    "slam_pf_get_weights_raw": (C.c_int, [_P, _D, _D]),
    "slam_pf_step": (C.c_int, [_P, _D, _D, _D, C.c_double, C.POINTER(PFResult)]),
    "slam_pf_resample": (C.c_int, [_P, C.c_double, C.c_int32, _I32]),
    "slam_pf_predict": (C.c_int, [_P, _D, _D]),
    "slam_pf_update": (C.c_int, [_P, _D, C.POINTER(PFResult)]),
    "slam_pf_resample_indices": (C.c_int, [_P, C.c_double, _I64, _I32]),
    "slam_pf_weight_sum": (C.c_int, [_P, _D]),
    "slam_debug_pair_normals": (C.c_int, [C.c_int, C.c_uint64, C.c_int64, C.c_uint32, C.c_uint64, _D]),
    "slam_pf_load_observations": (C.c_int, [_P, C.c_int32, _D]),
    "slam_pf_run": (C.c_int, [_P, C.c_int32, C.c_int32, _D, C.POINTER(PFResult)]),
    "slam_pf_enable_timing": (C.c_int, [_P, C.c_int32]),
    "slam_pf_timing": (C.c_int, [_P, C.c_int32, _D, _I64]),
    "slam_pf_set_graphs": (C.c_int, [_P, C.c_int32]),
    "slam_pf_prepare_graphs": (C.c_int, [_P, _D]),
    "slam_pf_set_scan_merged": (C.c_int, [_P, C.c_int32]),
    "slam_pf_set_ess_band": (C.c_int, [_P, C.c_double]),
    "slam_pf_set_resample_next": (C.c_int, [_P, C.c_int32]),
    "slam_pf_set_stream": (C.c_int, [_P, _P, C.c_int32]),
    "slam_motion_velocity": (C.c_int, [_D, C.c_int64, _D, C.c_double, C.c_double, _D, _D,
                                       C.c_int]),
    "slam_scan_detect": (C.c_int, [C.c_int64, _D, _D, C.c_int64, _D, C.c_double, C.c_double, _I32, _D,
                                   C.c_int]),
    "slam_scan_noise": (C.c_int, [C.c_int64, _D, _D, C.c_double, C.c_double, C.c_double, _D, C.c_int]),
    "slam_error_ellipse": (C.c_int, [C.c_int64, _D, C.c_double, C.c_int32, _D, C.c_int]),
    "slam_mt_create": (C.c_int, [_U32, C.c_int32, C.c_int32, C.c_double, C.c_int, C.POINTER(_P)]),
    "slam_mt_destroy": (C.c_int, [_P]),
    "slam_mt_set_state": (C.c_int, [_P, _U32, C.c_int32, C.c_int32, C.c_double]),
    "slam_mt_get_state": (C.c_int, [_P, _U32, _I32, _I32, _D]),
    "slam_mt_random_sample": (C.c_int, [_P, C.c_int64, _D]),
    "slam_mt_standard_normal": (C.c_int, [_P, C.c_int64, _D]),
    "slam_glibc_log": (C.c_int, [C.c_int64, _D, _D]),
    "slam_mt_jump_window": (C.c_int, [_U32, C.c_uint64, _U32]),
    "slam_pf_set_rng_mt19937": (C.c_int, [_P, _U32, C.c_int32, C.c_int32, C.c_double, _D]),
    "slam_pf_rng_mt19937_info": (C.c_int, [_P, C.POINTER(C.c_int64)]),
    "slam_pf_get_rng_mt19937": (C.c_int, [_P, _U32, _I32, _I32, _D]),
    "slam_pf_step_truth": (C.c_int, [_P, _D, _D, _D, C.POINTER(PFResult)]),
    "slam_pf_load_truth": (C.c_int, [_P, C.c_int32, _D]),
    "slam_comm_unique_id": (C.c_int, [C.c_char_p]),
    "slam_comm_create": (C.c_int, [C.c_char_p, C.c_int32, C.c_int32, C.c_int, C.POINTER(_P)]),
    "slam_comm_destroy": (C.c_int, [_P]),
    "slam_comm_info": (C.c_int, [_P, _I32, _I32]),
    "slam_comm_all_gather_host": (C.c_int, [_P, _P, _P, C.c_int64]),
    "slam_dist_shard_range": (C.c_int, [C.c_int64, C.c_int32, C.c_int32, _I64, _I64]),
    "slam_pf_create_dist_shard": (C.c_int, [C.POINTER(PFConfig), C.c_int64, C.c_int64, C.c_int64,
                                            C.c_int32, _D, C.c_int, C.POINTER(_P)]),
    "slam_dist_create": (C.c_int, [C.POINTER(_P), C.c_int32, C.c_int32, C.c_int32, C.POINTER(_P)]),
    "slam_dist_destroy": (C.c_int, [_P]),
    "slam_dist_handle_size": (C.c_int, [_I64]),
    "slam_dist_export": (C.c_int, [_P, _P]),
    "slam_dist_connect": (C.c_int, [_P, _P]),
    "slam_dist_connect_comm": (C.c_int, [_P, _P]),
    "slam_dist_set_collective": (C.c_int, [_P, _P]),
    "slam_dist_step": (C.c_int, [_P, _D, _D, C.POINTER(PFResult)]),
    "slam_dist_load_observations": (C.c_int, [_P, C.c_int32, _D]),
    "slam_dist_run": (C.c_int, [_P, C.c_int32, C.c_int32, _D, C.POINTER(PFResult)]),
    "slam_dist_prepare_graphs": (C.c_int, [_P, _D]),
    "slam_dist_set_merged": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_int32)]),
    "slam_ekf_create": (C.c_int, [C.POINTER(EKFConfig), C.c_int64, C.c_int, C.POINTER(_P)]),
    "slam_ekf_destroy": (C.c_int, [_P]),
    "slam_ekf_set_state": (C.c_int, [_P, _D, _D]),
    "slam_ekf_get_state": (C.c_int, [_P, _D, _D]),
    "slam_ekf_step": (C.c_int, [_P, _D, _D, _D, _D, _D]),
    "slam_ekf_run": (C.c_int, [_P, C.c_int32, _D, _D, _D]),
    "slam_ekf_run_device": (C.c_int, [_P, C.c_int32, _D, _P, _P]),
    "slam_ekf_load_observations": (C.c_int, [_P, C.c_int32, _D]),
    "slam_ekf_run_loaded": (C.c_int, [_P, C.c_int32, _D, C.c_int32]),
    "slam_ekf_synchronize": (C.c_int, [_P]),
    "slam_ekfslam_create": (C.c_int, [C.POINTER(EKFSLAMConfig), C.c_int64, C.c_int,
                                      C.POINTER(_P)]),
    "slam_ekfslam_destroy": (C.c_int, [_P]),
    "slam_ekfslam_set_state": (C.c_int, [_P, _D, _D]),
    "slam_ekfslam_init_diag": (C.c_int, [_P, _D, _D]),
    "slam_ekfslam_get_state": (C.c_int, [_P, _D, _D]),
    "slam_ekfslam_get_rows": (C.c_int, [_P, C.c_int64, _I64, _D]),
    "slam_ekfslam_predict": (C.c_int, [_P, _D]),
    "slam_ekfslam_update": (C.c_int, [_P, C.c_int32, _I64, _D]),
    "slam_ekfslam_step": (C.c_int, [_P, _D, C.c_int32, _I64, _D]),
    "slam_ekfslam_timing": (C.c_int, [_P, _D]),
    "slam_graph_create": (C.c_int, [C.POINTER(GraphConfig), C.c_int, C.POINTER(_P)]),
    "slam_graph_destroy": (C.c_int, [_P]),
    "slam_graph_set_poses": (C.c_int, [_P, C.c_int64, _D]),
    "slam_graph_get_poses": (C.c_int, [_P, _D]),
    "slam_graph_set_edges": (C.c_int, [_P, C.c_int64, _P]),
    "slam_graph_update": (C.c_int, [_P, _D]),
    "slam_graph_optimize": (C.c_int, [_P, C.c_double, C.c_int32, _D, _I32]),
    "slam_graph_get_system": (C.c_int, [_P, _I64, _I64, _D, _D, _D]),
    "slam_graph_get_bsr": (C.c_int, [_P, _I64, _I64, _I64, _D]),
    "slam_graph_get_delta": (C.c_int, [_P, _D]),
    "slam_graph_timing": (C.c_int, [_P, _D]),
    "slam_graph_cond_info": (C.c_int, [_P, _D]),
    "slam_graph_gate_info": (C.c_int, [_P, _D]),
    "slam_graph_linearize_solve": (C.c_int, [C.POINTER(GraphConfig), _P, C.c_int64, _D, C.c_int64,
                                             _D, C.c_int]),
    "slam_graph_pair_halves": (C.c_int, [C.c_int64, _P, C.c_int64, C.c_int, _I64, _P]),
}

_lib = None


class SlamError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{msg} (code {code})")
        self.code = code


def load():
    """Load libslam_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not found: build it with `make -C slam-robot_simu_amd` "
                          "(there is no CPU fallback)")
    lib = C.CDLL(LIB_PATH)
    variant = "SLAM_HIP_LIB" in os.environ      # development variant: may predate entry points
    for name, (res, args) in SIGNATURES.items():
        if variant and not hasattr(lib, name):
            continue
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def check(rc, what=""):
    if rc != SLAM_OK:
        msg = load().slam_last_error().decode(errors="replace")
        if rc == SLAM_ERR_INDEX:
            raise IndexError(msg)
        raise SlamError(rc, f"{what}: {msg}" if what else msg)


def device_count() -> int:
    n = C.c_int(0)
    check(load().slam_device_count(C.byref(n)), "slam_device_count")
    return n.value


def dptr(a):
    """Pointer to a C-contiguous float64 numpy array (or NULL for None)."""
    if a is None:
        return None
    return a.ctypes.data_as(_D)
