"""Device particle filter: a handle on libslam_hip's slam_pf_* entry points.

State lives in HBM as SoA fp64 arrays; this class only moves control,
observations and (in NumPy-stream mode) noise across the boundary.
"""
from __future__ import annotations

import ctypes as C
from collections.abc import Sequence

import numpy as np

from . import _lib
from ._lib import PFConfig, PFResult, check, dptr
from .rng import state_fields

BASE_ANG = np.pi / 2.0          # mylib/transform.py:12


def _f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None and a.shape != shape:
        a = a.reshape(shape)
    return a


def numpy_noise_factor(q):
    """The matrix numpy.random.multivariate_normal applies to standard
    normals: sqrt(s)[:, None] * v of svd(Q) (used by the device RNG so that
    its noise has the reference's covariance)."""
    _, s, v = np.linalg.svd(np.asarray(q, dtype=np.float64))
    return np.sqrt(s)[:, None] * v


def make_config(n_global, *, dt=0.1, q=None, r=None, x0=(10.0, 0.0, np.pi / 2), motion="linear",
                likelihood="product", alphas=(0.1,) * 6, ess_threshold=None, seed=0):
    """slam_pf_config from particle_filter.py:21-84's constants (keyword overrides)."""
    q = np.diag([0.03, 0.03, np.deg2rad(2.0)]) ** 2 if q is None else np.asarray(q, float)
    r = np.diag([0.3, 0.3]) ** 2 if r is None else np.asarray(r, float)
    cfg = PFConfig()
    cfg.dt = float(dt)
    cfg.ess_threshold = n_global / 100.0 if ess_threshold is None else float(ess_threshold)
    cfg.r_cov[:] = [float(v) for v in r.ravel()]
    cfg.q_factor[:] = [float(v) for v in numpy_noise_factor(q).ravel()]
    cfg.alphas[:] = [float(v) for v in alphas]
    cfg.x0[:] = [float(v) for v in x0]
    cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    cfg.motion = _lib.MOTION[motion]
    cfg.likelihood = _lib.LIKELIHOOD[likelihood]
    return cfg


class RunResults(Sequence):
    """The records of a device-resident batch (slam_pf_run / slam_dist_run):
    the C-ABI's slam_pf_result array as returned, each record read into the
    dict of DeviceParticleFilter._res when it is accessed (a batch's Python
    dicts cost ~6 us per step; building them lazily keeps that out of the
    batch's own call).  ``records`` is the same memory as a NumPy structured
    array."""

    def __init__(self, res, dicts=None):
        self._r = res
        self._d = dicts

    @classmethod
    def from_dicts(cls, dicts):
        """Records already formed as dicts (the confirm_ess path, whose dicts
        carry the host's ESS confirmation fields)."""
        return cls(None, list(dicts))

    @property
    def records(self):
        if self._r is None:
            raise AttributeError("records: this batch was returned as dicts (confirm_ess)")
        return np.ctypeslib.as_array(self._r)

    def __len__(self):
        return len(self._d) if self._d is not None else len(self._r)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        if self._d is not None:
            return self._d[i]
        return DeviceParticleFilter._res(self._r[i])

    def __add__(self, other):
        return list(self) + list(other)

    def __radd__(self, other):
        return list(other) + list(self)

    def __eq__(self, other):
        """Element-wise against any sequence of records: two runs
        compare by their records, not by identity."""
        if not isinstance(other, Sequence) or isinstance(other, (str, bytes)):
            return NotImplemented
        if len(self) != len(other):
            return False
        for a, b in zip(self, other):
            if a.keys() != b.keys():
                return False
            for k in a:
                x, y = np.asarray(a[k]), np.asarray(b[k])
                # NaN fields (a degenerate step's cov, det, ESS) compare equal
                nan_ok = x.dtype.kind in "fc" and y.dtype.kind in "fc"
                if not np.array_equal(x, y, equal_nan=nan_ok):
                    return False
        return True

    __hash__ = None

    def to_list(self):
        """The records as plain dicts (JSON-serialisable after .tolist() of the arrays)."""
        return list(self)

    def __repr__(self):
        return f"RunResults({list(self)!r})"


class DeviceParticleFilter:
    """Particles on one GPU.  Parameters mirror particle_filter.py:21-84."""

    def __init__(self, n_particles, landmarks, *, dt=0.1, q=None, r=None, x0=(10.0, 0.0, np.pi / 2),
                 motion="linear", likelihood="product", alphas=(0.1,) * 6, ess_threshold=None,
                 seed=0, device=0):
        lib = _lib.load()
        self.n = int(n_particles)
        self.lm = _f64(landmarks).reshape(-1, 2)
        self.nl = self.lm.shape[0]
        cfg = make_config(self.n, dt=dt, q=q, r=r, x0=x0, motion=motion, likelihood=likelihood,
                          alphas=alphas, ess_threshold=ess_threshold, seed=seed)
        self.motion = motion
        self.cfg = cfg
        self.r = np.diag([0.3, 0.3]) ** 2 if r is None else np.asarray(r, float)
        self.mt = False
        h = C.c_void_p()
        check(lib.slam_pf_create(C.byref(cfg), self.n, self.nl, dptr(self.lm), int(device),
                                 C.byref(h)), "slam_pf_create")
        self._h = h
        self._lib = lib
        self.resample_next = False
        self.last = None

    # ------------------------------------------------------------ lifetime
    def close(self):
        if getattr(self, "_h", None):
            self._lib.slam_pf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # --------------------------------------------------------------- state
    def set_state(self, x=None, y=None, th=None, w=None):
        arrs = [None if a is None else _f64(a, (self.n,)) for a in (x, y, th, w)]
        check(self._lib.slam_pf_set_state(self._h, *[dptr(a) for a in arrs]), "slam_pf_set_state")
        if w is not None:
            ww = arrs[3]
            self.resample_next = bool(1.0 / float(ww @ ww) < self.cfg.ess_threshold)
            self.set_resample_next(self.resample_next)        # the reference's dot decides

    def set_resample_next(self, on):
        """The next step's resample decision (particle_filter.py:210-211)."""
        check(self._lib.slam_pf_set_resample_next(self._h, int(bool(on))),
              "slam_pf_set_resample_next")
        self.resample_next = bool(on)

    # ESS within this relative distance of the threshold: the decision is
    # re-formed on the host as the reference forms it (its BLAS dot order)
    ESS_CONFIRM_BAND = 1e-9

    def _confirm_ess(self, out):
        """particle_filter.py:210-211 decides from `1 / (pw @ pw.T)` in the host
        BLAS's summation order; the device sums the same squares in its own
        fixed order (a few ulp apart).  Where the two could disagree -- the
        device's ESS within ESS_CONFIRM_BAND of ESS_TH -- the weights come back
        and the reference's own expression decides (the normalised weights are
        bit-identical, so the decision is too)."""
        th = self.cfg.ess_threshold
        out["ess_confirmed"] = False
        if not abs(out["ess"] - th) <= self.ESS_CONFIRM_BAND * th:
            return out
        pw = self.get_state()[3]
        ess = float(np.reciprocal(pw @ pw.T))
        rn = ess < th
        if rn != bool(out["resample_next"]):
            self.set_resample_next(rn)
        out["resample_next"] = rn
        out["ess_host"] = ess
        out["ess_confirmed"] = True
        self.resample_next = rn
        return out

    def get_state(self):
        out = [np.empty(self.n) for _ in range(4)]
        check(self._lib.slam_pf_get_state(self._h, *[dptr(a) for a in out]), "slam_pf_get_state")
        return tuple(out)

    def get_weights_raw(self):
        """(w_un, s): the last step's weights before normalisation and the
        np.sum the device divided them by (slam_pf_get_weights_raw)."""
        w = np.empty(self.n)
        s = C.c_double(0.0)
        check(self._lib.slam_pf_get_weights_raw(self._h, dptr(w), C.byref(s)),
              "slam_pf_get_weights_raw")
        return w, s.value

    def set_landmarks(self, lm):
        lm = _f64(lm).reshape(-1, 2)
        if lm.shape[0] != self.nl:
            raise ValueError("landmark count is fixed at construction")
        self.lm = lm
        check(self._lib.slam_pf_set_landmarks(self._h, dptr(lm)), "slam_pf_set_landmarks")

    # ---------------------------------------------------------------- step
    @staticmethod
    def _res(r: PFResult):
        return {"x_est": np.array(r.x_est[:]), "cov": np.array(r.cov[:]).reshape(3, 3),
                "max_val": r.max_val, "max_idx": int(r.max_idx), "ess": r.ess,
                "weight_sum": r.weight_sum, "resampled": bool(r.resampled),
                "resample_next": bool(r.resample_next), "status": r.status,
                "n_special": r.n_special, "ess_near": bool(r.ess_near), "dd_waves": r.dd_waves}

    def step(self, control, z, noise=None, u_resample=float("nan")):
        ctl = _f64(control, (2,))
        zz = _f64(z, (self.nl, 2))
        nz = None if noise is None else _f64(noise, (self.n, 3))
        res = PFResult()
        check(self._lib.slam_pf_step(self._h, dptr(ctl), dptr(zz), dptr(nz), float(u_resample),
                                     C.byref(res)), "slam_pf_step")
        out = self._res(res)
        self.resample_next = out["resample_next"]
        self._confirm_ess(out)
        self.last = out
        return out

    def resample(self, u_resample=float("nan"), force=False):
        flag = C.c_int32(0)
        check(self._lib.slam_pf_resample(self._h, float(u_resample), int(bool(force)),
                                         C.byref(flag)), "slam_pf_resample")
        if flag.value:
            self.resample_next = False
        return bool(flag.value)

    def predict(self, control, noise=None):
        ctl = _f64(control, (2,))
        nz = None if noise is None else _f64(noise, (self.n, 3))
        check(self._lib.slam_pf_predict(self._h, dptr(ctl), dptr(nz)), "slam_pf_predict")

    def update(self, z):
        zz = _f64(z, (self.nl, 2))
        res = PFResult()
        check(self._lib.slam_pf_update(self._h, dptr(zz), C.byref(res)), "slam_pf_update")
        out = self._res(res)
        self.resample_next = out["resample_next"]
        self._confirm_ess(out)
        return out

    def resample_indices(self, u_resample):
        idx = np.empty(self.n, dtype=np.int64)
        ns = C.c_int32(0)
        check(self._lib.slam_pf_resample_indices(self._h, float(u_resample),
                                                 idx.ctypes.data_as(_lib._I64), C.byref(ns)),
              "slam_pf_resample_indices")
        return idx, ns.value

    def weight_sum(self):
        s = C.c_double(0.0)
        check(self._lib.slam_pf_weight_sum(self._h, C.byref(s)), "slam_pf_weight_sum")
        return s.value

    # ------------------------------------------------------ device-resident
    def load_observations(self, z_all):
        z_all = _f64(z_all).reshape(-1, self.nl, 2)
        check(self._lib.slam_pf_load_observations(self._h, z_all.shape[0], dptr(z_all)),
              "slam_pf_load_observations")
        self._z_steps = z_all.shape[0]

    def prepare_graphs(self):
        """Capture every step graph ``run`` replays (both parities; 1-, 2-, 4-
        and 8-step graphs) now, so that no capture lands in a timed run;
        returns the capture time in ms."""
        ms = C.c_double(0.0)
        check(self._lib.slam_pf_prepare_graphs(self._h, C.byref(ms)), "slam_pf_prepare_graphs")
        return ms.value

    def run(self, first_step, controls, want_results=True, confirm_ess=False):
        """Device-resident steps [first_step, first_step + len(controls)) from
        the loaded observations (hipGraph replays, no host decision).  Each
        result carries ``ess_near``: the device's ESS fell within
        ESS_CONFIRM_BAND of ESS_TH, where the reference's `1 / (pw @ pw.T)`
        (BLAS order) could decide the next resample differently.

        ``confirm_ess=True`` (parity batches): one replayed step at a time, and
        every ess_near step's decision re-formed on the host by the reference's
        own expression before the next step runs (as ``step`` does); results
        then carry ``ess_confirmed`` / ``ess_host`` like ``step``'s."""
        controls = _f64(controls).reshape(-1, 2)
        k = controls.shape[0]
        if confirm_ess:
            outs = []
            for i in range(k):
                res = (PFResult * 1)()
                check(self._lib.slam_pf_run(self._h, int(first_step) + i, 1, dptr(controls[i:i + 1]),
                                            res), "slam_pf_run")
                out = self._res(res[0])
                self.resample_next = out["resample_next"]
                if out["ess_near"]:
                    self._confirm_ess(out)
                else:
                    out["ess_confirmed"] = False
                outs.append(out)
            return RunResults.from_dicts(outs) if want_results else None
        res = (PFResult * k)()
        check(self._lib.slam_pf_run(self._h, int(first_step), k, dptr(controls), res),
              "slam_pf_run")
        self.resample_next = bool(res[k - 1].resample_next)
        return RunResults(res) if want_results else None

    def set_ess_band(self, band):
        """Relative band of result['ess_near'] (and of the drop-in's host
        confirmation); default 1e-9."""
        check(self._lib.slam_pf_set_ess_band(self._h, float(band)), "slam_pf_set_ess_band")
        self.ESS_CONFIRM_BAND = float(band)

    # ------------------------------------------------ NumPy stream on device
    def use_numpy_stream(self, state=None):
        """Draw the reference's noise from NumPy's RandomState stream on the
        device, starting from `state` (np.random's global state when None):
        each step then draws [rand() if resampling] -> mvn(0, Q, NP) ->
        mvn(0, R, NL) in the reference's order (particle_filter.py:214, :165,
        :152) and observes the landmarks from the true pose on the device."""
        key, pos, hg, g = state_fields(state)
        rf = _f64(numpy_noise_factor(self.r))
        check(self._lib.slam_pf_set_rng_mt19937(self._h, key.ctypes.data_as(_lib._U32), pos, hg, g,
                                                dptr(rf)), "slam_pf_set_rng_mt19937")
        self.mt = True

    def rng_ring_info(self):
        """The device stream's word ring (slam_pf_rng_mt19937_info): bytes,
        segments per refill round, words per segment, requests per round."""
        out = (C.c_int64 * 4)()
        check(self._lib.slam_pf_rng_mt19937_info(self._h, out), "slam_pf_rng_mt19937_info")
        return dict(ring_bytes=out[0], segments=out[1], segment_words=out[2], requests_per_round=out[3])

    def rng_state(self):
        """The device stream's state as an np.random.get_state() tuple."""
        key = np.empty(624, dtype=np.uint32)
        pos, hg, g = C.c_int32(0), C.c_int32(0), C.c_double(0.0)
        check(self._lib.slam_pf_get_rng_mt19937(self._h, key.ctypes.data_as(_lib._U32), C.byref(pos),
                                                C.byref(hg), C.byref(g)), "slam_pf_get_rng_mt19937")
        return ("MT19937", key, pos.value, hg.value, g.value)

    @staticmethod
    def truth_input(x_true):
        """(x, y, cos, sin) of a (3, 1) true pose as world2robot forms them
        (mylib/transform.py:31-35)."""
        x_true = np.asarray(x_true, dtype=np.float64).reshape(3, 1)
        yaw = BASE_ANG - x_true[2, 0]
        return np.array([x_true[0, 0], x_true[1, 0], np.cos(yaw), np.sin(yaw)])

    def step_truth(self, control, x_true, want_z=False):
        """One step with the device stream: the observation of x_true is
        simulated on the device (z returned with want_z)."""
        ctl = _f64(control, (2,))
        t4 = self.truth_input(x_true)
        z = np.empty((self.nl, 2)) if want_z else None
        res = PFResult()
        check(self._lib.slam_pf_step_truth(self._h, dptr(ctl), dptr(t4), dptr(z), C.byref(res)),
              "slam_pf_step_truth")
        out = self._res(res)
        if want_z:
            out["z"] = z
        self.resample_next = out["resample_next"]
        self._confirm_ess(out)
        self.last = out
        return out

    def load_truth(self, poses):
        """True poses [k][3] of a device-resident batch (run() then simulates
        every step's observation on the device)."""
        poses = _f64(poses).reshape(-1, 3)
        t4 = np.ascontiguousarray(np.stack([self.truth_input(p) for p in poses]))
        check(self._lib.slam_pf_load_truth(self._h, t4.shape[0], dptr(t4)), "slam_pf_load_truth")
        self._truth_steps = t4.shape[0]

    def set_scan_merged(self, on=True):
        """Exact cumsum of a resample step in one launch (default where the
        grid is co-resident) or two; the results are bit-identical."""
        check(self._lib.slam_pf_set_scan_merged(self._h, int(bool(on))), "slam_pf_set_scan_merged")

    def enable_timing(self, on=True):
        check(self._lib.slam_pf_enable_timing(self._h, int(bool(on))), "slam_pf_enable_timing")

    def timing(self, kernel):
        ms = C.c_double(0.0)
        cnt = C.c_int64(0)
        check(self._lib.slam_pf_timing(self._h, int(kernel), C.byref(ms), C.byref(cnt)),
              "slam_pf_timing")
        return ms.value, cnt.value
