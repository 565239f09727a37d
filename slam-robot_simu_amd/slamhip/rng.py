"""NumPy's legacy RandomState stream on the GPU (libslam_hip's slam_mt_*).

The reference draws all of its noise from np.random's global RandomState
(particle_filter.py:152, :165, :214; motion_model.py:46-48).  DeviceRandomState
holds an MT19937 state on the device and draws exactly NumPy's numbers from it:
random_sample (two words per double) and standard_normal (the polar method with
the cached second normal, glibc's log).  State round-trips with
np.random.get_state() / set_state().
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, dptr


def state_fields(state=None):
    """(key uint32[624], pos, has_gauss, gauss) of a RandomState / get_state()
    tuple (the global generator's when None)."""
    if state is None:
        state = np.random.get_state()
    elif isinstance(state, np.random.RandomState):
        state = state.get_state()
    name, key, pos, has_gauss, gauss = state[:5]
    if name != "MT19937":
        raise ValueError(f"not an MT19937 state: {name}")
    key = np.ascontiguousarray(key, dtype=np.uint32)
    if key.shape != (624,):
        raise ValueError("MT19937 key must hold 624 words")
    return key, int(pos), int(has_gauss), float(gauss)


def _u32(a):
    return a.ctypes.data_as(_lib._U32)


class DeviceRandomState:
    """A RandomState whose draws run on one GPU."""

    def __init__(self, state=None, device=0):
        lib = _lib.load()
        key, pos, hg, g = state_fields(state)
        h = C.c_void_p()
        check(lib.slam_mt_create(_u32(key), pos, hg, g, int(device), C.byref(h)), "slam_mt_create")
        self._h = h
        self._lib = lib

    def close(self):
        if getattr(self, "_h", None):
            self._lib.slam_mt_destroy(self._h)
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

    def set_state(self, state):
        key, pos, hg, g = state_fields(state)
        check(self._lib.slam_mt_set_state(self._h, _u32(key), pos, hg, g), "slam_mt_set_state")

    def get_state(self):
        key = np.empty(624, dtype=np.uint32)
        pos, hg, g = C.c_int32(0), C.c_int32(0), C.c_double(0.0)
        check(self._lib.slam_mt_get_state(self._h, _u32(key), C.byref(pos), C.byref(hg), C.byref(g)),
              "slam_mt_get_state")
        return ("MT19937", key, pos.value, hg.value, g.value)

    def random_sample(self, n):
        out = np.empty(int(n))
        check(self._lib.slam_mt_random_sample(self._h, out.size, dptr(out)), "slam_mt_random_sample")
        return out

    def standard_normal(self, n):
        out = np.empty(int(n))
        check(self._lib.slam_mt_standard_normal(self._h, out.size, dptr(out)),
              "slam_mt_standard_normal")
        return out


def glibc_log(x):
    """glibc's log as the device evaluates it (the host copy of the restatement)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    check(_lib.load().slam_glibc_log(x.size, dptr(x), dptr(out)), "slam_glibc_log")
    return out


def jump_window(window, n_words):
    """The 624-word MT19937 window n_words further on (host jump-ahead)."""
    w = np.ascontiguousarray(window, dtype=np.uint32)
    out = np.empty(624, dtype=np.uint32)
    check(_lib.load().slam_mt_jump_window(_u32(w), int(n_words), _u32(out)), "slam_mt_jump_window")
    return out
