"""Sharded particle filter with a device-resident step (BASELINE config 3):
a handle on libslam_hip's slam_dist_* entry points.

One filter of ``n_global`` particles split into contiguous shards
(slam_dist_shard_range).  ``DistFilter(..., world=W)`` holds every shard in
this process on one GPU (LOCAL: tests, or several shards per GPU);
``DistFilter(..., world=W, rank=r, comm=...)`` holds rank r's shard, one
process per GPU, and bootstraps the peer-memory exchange through an RCCL
communicator (``Comm``) or any all-gather of bytes (``all_gather``).  No
PyTorch anywhere: the exchanges are device-side pushes over xGMI inside the
step's kernels, the bootstrap is RCCL from the library.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import PFResult, check, dptr
from .pf import DeviceParticleFilter, RunResults, _f64, make_config


class Comm:
    """An RCCL communicator (slam_comm_*).  ``unique_id()`` on one rank; the
    128 bytes reach every rank through the caller's bootstrap (e.g. the
    torch.distributed store, or a file)."""

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(_lib.load().slam_comm_unique_id(buf), "slam_comm_unique_id")
        return buf.raw

    def __init__(self, uid: bytes, world: int, rank: int, device: int = 0):
        self._lib = _lib.load()
        h = C.c_void_p()
        check(self._lib.slam_comm_create(uid, int(world), int(rank), int(device), C.byref(h)),
              "slam_comm_create")
        self._h = h
        self.world, self.rank = int(world), int(rank)

    def all_gather_bytes(self, data: bytes) -> list:
        n = len(data)
        out = C.create_string_buffer(n * self.world)
        check(self._lib.slam_comm_all_gather_host(self._h, data, out, n), "slam_comm_all_gather_host")
        return [out.raw[k * n:(k + 1) * n] for k in range(self.world)]

    def close(self):
        if getattr(self, "_h", None):
            self._lib.slam_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def shard_range(n_global, world, rank):
    g, n = C.c_int64(0), C.c_int64(0)
    check(_lib.load().slam_dist_shard_range(int(n_global), int(world), int(rank), C.byref(g),
                                            C.byref(n)), "slam_dist_shard_range")
    return g.value, n.value


class DistFilter:
    """One particle filter over ``world`` shards.

    Every wait on a peer is bounded; one that expires raises (SLAM_ERR_COMM)
    and leaves this filter permanently unusable -- every later step or run
    fails at once.  Recover by closing and recreating the DistFilter on every
    rank (slam_hip.h, slam_dist_step)."""

    def __init__(self, n_global, landmarks, *, world, rank=None, comm=None, all_gather=None,
                 device=0, connect=True, **cfg_kw):
        """connect=False (one rank per process): create the shard and its
        exchange region only; the caller then gathers ``export_handle()`` from
        every rank and calls ``connect(blobs)`` -- so a harness can agree on
        every rank's local success before and after the one collective."""
        lib = _lib.load()
        self._lib = lib
        self.n_global, self.world = int(n_global), int(world)
        self.lm = _f64(landmarks).reshape(-1, 2)
        self.nl = self.lm.shape[0]
        cfg = make_config(self.n_global, **cfg_kw)
        self.cfg = cfg
        self.ranks = list(range(self.world)) if rank is None else [int(rank)]
        self._shards = []
        self._d = None
        try:
            for r in self.ranks:
                g, n = shard_range(self.n_global, self.world, r)
                h = C.c_void_p()
                check(lib.slam_pf_create_dist_shard(C.byref(cfg), n, self.n_global, g, self.nl,
                                                    dptr(self.lm), int(device), C.byref(h)),
                      "slam_pf_create_dist_shard")
                self._shards.append((h, g, n))
            arr = (C.c_void_p * len(self._shards))(*[h.value for h, _, _ in self._shards])
            d = C.c_void_p()
            check(lib.slam_dist_create(arr, len(self._shards), self.world, self.ranks[0], C.byref(d)),
                  "slam_dist_create")
            self._d = d
            if rank is not None and connect:
                if comm is not None:
                    check(lib.slam_dist_connect_comm(d, comm._h), "slam_dist_connect_comm")
                else:
                    size = C.c_int64(0)
                    check(lib.slam_dist_handle_size(C.byref(size)), "slam_dist_handle_size")
                    mine = C.create_string_buffer(size.value)
                    check(lib.slam_dist_export(d, mine), "slam_dist_export")
                    blobs = all_gather(mine.raw)
                    allb = C.create_string_buffer(b"".join(blobs), size.value * self.world)
                    check(lib.slam_dist_connect(d, allb), "slam_dist_connect")
        except Exception:
            self.close()
            raise
        self.resample_next = False
        self.collective = False

    def export_handle(self) -> bytes:
        """This rank's exchange-region IPC handle (slam_dist_export)."""
        size = C.c_int64(0)
        check(self._lib.slam_dist_handle_size(C.byref(size)), "slam_dist_handle_size")
        mine = C.create_string_buffer(size.value)
        check(self._lib.slam_dist_export(self._d, mine), "slam_dist_export")
        return mine.raw

    def connect(self, blobs):
        """Open every peer's exchange region (blobs: every rank's
        export_handle(), rank order; slam_dist_connect preflights peer access)."""
        size = len(blobs[0])
        allb = C.create_string_buffer(b"".join(blobs), size * self.world)
        check(self._lib.slam_dist_connect(self._d, allb), "slam_dist_connect")

    def use_collectives(self, comm=None):
        """Exchange by collectives instead of peer-memory stores
        (slam_dist_set_collective): RCCL through ``comm`` (one rank per
        process; no connect needed -- the fallback when a peer's region cannot
        be mapped), or device copies between the held shards (LOCAL, comm
        None).  Steps are then host-orchestrated, without hipGraphs."""
        check(self._lib.slam_dist_set_collective(self._d, comm._h if comm is not None else None),
              "slam_dist_set_collective")
        self.collective = True

    def close(self):
        if getattr(self, "_d", None):
            self._lib.slam_dist_destroy(self._d)
            self._d = None
        for h, _, _ in getattr(self, "_shards", []):
            self._lib.slam_pf_destroy(h)
        self._shards = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def step(self, control, z):
        res = PFResult()
        check(self._lib.slam_dist_step(self._d, dptr(_f64(control, (2,))), dptr(_f64(z, (self.nl, 2))),
                                       C.byref(res)), "slam_dist_step")
        out = DeviceParticleFilter._res(res)
        self.resample_next = out["resample_next"]
        return out

    def load_observations(self, z_all):
        z_all = _f64(z_all).reshape(-1, self.nl, 2)
        check(self._lib.slam_dist_load_observations(self._d, z_all.shape[0], dptr(z_all)),
              "slam_dist_load_observations")

    def prepare_graphs(self):
        """DeviceParticleFilter.prepare_graphs for the sharded step."""
        ms = C.c_double(0.0)
        check(self._lib.slam_dist_prepare_graphs(self._d, C.byref(ms)), "slam_dist_prepare_graphs")
        return ms.value

    def run(self, first_step, controls, want_results=True):
        controls = _f64(controls).reshape(-1, 2)
        k = controls.shape[0]
        res = (PFResult * k)()
        check(self._lib.slam_dist_run(self._d, int(first_step), k, dptr(controls), res), "slam_dist_run")
        self.resample_next = bool(res[k - 1].resample_next)
        return RunResults(res) if want_results else None

    def set_merged(self, on=None):
        """Resample exchange in one launch (True) or five (False); None only
        reports.  Returns the form in use."""
        act = C.c_int32(0)
        check(self._lib.slam_dist_set_merged(self._d, -1 if on is None else int(bool(on)),
                                             C.byref(act)), "slam_dist_set_merged")
        return bool(act.value)

    def enable_timing(self, on=True):
        """HIP events around the fused kernel of every held shard (disables graphs)."""
        for h, _, _ in self._shards:
            check(self._lib.slam_pf_enable_timing(h, int(bool(on))), "slam_pf_enable_timing")

    def timing(self, kernel=0):
        """(total ms, launches) of the first held shard (slam_pf_timing kernel ids)."""
        ms, cnt = C.c_double(0.0), C.c_int64(0)
        check(self._lib.slam_pf_timing(self._shards[0][0], int(kernel), C.byref(ms), C.byref(cnt)),
              "slam_pf_timing")
        return ms.value, cnt.value

    def get_state(self):
        """Concatenated state of the held shards (x, y, th, w)."""
        parts = []
        for h, _, n in self._shards:
            out = [np.empty(n) for _ in range(4)]
            check(self._lib.slam_pf_get_state(h, *[dptr(a) for a in out]), "slam_pf_get_state")
            parts.append(out)
        return tuple(np.concatenate([p[k] for p in parts]) for k in range(4))
