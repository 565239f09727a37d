"""Sharded particle filter: one filter's particles split over several GPUs.

BASELINE config 3 (8 x 1,048,576 particles).  Each rank owns a contiguous
shard; per step the ranks exchange only small buffers:

  A  all-gather of approximate shard weight totals      (1 f64 / rank)
  B  all-gather of the exact-cumsum special lists        (~tens of 32-B entries)
  C  all-to-all-v of resampled particles                 (40 B / moved particle)
  D  all-gather of np.sum buffer partials                (1 f64 / 8192 particles)
  E  all-gather of reduction records                     (136 B / rank)

A-C run only on resampling steps.  D/E replace "an all-reduce for the weight
normalisation": gathering the partials and folding them in rank order keeps
the result bit-identical to the single-array reference order, which an RCCL
sum would not.

The orchestration below is written once against two small interfaces:
``comm`` (all_gather / all_to_all_v over torch tensors -- torch.distributed,
i.e. RCCL over xGMI on MI355X, or a same-process emulation) and the shard
phase methods (``DeviceShard`` here: the C-ABI on the GPU).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import PFConfig, PFResult, check, dptr
from .pf import DeviceParticleFilter, numpy_noise_factor, _f64


# --------------------------------------------------------------- communicators
class LocalComm:
    """All shards live in this process (tests, or several shards on one GPU)."""

    def __init__(self, world):
        self.world = world

    def all_gather(self, tensors):
        import torch
        g = torch.stack([t.reshape(-1) for t in tensors])
        return [g.clone() for _ in tensors]

    def all_to_all_v(self, sends, counts):
        """sends[s]: rows for every destination, grouped by destination in
        rank order; counts[s][d] rows from s to d."""
        import torch
        out = []
        for d in range(self.world):
            parts = []
            for s in range(self.world):
                off = int(sum(counts[s][:d]))
                parts.append(sends[s][off:off + int(counts[s][d])])
            out.append(torch.cat(parts))
        return out


class TorchComm:
    """One shard per process, torch.distributed (nccl = RCCL on ROCm, or gloo)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def all_gather(self, tensors):
        import torch
        (t,) = tensors
        t = t.reshape(-1).contiguous()
        out = torch.empty(self.world * t.numel(), dtype=t.dtype, device=t.device)
        self.dist.all_gather_into_tensor(out, t, group=self.group)
        return [out.view(self.world, t.numel())]

    def all_to_all_v(self, sends, counts):
        import torch
        (send,) = sends
        (mine,) = counts
        c = torch.tensor(np.asarray(mine, dtype=np.int64), device=send.device)
        allc = self.all_gather([c])[0].cpu().numpy()
        recv_counts = [int(allc[s][self.rank]) for s in range(self.world)]
        out = torch.empty((sum(recv_counts),) + tuple(send.shape[1:]), dtype=send.dtype,
                          device=send.device)
        self.dist.all_to_all_single(out, send.contiguous(), recv_counts,
                                    [int(v) for v in mine], group=self.group)
        return [out]


# ---------------------------------------------------------------- GPU shard
class DeviceShard:
    """Phase methods of one shard on one GPU (slam_pf_shard_* of the C-ABI).
    Exchange buffers are torch CUDA tensors on the current stream."""

    def __init__(self, n_local, n_global, gbase, landmarks, *, dt=0.1, q=None, r=None,
                 x0=(10.0, 0.0, np.pi / 2), motion="linear", likelihood="product",
                 alphas=(0.1,) * 6, seed=0, device=0):
        import torch
        self.torch = torch
        lib = _lib.load()
        self.lib = lib
        self.n, self.n_global, self.gbase = int(n_local), int(n_global), int(gbase)
        self.lm = _f64(landmarks).reshape(-1, 2)
        self.nl = self.lm.shape[0]
        q = np.diag([0.03, 0.03, np.deg2rad(2.0)]) ** 2 if q is None else np.asarray(q, float)
        r = np.diag([0.3, 0.3]) ** 2 if r is None else np.asarray(r, float)
        cfg = PFConfig()
        cfg.dt = float(dt)
        cfg.ess_threshold = self.n_global / 100.0
        cfg.r_cov[:] = [float(v) for v in r.ravel()]
        cfg.q_factor[:] = [float(v) for v in numpy_noise_factor(q).ravel()]
        cfg.alphas[:] = [float(v) for v in alphas]
        cfg.x0[:] = [float(v) for v in x0]
        cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        cfg.motion = _lib.MOTION[motion]
        cfg.likelihood = _lib.LIKELIHOOD[likelihood]
        self.cfg = cfg
        self.device = torch.device("cuda", device)
        h = C.c_void_p()
        check(lib.slam_pf_create_shard(C.byref(cfg), self.n, self.n_global, self.gbase, self.nl,
                                       dptr(self.lm), int(device), C.byref(h)),
              "slam_pf_create_shard")
        self._h = h
        stream = torch.cuda.current_stream(self.device)
        check(lib.slam_pf_set_stream(h, C.c_void_p(stream.cuda_stream), 1), "slam_pf_set_stream")
        sizes = np.zeros(4, dtype=np.int64)
        check(lib.slam_pf_shard_sizes(h, sizes.ctypes.data_as(_lib._I64)), "slam_pf_shard_sizes")
        self.nchunks, self.rec_bytes, self.spec_bytes, self.item_bytes = (int(v) for v in sizes)

    def close(self):
        if getattr(self, "_h", None):
            self.lib.slam_pf_destroy(self._h)
            self._h = None

    def _empty(self, shape, dtype):
        return self.torch.empty(shape, dtype=dtype, device=self.device)

    @staticmethod
    def _p(t):
        return C.c_void_p(t.data_ptr())

    def set_state(self, x=None, y=None, th=None, w=None):
        arrs = [None if a is None else _f64(a, (self.n,)) for a in (x, y, th, w)]
        check(self.lib.slam_pf_set_state(self._h, *[dptr(a) for a in arrs]), "slam_pf_set_state")

    def get_state(self):
        out = [np.empty(self.n) for _ in range(4)]
        check(self.lib.slam_pf_get_state(self._h, *[dptr(a) for a in out]), "slam_pf_get_state")
        return tuple(out)

    # -- phases
    def begin(self, control, z, noise, u, resample):
        ctl = _f64(control, (2,))
        zz = _f64(z, (self.nl, 2))
        nz = None if noise is None else _f64(noise, (self.n, 3))
        check(self.lib.slam_pf_shard_begin(self._h, dptr(ctl), dptr(zz), dptr(nz), float(u),
                                           int(bool(resample))), "slam_pf_shard_begin")

    def scan_local(self):
        t = self._empty((1,), self.torch.float64)
        check(self.lib.slam_pf_shard_scan_local(self._h, self._p(t)), "slam_pf_shard_scan_local")
        return t

    def classify(self, totals, rank, world):
        meta = self._empty((2,), self.torch.int64)
        check(self.lib.slam_pf_shard_classify(self._h, self._p(totals.contiguous()), rank, world,
                                              self._p(meta)), "slam_pf_shard_classify")
        return meta

    def export_specials(self, count, cap):
        words = self.spec_bytes // 8
        t = self.torch.zeros((cap, words), dtype=self.torch.int64, device=self.device)
        check(self.lib.slam_pf_shard_export_specials(self._h, int(count), self._p(t)),
              "slam_pf_shard_export_specials")
        return t

    def fold(self, lists, cap, meta_host, world, rank):
        meta = np.ascontiguousarray(meta_host, dtype=np.int64)
        check(self.lib.slam_pf_shard_fold(self._h, self._p(lists.contiguous()), int(cap),
                                          meta.ctypes.data_as(_lib._I64), world, rank),
              "slam_pf_shard_fold")

    def plan(self, gb):
        gb = np.ascontiguousarray(gb, dtype=np.int64)
        counts = np.zeros(len(gb) - 1, dtype=np.int64)
        check(self.lib.slam_pf_shard_plan(self._h, gb.ctypes.data_as(_lib._I64), len(gb) - 1,
                                          counts.ctypes.data_as(_lib._I64)), "slam_pf_shard_plan")
        self._n_send = int(counts.sum())
        return counts

    def export_items(self):
        words = self.item_bytes // 8
        t = self._empty((max(self._n_send, 1), words), self.torch.int64)
        check(self.lib.slam_pf_shard_export_items(self._h, self._p(t)), "slam_pf_shard_export_items")
        return t[:self._n_send]

    def import_items(self, items):
        check(self.lib.slam_pf_shard_import_items(self._h, self._p(items.contiguous()),
                                                  int(items.shape[0])), "slam_pf_shard_import_items")

    def predict_update(self):
        t = self._empty((self.nchunks,), self.torch.float64)
        check(self.lib.slam_pf_shard_predict_update(self._h, self._p(t)),
              "slam_pf_shard_predict_update")
        return t

    def normalize(self, all_parts):
        rec = self._empty((self.rec_bytes // 8,), self.torch.int64)
        flat = all_parts.reshape(-1).contiguous()
        check(self.lib.slam_pf_shard_normalize(self._h, self._p(flat), int(flat.numel()),
                                               self._p(rec)), "slam_pf_shard_normalize")
        return rec

    def finish(self, all_recs, world):
        res = PFResult()
        check(self.lib.slam_pf_shard_finish(self._h, self._p(all_recs.contiguous()), world,
                                            C.byref(res)), "slam_pf_shard_finish")
        return DeviceParticleFilter._res(res)


# ------------------------------------------------------------ orchestration
class ShardedFilter:
    """One filter over ``world`` equal shards.  ``shards``: the shards this
    process holds (all of them with LocalComm, one with TorchComm), with their
    global ranks in ``ranks``."""

    def __init__(self, shards, ranks, comm, n_global):
        self.shards, self.ranks, self.comm = list(shards), list(ranks), comm
        self.world = comm.world
        if isinstance(comm, LocalComm):
            # LocalComm stacks its inputs in list order: shards[i] must be rank i
            if self.ranks != list(range(self.world)):
                raise ValueError("LocalComm needs every shard, in rank order (ranks == 0..world-1)")
        self.n_global = int(n_global)
        n = self.shards[0].n
        assert all(s.n == n for s in self.shards) and n * self.world == self.n_global, \
            "equal shard sizes required"
        self.n_local = n
        self.gb = np.arange(self.world + 1, dtype=np.int64) * n
        self.resample_next = False

    def step(self, control, z, noise=None, u_resample=float("nan")):
        """noise: (n_global, 3) host array (NumPy stream) or None (device RNG)."""
        res = self.resample_next
        for s, r in zip(self.shards, self.ranks):
            nz = None if noise is None else noise[self.gb[r]:self.gb[r + 1]]
            s.begin(control, z, nz, u_resample, res)
        if res:
            tot = [s.scan_local() for s in self.shards]
            tot_g = self.comm.all_gather(tot)
            metas = [s.classify(t.reshape(-1), r, self.world)
                     for s, t, r in zip(self.shards, tot_g, self.ranks)]
            meta_g = self.comm.all_gather(metas)
            meta_host = meta_g[0].reshape(self.world, 2).cpu().numpy()
            cap = max(int(meta_host[:, 0].max()), 1)
            lists = [s.export_specials(meta_host[r, 0], cap) for s, r in zip(self.shards, self.ranks)]
            lists_g = self.comm.all_gather(lists)
            for s, L, r in zip(self.shards, lists_g, self.ranks):
                s.fold(L, cap, meta_host, self.world, r)
            counts = [s.plan(self.gb) for s in self.shards]
            items = [s.export_items() for s in self.shards]
            recv = self.comm.all_to_all_v(items, counts)
            for s, it in zip(self.shards, recv):
                s.import_items(it)
        parts = [s.predict_update() for s in self.shards]
        parts_g = self.comm.all_gather(parts)
        recs = [s.normalize(p) for s, p in zip(self.shards, parts_g)]
        recs_g = self.comm.all_gather(recs)
        outs = [s.finish(R, self.world) for s, R in zip(self.shards, recs_g)]
        self.resample_next = outs[0]["resample_next"]
        return outs[0]

    def get_state(self):
        """Concatenated state of the shards held here (LocalComm: the whole filter)."""
        parts = [s.get_state() for s in self.shards]
        return tuple(np.concatenate([p[k] for p in parts]) for k in range(4))

    def close(self):
        for s in self.shards:
            s.close()
