"""Test double of one particle-filter shard on the CPU (NumPy), with the phase
methods and exchange-buffer shapes of slamhip.shard.DeviceShard.  Used to run
the product orchestration (slamhip.shard.ShardedFilter) under torch.distributed
gloo on CPU.  Its internal payloads are simpler than the device's (the
"special list" it exports is its whole weight array, so the receiving ranks can
form the global sequential cumsum directly), but every exchange goes through
the same all-gather / all-to-all-v calls, in the same order, with the same
dtypes.  Arithmetic follows the oracle (oracle/pf_oracle.py)."""
import numpy as np
import torch

import pf_oracle as po


class NumpyShard:
    def __init__(self, n_local, n_global, gbase, landmarks, *, dt=0.1, motion="linear"):
        self.n, self.n_global, self.gbase = n_local, n_global, gbase
        self.p = po.PFParams(period_ms=dt * 1000, n_particles=n_global, landmarks=landmarks,
                             motion=motion)
        x0 = self.p.x0
        self.x = np.full(n_local, x0[0])
        self.y = np.full(n_local, x0[1])
        self.th = np.full(n_local, x0[2])
        self.w = np.full(n_local, 1 / n_global)
        self.ref = x0.copy()
        self.nchunks = (n_local + po.NP_SUM_CHUNK - 1) // po.NP_SUM_CHUNK
        self.spec_bytes = 8
        self.item_bytes = 40

    def close(self):
        pass

    def get_state(self):
        return self.x.copy(), self.y.copy(), self.th.copy(), self.w.copy()

    # ---- phases
    def begin(self, control, z, noise, u, resample):
        self.control, self.z, self.noise, self.u = control, np.asarray(z), noise, u
        self.resampled = bool(resample)

    def scan_local(self):
        return torch.tensor([float(np.sum(self.w))], dtype=torch.float64)

    def classify(self, totals, rank, world):
        return torch.tensor([self.n, 0], dtype=torch.int64)

    def export_specials(self, count, cap):
        t = torch.zeros((cap, 1), dtype=torch.int64)
        t[:count, 0] = torch.from_numpy(self.w.view(np.int64).copy())
        return t

    def fold(self, lists, cap, meta_host, world, rank):
        ws = [lists.reshape(world, cap)[r, :meta_host[r, 0]].numpy().view(np.float64)
              for r in range(world)]
        wall = np.concatenate(ws)
        self.cum = np.cumsum(wall)                       # particle_filter.py:212, global order

    def plan(self, gb):
        N = self.n_global
        pos = po.resample_positions(N, self.u * (1 / N))
        hi_all = np.searchsorted(pos, self.cum, side="right")   # #positions <= c_j
        hi_all[-1] = N
        lo_all = np.concatenate([[0], hi_all[:-1]])
        lo = lo_all[self.gbase:self.gbase + self.n]
        hi = hi_all[self.gbase:self.gbase + self.n]
        self.items = []
        counts = np.zeros(len(gb) - 1, dtype=np.int64)
        for d in range(len(gb) - 1):
            sel = np.nonzero((hi > gb[d]) & (lo < gb[d + 1]))[0]
            for j in sel:
                self.items.append((self.x[j], self.y[j], self.th[j],
                                   max(lo[j], gb[d]), min(hi[j], gb[d + 1])))
            counts[d] = len(sel)
        return counts

    def export_items(self):
        a = np.zeros((len(self.items), 5), dtype=np.int64)
        for k, (x, y, th, lo, hi) in enumerate(self.items):
            a[k, :3] = np.array([x, y, th]).view(np.int64)
            a[k, 3:] = (lo, hi)
        return torch.from_numpy(a)

    def import_items(self, items):
        a = items.numpy()
        f = a[:, :3].copy().view(np.float64)
        for k in range(a.shape[0]):
            lo, hi = a[k, 3] - self.gbase, a[k, 4] - self.gbase
            self.x[lo:hi], self.y[lo:hi], self.th[lo:hi] = f[k, 0], f[k, 1], f[k, 2]
        self.w[:] = 1 / self.n_global

    def predict_update(self):
        p = self.p
        v, om = self.control
        if p.motion == "linear":
            xn, yn, tn = po.motion_linear(self.x, self.y, self.th, p.dt, v, om)
            self.x, self.y, self.th = (xn + self.noise[:, 0], yn + self.noise[:, 1],
                                       tn + self.noise[:, 2])
        else:
            self.x, self.y, self.th = po.motion_velocity(self.x, self.y, self.th, v, om, p.dt,
                                                         p.alphas, self.noise)
        f = po.landmark_factors(self.x, self.y, self.th, p.lm, self.z, p.r)
        self.w_un = self.w * f.prod(axis=1)
        return torch.from_numpy(po.chunk_partials(self.w_un))

    def normalize(self, all_parts):
        s = 0.0
        for v in all_parts.reshape(-1).numpy():
            s += float(v)                                 # buffer partials left to right
        self.s = s
        w = self.w_un / s
        w[np.isnan(w)] = 1 / self.n_global
        self.w = w
        i = int(np.argmax(w))
        d = np.stack([self.x - self.ref[0], self.y - self.ref[1], self.th - self.ref[2]])
        rec = np.concatenate([[w[i], self.gbase + i, w.sum(), (w * w).sum()],
                              (d * w).sum(axis=1), [(w * d[a] * d[b]).sum() for a in range(3)
                                                    for b in range(a, 3)],
                              [self.x[i], self.y[i], self.th[i]]])
        return torch.from_numpy(rec)

    def finish(self, all_recs, world):
        R = all_recs.reshape(world, -1).numpy()
        win = 0
        for k in range(1, world):
            if R[k, 0] > R[win, 0]:
                win = k                                   # first index on ties (rank order)
        sw, sw2 = R[:, 2].sum(), R[:, 3].sum()
        m1 = R[:, 4:7].sum(axis=0) / sw
        m2 = R[:, 7:13].sum(axis=0) / sw
        full = np.array([[m2[0], m2[1], m2[2]], [m2[1], m2[3], m2[4]], [m2[2], m2[4], m2[5]]])
        cov = full - np.outer(m1, m1)
        x_est = R[win, 13:16].copy()
        self.ref = x_est.copy()
        ess = 1 / sw2
        return {"x_est": x_est, "cov": cov, "max_val": R[win, 0], "max_idx": int(R[win, 1]),
                "ess": ess, "weight_sum": self.s, "resampled": self.resampled,
                "resample_next": bool(ess < self.n_global / 100.0)}
