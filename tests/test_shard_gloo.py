"""The sharded-filter orchestration (slamhip.shard.ShardedFilter + TorchComm)
under torch.distributed gloo, world size 2, on CPU, with NumPy shard doubles
(tests/shard_double.py).  The 2-rank run must equal the single-array oracle
step for step: resampling decisions, argmax index, estimate, weights.  The
GPU counterpart (tests/test_gpu_shard.py) runs the same orchestration over the
HIP shards."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ORACLE, PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(n_global, nl, steps, seed):
    import sys
    sys.path.insert(0, ORACLE)
    import pf_oracle as po
    rs = np.random.RandomState(seed)
    lm = rs.uniform(-10, 10, (nl, 2))
    p = po.PFParams(n_particles=n_global, landmarks=lm)
    world = po.PFWorld(p)
    np.random.seed(seed + 1)
    zs, noises, us = [], [], []
    for _ in range(steps):
        world.advance()
        noises.append(np.random.multivariate_normal([0.0, 0.0, 0.0], p.q, n_global))
        zs.append(world.observe())
        us.append(np.random.rand())
    return lm, zs, noises, us, p


def _worker(rank, world, port, n_local, nl, steps, q):
    import sys
    for pth in (PKG, ORACLE, os.path.join(ROOT, "tests")):
        sys.path.insert(0, pth)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from shard_double import NumpyShard
    from slamhip.shard import ShardedFilter, TorchComm
    n_global = n_local * world
    lm, zs, noises, us, p = _inputs(n_global, nl, steps, 11)
    sh = NumpyShard(n_local, n_global, rank * n_local, lm)
    filt = ShardedFilter([sh], [rank], TorchComm(), n_global)
    rows = []
    try:
        for k in range(steps):
            u = us[k] if filt.resample_next else float("nan")
            out = filt.step((p.vel, p.omega), zs[k], noises[k], u)
            rows.append((out["resampled"], out["max_idx"], out["x_est"].copy(), out["ess"]))
        x, y, th, w = filt.get_state()
        q.put((rank, rows, w))
    except Exception as e:                       # report instead of hanging the peer
        q.put((rank, repr(e), None))
        raise
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_matches_single_array_oracle():
    import pf_oracle as po
    n_local, nl, steps, world = 8192, 20, 25, 2
    n_global = n_local * world
    lm, zs, noises, us, p = _inputs(n_global, nl, steps, 11)
    orc = po.PFOracle(p)
    ref = []
    for k in range(steps):
        res = orc.needs_resample()
        out = orc.step(zs[k], noises[k], us[k] * p.np_recip if res else None)
        ref.append((res, out["max_idx"], out["x_est"], po.ess_of(orc.w)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_local, nl, steps, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    results = [q.get(timeout=240) for _ in range(world)]
    errs = [r for r in results if r[2] is None]
    assert not errs, errs
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    results.sort(key=lambda t: t[0])
    assert sum(r[0] for r in ref) >= 3, "the run must exercise resampling"
    for rank, rows, w in results:
        for k, (a, b) in enumerate(zip(rows, ref)):
            assert a[0] == b[0], f"rank {rank} step {k}: resample decision"
            assert a[1] == b[1], f"rank {rank} step {k}: argmax {a[1]} != {b[1]}"
            np.testing.assert_array_equal(a[2], b[2])
            assert abs(a[3] - b[3]) <= 1e-9 * b[3]
        np.testing.assert_array_equal(w, orc.w[rank * n_local:(rank + 1) * n_local])
