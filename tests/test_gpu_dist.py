"""The sharded particle filter's device-resident step (slam_dist_*, BASELINE
config 3) against one handle holding all particles: bit-identical weights,
particles, resample decisions, argmax, estimate and np.sum, step by step.

  * LOCAL: every shard in this process on one GPU (the multi-GPU step's
    kernels, exchanges and signalling, phase by phase on one stream);
  * one rank per process: a 1-rank RCCL communicator (slam_comm_*) bootstraps
    the exchange; two processes sharing the GPU exchange through IPC-opened
    peer regions (the path of one process per GPU).
"""
import multiprocessing as mp
import os
import sys

import numpy as np
import pytest

import pf_oracle as po

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _world(n_global, nl, steps, seed):
    rs = np.random.RandomState(seed)
    lm = rs.uniform(-10, 10, (nl, 2))
    p = po.PFParams(n_particles=n_global, landmarks=lm, motion="velocity")
    wd = po.PFWorld(p)
    np.random.seed(seed + 1)
    zs = []
    for _ in range(steps):
        wd.advance()
        zs.append(wd.observe())
    return lm, np.array(zs), p


def _same(a, b, k):
    assert a["resampled"] == b["resampled"], k
    assert a["max_idx"] == b["max_idx"], (k, a["max_idx"], b["max_idx"])
    np.testing.assert_array_equal(a["x_est"], b["x_est"])
    assert a["max_val"] == b["max_val"] and a["weight_sum"] == b["weight_sum"], k
    np.testing.assert_allclose(a["cov"], b["cov"], rtol=1e-7, atol=1e-13)
    assert abs(a["ess"] - b["ess"]) <= 1e-9 * a["ess"]
    assert a["resample_next"] == b["resample_next"], k


@pytest.mark.parametrize("world,n_global,nl,lik", [(3, 3 * 65536, 20, "logsum"),
                                                  (2, 2 * 8192 + 1000, 5, "product"),
                                                  (8, 8 << 20, 100, "logsum"),
                                                  # NP > 2^20 with a partial last slice of
                                                  # the single finalize's pre-pass (round 5)
                                                  (2, (1 << 21) + 12345, 20, "logsum")])
def test_dist_local_steps_match_single(world, n_global, nl, lik):
    from slamhip.dist import DistFilter
    from slamhip.pf import DeviceParticleFilter
    steps = 24
    lm, zs, p = _world(n_global, nl, steps, 40 + world)
    single = DeviceParticleFilter(n_global, lm, motion="velocity", likelihood=lik, seed=21)
    dist = DistFilter(n_global, lm, world=world, motion="velocity", likelihood=lik, seed=21)
    n_res = 0
    try:
        for k in range(steps):
            a = single.step((p.vel, p.omega), zs[k])
            b = dist.step((p.vel, p.omega), zs[k])
            _same(a, b, k)
            n_res += a["resampled"]
        for u, v in zip(single.get_state(), dist.get_state()):
            np.testing.assert_array_equal(u, v)
        assert n_res >= 2
    finally:
        dist.close()
        single.close()


def test_dist_local_graph_run_matches_single():
    """The bench path: observations loaded once, steps replayed as hipGraphs."""
    from slamhip.dist import DistFilter
    from slamhip.pf import DeviceParticleFilter
    world, n_global, nl, steps = 4, 4 << 18, 100, 20
    lm, zs, p = _world(n_global, nl, steps, 7)
    ctl = np.tile([p.vel, p.omega], (steps, 1))
    single = DeviceParticleFilter(n_global, lm, motion="velocity", likelihood="logsum", seed=3)
    dist = DistFilter(n_global, lm, world=world, motion="velocity", likelihood="logsum", seed=3)
    try:
        single.load_observations(zs)
        dist.load_observations(zs)
        ra = single.run(0, ctl[:4]) + single.run(4, ctl[4:])
        rb = dist.run(0, ctl[:4]) + dist.run(4, ctl[4:])
        for k, (a, b) in enumerate(zip(ra, rb)):
            _same(a, b, k)
        assert sum(r["resampled"] for r in ra) >= 2
        for u, v in zip(single.get_state(), dist.get_state()):
            np.testing.assert_array_equal(u, v)
    finally:
        dist.close()
        single.close()


@pytest.mark.parametrize("merged", [True, False])
def test_dist_one_shard_resample_forms_match_single(merged):
    """One held shard (the bench's N = 1 sharded form, and one process per GPU):
    the resample exchange in one launch (dist_resample_merged_kernel) and in
    five, against one handle -- at the bench size, replayed as hipGraphs."""
    from slamhip.dist import DistFilter
    from slamhip.pf import DeviceParticleFilter
    n, nl, steps = 1 << 20, 100, 20
    lm, zs, p = _world(n, nl, steps, 17)
    ctl = np.tile([p.vel, p.omega], (steps, 1))
    single = DeviceParticleFilter(n, lm, motion="velocity", likelihood="logsum", seed=13)
    dist = DistFilter(n, lm, world=1, motion="velocity", likelihood="logsum", seed=13)
    try:
        assert dist.set_merged(None)                 # the default where the grid fits
        assert dist.set_merged(merged) == merged
        single.load_observations(zs)
        dist.load_observations(zs)
        ra = single.run(0, ctl[:3]) + single.run(3, ctl[3:])
        rb = dist.run(0, ctl[:3]) + dist.run(3, ctl[3:])
        for k, (a, b) in enumerate(zip(ra, rb)):
            _same(a, b, k)
        assert sum(r["resampled"] for r in ra) >= 3
        for u, v in zip(single.get_state(), dist.get_state()):
            np.testing.assert_array_equal(u, v)
    finally:
        dist.close()
        single.close()


def test_comm_one_rank_rccl():
    """slam_comm over RCCL with one rank: the bootstrap all-gather, and a
    one-rank DistFilter connected through it."""
    from slamhip.dist import Comm, DistFilter
    from slamhip.pf import DeviceParticleFilter
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    try:
        assert comm.all_gather_bytes(b"slam-hip") == [b"slam-hip"]
        n, nl, steps = 3 * 8192, 20, 12
        lm, zs, p = _world(n, nl, steps, 11)
        single = DeviceParticleFilter(n, lm, motion="velocity", likelihood="logsum", seed=5)
        dist = DistFilter(n, lm, world=1, rank=0, comm=comm, motion="velocity", likelihood="logsum",
                          seed=5)
        try:
            for k in range(steps):
                _same(single.step((p.vel, p.omega), zs[k]), dist.step((p.vel, p.omega), zs[k]), k)
        finally:
            dist.close()
            single.close()
    finally:
        comm.close()


def _rank_main(rank, world, n, lm, zs, ctl, q_out, q_in, conn, kw=None):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "slam-robot_simu_amd"))
    from slamhip.dist import DistFilter

    def all_gather(mine):
        conn.send((rank, mine))
        return conn.recv()

    try:
        d = DistFilter(n, lm, world=world, rank=rank, all_gather=all_gather, motion="velocity",
                       likelihood="logsum", seed=8, **(kw or {}))
        d.load_observations(zs)
        merged = d.set_merged(None)
        res = d.run(0, ctl)
        st = d.get_state()
        d.close()
        q_out.put((rank, [(r["max_idx"], r["weight_sum"], r["resampled"]) for r in res], st + (merged,)))
    except Exception as e:              # reported to the parent
        q_out.put((rank, repr(e), None))


@pytest.mark.parametrize("world,tight,extra", [(2, False, 0), (4, False, 0), (3, True, 0),
                                               (2, True, 1000), (2, False, 1000)])
def test_dist_two_processes_share_one_gpu(world, tight, extra):
    """Two (four) ranks, one process each, one GPU: the IPC path of one process
    per GPU (exchange regions exported / opened, device-side signalling across
    processes), replayed as hipGraphs; compared with one handle.  tight: a
    sharp likelihood (R = 0.1^2 I) and a resample every step, so a few
    particles carry the weight and their runs span whole shards -- the
    merged exchange's runs stored into peers' regions, with their carries.
    extra: particles beyond whole shards (a ragged last shard: 73,728 + 58,344)."""
    from slamhip.pf import DeviceParticleFilter
    n, nl, steps = world * 65536 + extra, 50, 16
    lm, zs, p = _world(n, nl, steps, 23)
    kw = dict(r=np.diag([0.1, 0.1]) ** 2, ess_threshold=float(n)) if tight else {}
    ctl = np.tile([p.vel, p.omega], (steps, 1))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pipes = [ctx.Pipe() for _ in range(world)]
    procs = [ctx.Process(target=_rank_main, args=(r, world, n, lm, zs, ctl, q, None, pipes[r][1], kw))
             for r in range(world)]
    for pr in procs:
        pr.start()
    try:
        blobs = [None] * world
        for r in range(world):
            rr, b = pipes[r][0].recv()
            blobs[rr] = b
        for r in range(world):
            pipes[r][0].send(blobs)
        out = {}
        for _ in range(world):
            rank, res, st = q.get(timeout=240)
            assert st is not None, res
            out[rank] = (res, st)
    finally:
        for pr in procs:
            pr.join(timeout=60)
            if pr.is_alive():
                pr.kill()
    with DeviceParticleFilter(n, lm, motion="velocity", likelihood="logsum", seed=8, **kw) as single:
        single.load_observations(zs)
        ref = single.run(0, ctl)
        xs = single.get_state()
    if tight:
        assert all(r["resampled"] for r in ref[1:])
        print("tight ess", [round(r["ess"], 1) for r in ref])
        assert min(r["ess"] for r in ref) < n / 1000             # a few particles serve long runs
    for rank in range(world):
        res, st = out[rank]
        # one shard per process: the one-launch resample exchange (unless the
        # five-launch form is asked for, SLAM_DIST_MERGED=0)
        assert st[4] == (os.environ.get("SLAM_DIST_MERGED", "1") != "0")
        assert [(r["max_idx"], r["weight_sum"], r["resampled"]) for r in ref] == res
    for k in range(4):
        np.testing.assert_array_equal(np.concatenate([out[r][1][k] for r in range(world)]), xs[k])


@pytest.mark.parametrize("world,n_global,nl,lik", [(2, 2 * 8192 + 1000, 5, "product"),
                                                  (4, 4 << 18, 100, "logsum"),
                                                  (8, 8 << 20, 100, "logsum")])
def test_dist_collective_local_matches_single(world, n_global, nl, lik):
    """Collective mode (slam_dist_set_collective) with every shard held: the
    exchanges as host-orchestrated collectives (device copies between the held
    regions standing for RCCL's all-gathers and grouped send/recv), step by
    step and as a run, bit-identical to one handle."""
    from slamhip.dist import DistFilter
    from slamhip.pf import DeviceParticleFilter
    steps = 20
    lm, zs, p = _world(n_global, nl, steps, 60 + world)
    ctl = np.tile([p.vel, p.omega], (steps, 1))
    single = DeviceParticleFilter(n_global, lm, motion="velocity", likelihood=lik, seed=9)
    dist = DistFilter(n_global, lm, world=world, motion="velocity", likelihood=lik, seed=9)
    try:
        dist.use_collectives()
        assert not dist.set_merged(None)
        ra, rb = [], []
        for k in range(6):
            ra.append(single.step((p.vel, p.omega), zs[k]))
            rb.append(dist.step((p.vel, p.omega), zs[k]))
        single.load_observations(zs)
        dist.load_observations(zs)
        ra += single.run(6, ctl[6:])
        rb += dist.run(6, ctl[6:])
        for k, (a, b) in enumerate(zip(ra, rb)):
            _same(a, b, k)
        assert sum(r["resampled"] for r in ra) >= 1          # the resample exchange ran
        for u, v in zip(single.get_state(), dist.get_state()):
            np.testing.assert_array_equal(u, v)
    finally:
        dist.close()
        single.close()


def test_dist_collective_one_rank_rccl_matches_single():
    """Collective mode through a 1-rank RCCL communicator (the one-process-per-
    GPU fallback, without any IPC mapping), at the bench size."""
    from slamhip.dist import Comm, DistFilter
    from slamhip.pf import DeviceParticleFilter
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    n, nl, steps = 1 << 20, 100, 16
    lm, zs, p = _world(n, nl, steps, 23)
    ctl = np.tile([p.vel, p.omega], (steps, 1))
    try:
        single = DeviceParticleFilter(n, lm, motion="velocity", likelihood="logsum", seed=31)
        dist = DistFilter(n, lm, world=1, rank=0, connect=False, motion="velocity",
                          likelihood="logsum", seed=31)
        try:
            dist.use_collectives(comm)
            assert dist.prepare_graphs() < 5.0          # nothing to capture
            single.load_observations(zs)
            dist.load_observations(zs)
            ra, rb = single.run(0, ctl), dist.run(0, ctl)
            for k, (a, b) in enumerate(zip(ra, rb)):
                _same(a, b, k)
            assert sum(r["resampled"] for r in ra) >= 3
            for u, v in zip(single.get_state(), dist.get_state()):
                np.testing.assert_array_equal(u, v)
        finally:
            dist.close()
            single.close()
    finally:
        comm.close()
