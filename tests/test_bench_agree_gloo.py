"""bench.py's multi-rank agreement protocol on CPU (world size 2, gloo): the
sharded setup and run phases of measure_sharded use bench.Agreement, so that a
failure on ONE rank -- after the communicator exists, e.g. a peer GPU that
cannot be mapped in slam_dist_connect -- sends every rank to the replica
fallback at the same checkpoint, with every collective still paired.  The GPU
work is replaced by plain functions; the collectives are the real ones
(all_reduce MIN of the ok flags, barrier, all_gather_object of the errors)."""
import os
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _agree(ok):
    import torch
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item()) == 1


def _worker(rank, world, port, fail_rank, fail_phase, q, fallback=False):
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    log = []

    def work(phase):
        log.append(phase)
        if rank == fail_rank and phase == fail_phase:
            raise RuntimeError(f"injected {phase}")
        return phase

    def sharded():
        ag = bench.Agreement(_agree, rank)
        ag.attempt(work, "create")
        ag.checkpoint("shard create")
        blob = ag.attempt(work, "export")
        blobs = [None] * world
        dist.all_gather_object(blobs, blob)                 # the handle exchange collective
        ag.checkpoint("handle exchange")
        mode, why = bench.connect_exchange(ag, lambda: work("connect"),
                                           (lambda: work("collectives")) if fallback else None)
        # the real bench.timed_runs over a stand-in filter: a failure in any of
        # its phases must still pair every barrier and reach the agreement
        import numpy as np

        class Filt:
            def prepare_graphs(self):
                return work("prepare")

            def run(self, first, ctl, want_results=True):
                return work({0: "warmup", 2: "timed"}.get(first, "timing run"))

            def enable_timing(self, on):
                work("enable timing")

            def timing(self, k):
                return (0.0, 0)

        bench.timed_runs(Filt(), np.zeros((6, 2)), 2, 2, dist.barrier, ag)
        return "sharded" if mode == "peer" else "sharded-rccl"

    try:
        mode, phase = sharded(), None
    except bench.ShardedFailure as e:
        phase, mine = e.args
        errs = [None] * world
        dist.all_gather_object(errs, mine)
        mode = "replicas"
        phase = phase + " | " + "; ".join(x for x in errs if x)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, mode, phase, log))


@pytest.mark.parametrize("fail_rank,fail_phase,expect_phase",
                         [(None, None, None), (1, "connect", "connect"), (0, "export", "handle exchange"),
                          (1, "timed", "run"), (0, "create", "shard create"),
                          (0, "prepare", "warm-up"), (1, "warmup", "warm-up"),
                          (0, "timing run", "timing")])
def test_one_rank_failure_agreed(fail_rank, fail_phase, expect_phase):
    import socket
    world = 2
    with socket.socket() as sk:                          # a free local port
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fail_rank, fail_phase, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    modes = {m for _, m, _, _ in res}
    if fail_rank is None:
        assert modes == {"sharded"}
        return
    assert modes == {"replicas"}, res
    for _, _, phase, log in res:
        assert phase.startswith(expect_phase), phase
        assert f"rank {fail_rank}" in phase and f"injected {fail_phase}" in phase
    # the failing rank did no work after its failure; the others stopped at the checkpoint
    flog = res[fail_rank][3]
    assert flog[-1] == fail_phase


@pytest.mark.parametrize("fail_phase,expect", [("connect", "sharded-rccl"), ("collectives", "replicas")])
def test_connect_failure_falls_back_to_collectives(fail_phase, expect):
    """A peer-memory connect failure on one rank sends every rank to the
    collective exchange together (bench.connect_exchange); only if that fails
    as well do the ranks fall back to replicas."""
    import socket
    world = 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker_two, args=(r, world, port, fail_phase, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert {m for _, m, _, _ in res} == {expect}, res
    if expect == "replicas":
        for _, _, phase, _ in res:
            assert phase.startswith("collectives"), phase


def _worker_two(rank, world, port, fail_phase, q):
    """rank 1 fails its connect (and, for fail_phase "collectives", its
    collective setup too)."""
    sys.path.insert(0, ROOT)
    import bench
    fail = {"connect"} | ({"collectives"} if fail_phase == "collectives" else set())
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    log = []

    def work(phase):
        log.append(phase)
        if rank == 1 and phase in fail:
            raise RuntimeError(f"injected {phase}")
        return phase

    try:
        ag = bench.Agreement(_agree, rank)
        mode, why = bench.connect_exchange(ag, lambda: work("connect"), lambda: work("collectives"))
        mode, phase = ("sharded" if mode == "peer" else "sharded-rccl"), None
    except bench.ShardedFailure as e:
        mode, phase = "replicas", e.args[0]
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, mode, phase, log))
