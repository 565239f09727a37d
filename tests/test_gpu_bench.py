"""bench.py's output contract on a real GPU: one JSON line with the metric,
the whole-job value, the roofline object of the fused kernel and the step
breakdown (short run: no secondary rows, no CPU baselines)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bench_json_contract():
    env = dict(os.environ)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "8",
                        "--warmup", "2", "--no-secondary", "--no-cpu-baseline"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                "roofline"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 8 and d["warmup"] == 2
    assert d["unit"] == "particle-observation updates/s" and d["value"] > 1e10
    assert abs(d["value"] - 2 ** 20 * 100 / (d["ms_per_step"] / 1e3)) <= 1e-6 * d["value"]
    rf = d["roofline"]
    assert rf["bound"] in ("valu_fp64", "hbm") and 0 < rf["frac"] <= 1
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-12
    # the binding one of executed fp64 and HBM bytes
    assert rf["frac"] >= rf["hbm"]["frac"] - 1e-15
    if rf["fp64"]["frac"] is not None:
        assert rf["frac"] >= rf["fp64"]["frac"] - 1e-15
    assert d["closed_form_fallback_waves"] == 0 and d["ess_near_steps"] >= 0
    assert d["config"]["particles_per_gpu"] == 2 ** 20 and d["config"]["landmarks"] == 100


def _bench_line(cmd):
    r = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ), capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("launcher", ["direct", "torchrun"])
def test_bench_sharded_mode(launcher):
    # --mode sharded: the device-resident sharded step over one shard, in-process
    # or as a 1-rank group under torch.distributed.run
    args = [os.path.join(ROOT, "bench.py"), "--mode", "sharded", "--steps", "6", "--warmup", "2",
            "--no-secondary", "--no-cpu-baseline"]
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", "29533"] + args
    else:
        cmd = [sys.executable] + args
    d = _bench_line(cmd)
    assert d["config"]["parallelism"] == "sharded1"
    assert d["n_gpus"] == 1 and d["steps"] == 6 and d["value"] > 1e9
    assert d["resample_steps"] >= 0 and d["roofline"]["avg_launch_ms"] > 0


@pytest.mark.parametrize("world,total", [(2, None), (3, 3 * 65536), (4, 4 * 65536)])
def test_bench_sharded_ranks_share_one_gpu(world, total):
    """bench.py's N > 1 path (the default --mode sharded) with 2-4 ranks on the
    one GPU of the test box: IPC-opened exchange regions across processes, the
    run's own parity check (PARITY_STEPS sharded steps, the state gathered to
    rank 0 and compared bit for bit with one handle of all the particles), the
    timed hipGraph replays, max-over-ranks timing, one JSON line from rank 0.
    Two ranks at the weak-scaling size (2^20 each); three and four at 65,536
    per rank (--total-particles): each rank's resample exchange is one launch
    whose grid must be co-resident and waits on its peers', and on one shared
    GPU three such 512-block grids of 2^20-particle shards oversubscribe it (the
    waits expire; on the 8-GPU node every rank has its own GPU -- DESIGN 9)."""
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "8", "--warmup", "2",
            "--no-secondary", "--no-cpu-baseline", "--settle-steps", "62"]
    if total:
        args += ["--total-particles", str(total)]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
           str(world), "--master-addr", "127.0.0.1", "--master-port", str(29560 + world)] + args
    env = dict(os.environ, SLAM_BENCH_SHARE_GPU="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    n_total = total or world * 2 ** 20
    assert d["n_gpus"] == world and d["config"]["parallelism"] == f"sharded{world}"
    assert d["value"] > 1e9 and d["resample_steps"] >= 1
    assert abs(d["value"] - n_total * 100 / (d["ms_per_step"] / 1e3)) <= 1e-6 * d["value"]
    pc = d["parity_check"]
    assert pc["bit_identical"] and pc["first_mismatch"] is None and pc["steps"] == 8, pc
    assert pc["resample_steps"] >= 1 and pc["cov_max_rel"] <= 1e-7, pc


def test_bench_sharded_parity_mismatch_falls_back_to_replicas():
    """A sharded run whose gathered state differs from the single handle's (one
    ulp injected into the gathered x on rank 0): every rank leaves the sharded
    mode, the line measures replicas and carries the failed check."""
    args = [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "2",
            "--no-secondary", "--no-cpu-baseline", "--settle-steps", "31"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29539"] + args
    env = dict(os.environ, SLAM_BENCH_SHARE_GPU="1", SLAM_BENCH_PARITY_INJECT="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["config"]["parallelism"] == "replicas2"
    pc = d["parity_check"]
    assert not pc["bit_identical"] and pc["first_mismatch"].startswith("final x[12345]"), pc
    assert d["sharded_error"].startswith("parity"), d["sharded_error"]


def test_bench_sharded_failure_falls_back_to_replicas():
    """Ranks that cannot run the sharded exchange (a failure injected before the
    exchange is set up): the ranks agree and measure independent replicas, and
    the line says so."""
    args = [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "2",
            "--no-secondary", "--no-cpu-baseline"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29543"] + args
    env = dict(os.environ, SLAM_BENCH_SHARE_GPU="1", SLAM_BENCH_FAIL_SHARDED="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["config"]["parallelism"] == "replicas2"
    assert "injected" in d["sharded_error"] and d["value"] > 1e10


def test_bench_sharded_one_rank_failure_falls_back_together():
    """A failure on ONE rank after the exchange regions are set up (as a peer
    GPU that cannot be mapped would raise in slam_dist_connect): the ranks meet
    at the same agreement point, fall back to replicas together, and the line
    names the phase and the failing rank."""
    args = [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "2",
            "--no-secondary", "--no-cpu-baseline"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29547"] + args
    env = dict(os.environ, SLAM_BENCH_SHARE_GPU="1", SLAM_BENCH_FAIL_SHARDED_RANK="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["config"]["parallelism"] == "replicas2"
    assert d["sharded_error"].startswith("connect") and "rank 1" in d["sharded_error"]


def test_bench_strong_scaling_mode():
    """--total-particles: one filter of T particles over the ranks (here two
    ranks on one GPU, T = 2^21: 2^20 per rank), scaling 'strong'."""
    args = [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "2",
            "--no-secondary", "--no-cpu-baseline", "--total-particles", str(1 << 21)]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29549"] + args
    env = dict(os.environ, SLAM_BENCH_SHARE_GPU="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["scaling"] == "strong" and d["config"]["particles_total"] == 1 << 21
    assert d["config"]["particles_per_gpu"] == 1 << 20
    assert abs(d["value"] - (1 << 21) * 100 / (d["ms_per_step"] / 1e3)) <= 1e-6 * d["value"]
