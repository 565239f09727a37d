#!/usr/bin/env python
"""Benchmark: particle-observation updates/s of the MI355X particle filter.

Workload (BASELINE.json configs[1]): 1,048,576 particles x 100 landmarks per
GPU, velocity motion model (motion_model.py:31-62, a1..a6 = 0.1, dt = 0.1 s),
systematic resampling with the exact sequential-cumsum semantics, on-device
Philox noise.  A "step" is one full estimator step on one batch: [resample]
-> predict -> likelihood -> normalise -> ESS/argmax/covariance.  Observations
for every step are simulated on the host and uploaded BEFORE the timed region
(inputs resident in HBM).

    python bench.py [--gpus N] [--steps K] [--warmup W]

N > 1 is launched by torch.distributed.run (one process per GPU) and runs
--mode sharded by default: the ranks are ONE filter over N x 2^20 particles
(BASELINE configs[2], weak scaling: 2^20 per GPU) through slamhip.dist --
the device-resident step whose exchanges (exact-cumsum specials, resampled
particles, per-rank reduction records) are pushes into peer memory over xGMI
with device-side signalling, bootstrapped over an RCCL communicator; 8 steps
per hipGraph, no host decision per step.  --mode replicas runs independent
Monte-Carlo realisations (no data-path exchange; the N = 1 default).  At N = 1
the line also carries "sharded1": the sharded step's kernels on one shard, and
"strong_single": one handle of 2^23 particles (the strong-scaling reference).

    --total-particles T   strong scaling: one filter of T particles split over
                          the N ranks (T / N per GPU; "scaling": "strong")

The sharded setup and run agree across ranks at fixed points (every rank
reaches the same collectives whether or not it failed locally), so one rank's
failure sends every rank to the replica fallback together.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_simu_amd"))

METRIC = "particle-observation updates/sec @1M particles×100 landmarks; 1/2/4/8-GPU scaling"
NP_PER_GPU = 1 << 20
STRONG_TOTAL = 1 << 23          # BASELINE configs[2]'s total particles
NL = 100
FP64_PEAK_TFLOPS = 78.6          # MI355X FP64 (vector = matrix), spec
HBM_PEAK_GBS = 8000.0
VALU_SLOTS_PER_S = 1024 * 2.4e9 / 4   # wave64 VALU instructions/s: 1,024 SIMDs, 4 cycles each, 2.4 GHz
# The reference algorithm's fp64 operations per particle-landmark update (fma =
# 2, exp = div = 1) -- reported as "reference_equivalent_tflops" only: the
# log-sum kernel evaluates the landmark sum in closed form and does not execute
# them; roofline.achieved is the kernel's EXECUTED fp64 work (PMC).
#   product (particle_filter.py:187-192 + mlab.bivariate_normal, factor by factor):
#     diff 2, rotate 6, residual 2, q = dx^2/sx^2 + dy^2/sy^2 5, -q/2 1, exp 1,
#     /den 1, running product 1  -> 19
#   logsum (same density, one exp per particle): diff 2, rotate+residual 8,
#     dx^2 + dy^2 accumulated 4 -> 14
FLOPS_PER_UPDATE = {"product": 19, "logsum": 14}
# algorithmic HBM bytes per particle per step of the fused kernel:
#   read x,y,th (24) + w (8), write x,y,th (24) + w_un (8)
BYTES_PER_PARTICLE = 64


def simulate_world(n_steps, seed=1):
    """Truth (motion_model.py:64-86, noise free) + landmark observations
    (particle_filter.py:144-154)."""
    from mylib import limit
    from mylib import transform as tf
    rs = np.random.RandomState(seed)
    lm = rs.uniform(-10.0, 10.0, (NL, 2))
    omega = np.deg2rad(10.0)
    vel = 10.0 * omega
    dt = 0.1
    r = np.diag([0.3, 0.3]) ** 2
    x = np.array([[10.0], [0.0], [np.pi / 2]])
    zs = np.empty((n_steps, NL, 2))
    poses = np.empty((n_steps, 3))
    for k in range(n_steps):
        a = vel / omega
        b = limit.limit_angle(omega * dt)
        y2 = limit.limit_angle(x[2, 0] + b)
        x = np.array([[x[0, 0] + a * (-np.sin(x[2, 0]) + np.sin(y2))],
                      [x[1, 0] + a * (np.cos(x[2, 0]) - np.cos(y2))], [y2]])
        zs[k] = tf.world2robot(x, lm) + rs.multivariate_normal([0.0, 0.0], r, NL)
        poses[k] = x[:, 0]
    simulate_world.poses = poses
    return lm, zs, (vel, omega, dt)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _pinned_init(core):
    os.sched_setaffinity(0, {core})


def _cpu_faithful_sample(n_steps, n=NP_PER_GPU):
    """The oracle's faithful port (per-particle loop of particle_filter.py:185-192,
    velocity motion model) at the C2 size itself -- 1,048,576 particles x 100
    landmarks, BASELINE.md's "time a few CPU steps" -- for n_steps whole steps
    (~12-20 s each); runs in a child pinned to one core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pf_oracle as po
    lm, zs, (vel, omega, dt) = simulate_world(max(n_steps, 1), seed=2)
    p = po.PFParams(period_ms=100, n_particles=n, landmarks=lm, motion="velocity")
    pf = po.PFOracle(p)
    rs = np.random.RandomState(0)
    steps, t_used = 0, 0.0
    while steps < n_steps:
        g = rs.standard_normal(3 * n).reshape(n, 3)
        t0 = time.perf_counter()
        if pf.needs_resample():
            idx = po.systematic_indices(pf.w, rs.random_sample() * p.np_recip)
            pf.x, pf.y, pf.th = pf.x[idx], pf.y[idx], pf.th[idx]
            pf.w = np.full(n, p.np_recip)
        pf.x, pf.y, pf.th = po.motion_velocity(pf.x, pf.y, pf.th, vel, omega, dt, p.alphas, g)
        pf.w, _ = po.likelihood_loop(pf.x, pf.y, pf.th, pf.w, p.lm, zs[steps], p.r)
        i = int(np.argmax(pf.w))
        _ = (pf.x[i], pf.y[i], pf.th[i])
        t_used += time.perf_counter() - t0
        steps += 1
    return n, steps, t_used, sorted(os.sched_getaffinity(0))


def cpu_baseline(n_steps=2):
    """The oracle's faithful port on ONE host core (the reference is
    single-threaded Python) at the C2 size: a spawned child pinned with
    sched_setaffinity (taskset) to the first core this process may use, BLAS
    threads 1."""
    import multiprocessing as mp
    core = min(os.sched_getaffinity(0))
    saved = {k: os.environ.get(k) for k in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS")}
    os.environ.update(OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1")
    try:
        with mp.get_context("spawn").Pool(1, initializer=_pinned_init, initargs=(core,)) as pool:
            n, steps, t_used, cpus = pool.apply(_cpu_faithful_sample, (n_steps,))
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return {"value": n * NL * steps / t_used, "unit": "particle-observation updates/s",
            "cores": 1, "kind": "port", "cpu_model": cpu_model(), "pinned_cpus": cpus,
            "sample": f"oracle faithful per-particle loop, {n} particles x {NL} landmarks x "
                      f"{steps} steps (velocity model), {t_used:.1f} s on core {core} "
                      "(sched_setaffinity, OPENBLAS_NUM_THREADS=1)"}


def _vec_shard_steps(args):
    """Worker of cpu_baseline_vectorised: the vectorised oracle step (predict
    with the velocity model, factor-by-factor likelihood, normalise, ESS and
    systematic resample when due, estimate) on one shard of particles."""
    n, steps, seed = args
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pf_oracle as po
    lm, zs, (vel, omega, dt) = simulate_world(steps, seed=2)
    p = po.PFParams(period_ms=100, n_particles=n, landmarks=lm, motion="velocity")
    pf = po.PFOracle(p)
    rs = np.random.RandomState(seed)
    t0 = time.perf_counter()
    for k in range(steps):
        g = rs.standard_normal(3 * n).reshape(n, 3)
        ofs = rs.random_sample() * p.np_recip if pf.needs_resample() else None
        pf.step(zs[k], g, ofs, control=(vel, omega))
    return time.perf_counter() - t0


def cpu_baseline_vectorised(n_per_proc=1 << 15, steps=6):
    """A stronger CPU baseline than the faithful loop: the oracle's vectorised
    NumPy step (bit-identical to the loop form) on every usable host core, one
    independent shard per process (at most 16 processes, the box's CPU share)."""
    import multiprocessing as mp
    procs = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity")
                       else (os.cpu_count() or 1)))
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(procs) as pool:
        per = pool.map(_vec_shard_steps, [(n_per_proc, steps, 100 + r) for r in range(procs)])
    wall = time.perf_counter() - t0
    busy = max(per)
    return {"value": procs * n_per_proc * NL * steps / busy,
            "unit": "particle-observation updates/s", "cores": procs, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"oracle vectorised NumPy step (velocity model), {procs} processes x "
                      f"{n_per_proc} particles x {NL} landmarks x {steps} steps, slowest "
                      f"process {busy:.1f} s (pool wall {wall:.1f} s incl. start-up)"}


PF_SOURCES = ("pf_kernels.inl", "pf_kernels.hpp", "fastmath.hpp", "common.hpp")


def pf_sources_sha():
    """sha256 over the sources the fused PF kernel is compiled from."""
    import hashlib
    h = hashlib.sha256()
    for name in PF_SOURCES:
        with open(os.path.join(ROOT, "slam-robot_simu_amd", "csrc", name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def load_pmc_traffic(likelihood="logsum"):
    """Per-launch counters of the fused kernel from the rocprofv3 PMC passes of
    tools/pmc.sh (profiles/pmc_traffic.json): HBM bytes (FETCH_SIZE x2 +
    WRITE_SIZE per the microarch guide), executed fp64 flops
    (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 x 64 lanes, fma = 2) and VALU
    wave-instructions.  The counters cannot be read from inside this process;
    the file records the sources it was measured on, and figures measured on
    other sources are reported as null (stale), never as this kernel's."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except Exception:
        return None, "no profiles/pmc_traffic.json", {}
    cur = pf_sources_sha()
    if d.get("sources_sha") != cur:
        return None, f"stale: measured on sources {d.get('sources_sha')}, current {cur}", {}
    if likelihood != "logsum":
        k = d.get("kernels", {}).get(likelihood, {})
        return k.get("hbm_bytes"), f"rocprofv3 PMC ({d.get('source')}), sources {cur}", k
    return d.get("fused_kernel_hbm_bytes_per_launch"), \
        f"rocprofv3 PMC ({d.get('source')}), sources {cur}", d.get("fused_kernel", {})


def fused_roofline(likelihood, n_particles, fused_avg_s):
    """Roofline of the fused predict + likelihood kernel from EXECUTED work
    (VERDICT r2): executed fp64 flops (PMC) / the live average launch against
    the fp64 peak, and HBM bytes / launch against 8 TB/s -- the binding one of
    the two is `bound` / `achieved` / `frac`; the VALU issue fraction (the
    kernel's actual limiter) and the reference algorithm's flop-equivalent rate
    are reported beside them."""
    traffic, src, pmc = load_pmc_traffic(likelihood)
    alg_bytes = BYTES_PER_PARTICLE * n_particles
    hbm_alg_gbs = alg_bytes / fused_avg_s / 1e9
    hbm = {"achieved": hbm_alg_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": hbm_alg_gbs / HBM_PEAK_GBS, "algorithmic_bytes": alg_bytes,
           "note": "64 B/particle: x, y, th (24) + w (8) read and written"}
    if traffic:
        hbm["traffic_gbs"] = traffic / fused_avg_s / 1e9
        hbm["traffic_frac"] = hbm["traffic_gbs"] / HBM_PEAK_GBS
    fp = {"achieved": None, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": None}
    if pmc.get("fp64_flops"):
        fp["achieved"] = pmc["fp64_flops"] / fused_avg_s / 1e12
        fp["frac"] = fp["achieved"] / FP64_PEAK_TFLOPS
        fp["executed_flops_per_launch"] = pmc["fp64_flops"]
    fp_frac = fp["frac"] if fp["frac"] is not None else -1.0
    main = fp if fp_frac >= hbm["frac"] else hbm
    rf = {"bound": "valu_fp64" if main is fp else "hbm",
          "kernel": f"pf_fused_kernel<velocity, {likelihood}> (predict + likelihood + block epilogue)",
          "achieved": main["achieved"], "peak": main["peak"], "unit": main["unit"],
          "frac": main["frac"], "traffic": traffic, "traffic_source": src,
          "avg_launch_ms": fused_avg_s * 1e3, "fp64": fp, "hbm": hbm,
          "reference_equivalent_tflops":
              FLOPS_PER_UPDATE[likelihood] * n_particles * NL / fused_avg_s / 1e12,
          "note": "achieved/frac: the binding one of executed fp64 (PMC flops / live launch "
                  "time / 78.6 TF) and HBM (algorithmic bytes / live launch time / 8 TB/s); "
                  "the kernel is VALU-issue bound (valu_issue_frac: PMC wave64 VALU "
                  "instructions x 4 cycles over 1,024 SIMDs x 2.4 GHz); "
                  "reference_equivalent_tflops counts the reference's per-landmark flops "
                  "(SURVEY 8(d)), which the closed-form log-sum does not execute"}
    if pmc.get("SQ_INSTS_VALU"):
        rf["valu_issue_frac"] = pmc["SQ_INSTS_VALU"] / (VALU_SLOTS_PER_S * fused_avg_s)
        rf["valu_insts_per_launch"] = pmc["SQ_INSTS_VALU"]
    return rf


# ----------------------------------------------------------- secondary rows
def bench_ekf_batch(batch=1 << 20, steps=64, device=0):
    """A14 batched: 2^20 independent 3-state EKFs x 64 steps in one launch,
    observations uploaded before the timed region (resident in HBM)."""
    from slamhip.ekf import DeviceEKF
    rs = np.random.RandomState(7)
    dev = DeviceEKF(batch, device=device)
    t = np.arange(1, steps + 1) * 0.1 * np.deg2rad(10.0)
    z = np.stack([10 * np.cos(t), 10 * np.sin(t)], 1)[:, None, :] + rs.standard_normal((steps, batch, 2))
    dev.load_observations(z)
    del z
    dev.run_loaded(steps)
    dev.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        dev.run_loaded(steps)
    dev.synchronize()
    dt = (time.perf_counter() - t0) / reps
    dev.close()
    fs = batch * steps / dt
    byt = 40.0 * batch * steps        # z read 16 B + x_hat write 24 B per filter-step
    return {"workload": "EKF localisation (extended_kalman_filter.py:108-128), 1,048,576 "
                        "filters x 64 steps per launch", "value": fs, "unit": "filter-steps/s",
            "ms_per_launch": dt * 1e3,
            "roofline": {"bound": "hbm", "achieved": byt / dt / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": byt / dt / 1e9 / HBM_PEAK_GBS,
                         "note": "40 algorithmic B per filter-step (z in, x_hat out); the kernel "
                                 "is fp64-VALU issue bound in practice (PMC: 221 VALU "
                                 "instructions per filter-step before the adjugate / "
                                 "structural-zero cleanup, ~142 algorithmic flops, ~1.5 GHz "
                                 "effective clock under fp64 load); prefetching z, coalescing "
                                 "the x_hat stores through LDS or a lean sincos did not move it"}}


def _scan_measure(pose, lmk):
    """ScanSensor measurement (graph_based_slam.py:150-153) of landmarks lmk
    (k,3: x, y, heading) from pose (3,): range, bearing, orientation."""
    psi = np.pi / 2 - pose[2]
    dx, dy = lmk[:, 0] - pose[0], lmk[:, 1] - pose[1]
    rx = np.cos(psi) * dx - np.sin(psi) * dy
    ry = np.sin(psi) * dx + np.cos(psi) * dy
    wrap = lambda a: np.mod(a + np.pi, 2 * np.pi) - np.pi
    return np.column_stack([np.hypot(rx, ry), np.arctan2(ry, rx), wrap(psi + lmk[:, 2])])


def bench_ekfslam(n_lm=10000, k=20, steps=6, device=0):
    """BASELINE config 4: EKF-SLAM, n = 30,003 (P = 7.2 GB in HBM), the 20
    nearest landmarks observed per step (a rank-60 covariance update)."""
    from slamhip.ekf import DeviceEKFSLAM
    rs = np.random.RandomState(4)
    lmk = np.column_stack([rs.uniform(-100, 100, (n_lm, 2)), rs.uniform(-np.pi, np.pi, n_lm)])
    pose = np.array([50.0, 0.0, np.pi / 2])
    dt, ctl = 0.1, (5.0, 0.1)
    dev = DeviceEKFSLAM(n_lm, dt=dt, device=device)
    n = 3 + 3 * n_lm
    mu0 = np.concatenate([pose, (lmk + rs.normal(0, 0.5, lmk.shape)).ravel()])
    dev.init_diag(mu0, np.concatenate([[1e-4, 1e-4, 1e-5], np.full(n - 3, 0.25)]))
    times, rank_ms = [], []
    for s in range(steps + 2):
        a = dt * np.cos(pose[2]), dt * np.sin(pose[2])
        pose = np.array([pose[0] + ctl[0] * a[0], pose[1] + ctl[0] * a[1],
                         np.mod(pose[2] + ctl[1] * dt + np.pi, 2 * np.pi) - np.pi])
        ids = np.argpartition(np.hypot(lmk[:, 0] - pose[0], lmk[:, 1] - pose[1]), k)[:k]
        obs = _scan_measure(pose, lmk[ids])
        obs[:, 0] *= 1 + 0.01 * rs.standard_normal(k)
        t0 = time.perf_counter()
        dev.step(ctl, ids, obs)
        if s >= 2:
            times.append(time.perf_counter() - t0)
            rank_ms.append(dev.timing()["rank_update_ms"])
    tm = dev.timing()
    dev.close()
    rk = float(np.mean(rank_ms)) / 1e3
    byt = 16.0 * n * (n + 1) / 2          # lower triangle of P read + written once
    flops = 2.0 * (3 * k) * n * (n + 1) / 2
    return {"workload": "EKF-SLAM C4: 10,000 landmarks (n = 30,003, P = 7.2 GB), 20 observed "
                        "per step", "value": 1.0 / float(np.mean(times)), "unit": "updates/s",
            "ms_per_update": float(np.mean(times)) * 1e3, "last_update_breakdown_ms": tm,
            "roofline": {"bound": "hbm", "kernel": "eks_rank_update_frag_kernel (fp64 MFMA)",
                         "achieved": byt / rk / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": byt / rk / 1e9 / HBM_PEAK_GBS,
                         "tflops": flops / rk / 1e12, "avg_launch_ms": rk * 1e3}}


def bench_graph(n_poses=50000, iters=3, device=0):
    """BASELINE config 5: graph-based SLAM, 50,000 poses, ~200,000 edges of the
    setPairObs form; one Gauss-Newton iteration = linearise + assemble + PCG
    solve + pose update, all on the device."""
    from slamhip.graph import DeviceGraph, circle_graph
    init, truth, edges = circle_graph(n_poses, n_landmarks=64, seed=0, odom_noise=0.002)
    dev = DeviceGraph(solver="pcg", pcg_tol=1e-10, device=device)
    dev.set_poses(init)
    t0 = time.perf_counter()
    dev.set_edges(edges)
    t_first = time.perf_counter() - t0             # includes the buffers' allocation
    t_sets = []
    for _ in range(5):                             # a new edge set of the same size (per frame)
        t0 = time.perf_counter()
        dev.set_edges(edges)
        t_sets.append(time.perf_counter() - t0)
    t_struct = float(np.median(t_sets))
    dev.update()                                   # warm-up iteration (cold cond estimate)
    cond_first = dev.cond_info()
    per, brk, conds = [], [], []
    for _ in range(iters):
        t0 = time.perf_counter()
        st = dev.update()
        per.append(time.perf_counter() - t0)
        brk.append(dev.timing())
        conds.append(dict(dev.cond_info(), cond=st[3], det=st[2]))
    gate = dev.gate_info()
    dev.close()

    def per_iteration(cond):
        # the same iterations with another gate mode: "off" (no gate), "estimate"
        # (the LOBPCG estimate to its tight convergence, round 4's gate)
        g = DeviceGraph(solver="pcg", pcg_tol=1e-10, cond=cond, device=device)
        g.set_poses(init)
        g.set_edges(edges)
        g.update()
        out = []
        for _ in range(iters):
            t0 = time.perf_counter()
            g.update()
            out.append(time.perf_counter() - t0)
        g.close()
        return out

    per_off = per_iteration("off")
    per_est = per_iteration("estimate")
    lin = float(np.mean([b["linearize_ms"] for b in brk])) / 1e3
    return {"workload": f"graph SLAM C5: {n_poses} poses, {len(edges)} edges, block-Jacobi PCG",
            "value": 1.0 / float(np.mean(per)), "unit": "Gauss-Newton iterations/s",
            "ms_per_iteration": float(np.mean(per)) * 1e3, "structure_build_ms": t_struct * 1e3,
            "structure_build_first_ms": t_first * 1e3,
            "structure_build_max_ms": max(t_sets) * 1e3,
            "structure_build_each_ms": [t * 1e3 for t in t_sets],
            "breakdown_ms": brk[-1], "is_calc": bool(st[0]),
            "cond": conds[-1]["cond"], "cond_estimate": conds[-1],
            "cond_estimate_first_update": cond_first,
            "gate": "margin (graph_based_slam.py:494-496: an estimate with margins, not a "
                    "certificate -- log-det interval whose lower end holds unless the Ritz "
                    "lambda_min over-estimates by > 1000x, cond estimate with an early "
                    "decision at a factor-100 margin)",
            "gate_info": gate,
            "ms_per_iteration_without_cond": float(np.mean(per_off)) * 1e3,
            "ms_per_iteration_estimate_gate": float(np.mean(per_est)) * 1e3,
            "linearize_edges_per_s": len(edges) / lin,
            "roofline": {"bound": "hbm", "kernel": "graph_linearize_kernel",
                         "achieved": (80 + 48 + 336) * len(edges) / lin / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": (80 + 48 + 336) * len(edges) / lin / 1e9 / HBM_PEAK_GBS,
                         "note": "80 B edge + 2 x 24 B poses in, 336 B blocks out per edge"}}


def _blas_threads():
    try:
        from threadpoolctl import threadpool_info
        return max([d.get("num_threads", 1) for d in threadpool_info()
                    if d.get("user_api") == "blas"] or [1])
    except Exception:
        return None


def cpu_ekf_batch(seconds_target=3.0):
    """The oracle's ekf_update (extended_kalman_filter.py:108-128, NumPy per
    filter-step, as the reference runs it) on one host core, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ekf_oracle as eo
    p = eo.EKFParams()
    rs = np.random.RandomState(5)
    x, P = np.array([10.0, 0.0, np.pi / 2]), np.diag([0.01, 0.01, 0.001])
    zs = rs.standard_normal((4096, 2)) + np.array([10.0, 0.0])
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds_target:
        _, x, P = eo.ekf_update(x, P, zs[steps % len(zs)], p)
        steps += 1
    dt = time.perf_counter() - t0
    return {"value": steps / dt, "unit": "filter-steps/s", "cores": 1, "kind": "port",
            "sample": f"oracle ekf_update, one filter, {steps} steps, {dt:.1f} s on 1 core"}


def cpu_ekfslam(n_lm=None, k=20):
    """One EKF-SLAM update of the oracle restatement (dense NumPy, BLAS threads).
    At the C4 size (n = 30,003) it needs ~30 GB of host RAM (P, its copy and
    the K S K^T temporaries); with less than 64 GB available the sample is
    n = 3,003 and the unit names the sample size."""
    import psutil
    if n_lm is None:
        n_lm = 10000 if psutil.virtual_memory().available >= 64e9 else 1000
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ekf_oracle as eo
    rs = np.random.RandomState(4)
    lmk = np.column_stack([rs.uniform(-100, 100, (n_lm, 2)), rs.uniform(-np.pi, np.pi, n_lm)])
    pose = np.array([50.0, 0.0, np.pi / 2])
    n = 3 + 3 * n_lm
    mu = np.concatenate([pose, (lmk + rs.normal(0, 0.5, lmk.shape)).ravel()])
    P = np.diag(np.concatenate([[1e-4, 1e-4, 1e-5], np.full(n - 3, 0.25)]))
    ids = np.argpartition(np.hypot(lmk[:, 0] - pose[0], lmk[:, 1] - pose[1]), k)[:k]
    obs = _scan_measure(pose, lmk[ids])
    q = np.diag([0.1, 0.1, np.deg2rad(0.1)]) ** 2
    t0 = time.perf_counter()
    mu, P = eo.ekfslam_step(mu, P, (5.0, 0.1), ids, obs, 0.1, q,
                            (0.05, np.deg2rad(2.0), np.deg2rad(2.0)))
    dt = time.perf_counter() - t0
    del P
    unit = "updates/s" if n_lm == 10000 else f"updates/s at n = {n}"
    return {"value": 1.0 / dt, "unit": unit, "cores": _blas_threads(),
            "kind": "port",
            "sample": f"oracle ekfslam_step, n = {n}, k = {k}, one update (dense NumPy / BLAS), "
                      f"{dt:.2f} s"}


def secondary(device=0, cpu=True):
    out = {}
    for name, fn, cfn in (("ekf_batch", bench_ekf_batch, cpu_ekf_batch),
                          ("ekfslam_c4", bench_ekfslam, cpu_ekfslam),
                          ("graph_c5", bench_graph, None)):
        try:
            out[name] = fn(device=device)
            if cpu and cfn is not None:
                out[name]["cpu_baseline"] = cfn()
        except Exception as e:            # reported, never silently replaced
            out[name] = {**out.get(name, {}), "error": f"{type(e).__name__}: {e}"}
    return out


class ShardedFailure(RuntimeError):
    """The sharded mode failed on some rank (every rank raises it together)."""


class Agreement:
    """Fixed agreement points for a multi-rank phase sequence: every rank runs
    the same collectives in the same order whether or not its own work failed
    (a failed rank skips the work, not the collectives), and at each
    checkpoint all ranks learn -- through one MIN all-reduce of an ok flag --
    whether any rank failed, and then raise ShardedFailure together.

    agree(ok: bool) -> bool is the all-reduce (True when every rank is ok)."""

    def __init__(self, agree, rank=0):
        self.agree, self.rank, self.err = agree, rank, None

    def attempt(self, fn, *a, **kw):
        if self.err is not None:
            return None
        try:
            return fn(*a, **kw)
        except Exception as e:                      # noqa: BLE001 - agreed on below
            self.err = e
            return None

    def checkpoint(self, phase):
        if not self.agree(self.err is None):
            mine = None if self.err is None else f"rank {self.rank}: {type(self.err).__name__}: {self.err}"
            raise ShardedFailure(phase, mine)


def connect_exchange(ag, connect, use_collectives=None):
    """The sharded filter's exchange: the peer-memory connect on every rank; if
    it failed on any rank (a peer's region that cannot be mapped), every rank
    switches to the collective exchange (RCCL all-gathers and grouped
    send/recv between the step's kernels) when use_collectives is given.
    Returns (mode, why): "peer" or "rccl", and the agreed failure that led to
    the fallback.  Raises ShardedFailure when no exchange could be set up."""
    ag.attempt(connect)
    try:
        ag.checkpoint("connect")
        return "peer", None
    except ShardedFailure as e:
        if use_collectives is None:
            raise
        ag.err = None                       # every rank knows; start the fallback together
        ag.attempt(use_collectives)
        ag.checkpoint("collectives")
        return "rccl", e.args


SETTLE_BATCH = 31      # 16 + 8 + 4 + 2 + 1: every captured graph shape once per batch
PARITY_STEPS = 8       # sharded runs: steps replayed against one handle before timing
NS_ROUND_STEPS = 64    # NumPy-stream timing window: two of its ring-refill periods


def compare_to_single(recs, state, ref_recs, ref_state):
    """A sharded run's records and gathered final state against one handle's
    run of the same filter (same seed, observations and controls): the fields
    the sharded step reproduces bit for bit (argmax, estimate, max, np.sum,
    resample decisions; particles and weights) and the covariance, which the
    shards reduce in another fixed order (1e-7, as tests/test_gpu_configs.py's
    C3).  Returns (bit_identical, worst cov relative difference, first
    mismatch or None)."""
    first, worst = None, 0.0
    for k, (a, b) in enumerate(zip(ref_recs, recs)):
        for f in ("resampled", "resample_next", "max_idx", "max_val", "weight_sum", "x_est"):
            if first is None and not np.array_equal(a[f], b[f]):
                first = f"step {k}: {f} {b[f]!r} != single {a[f]!r}"
        den = np.maximum(np.abs(a["cov"]), 1e-13)
        worst = max(worst, float(np.max(np.abs(a["cov"] - b["cov"]) / den)))
    for name, u, v in zip(("x", "y", "th", "w"), ref_state, state):
        if first is None and not np.array_equal(u, v):
            i = int(np.flatnonzero(u != v)[0])
            first = f"final {name}[{i}] {v[i]!r} != single {u[i]!r}"
    if first is None and worst > 1e-7:
        first = f"cov relative difference {worst:.3g} > 1e-7"
    return first is None, worst, first


def settle(run, ctl, n):
    """`n` untimed steps (whole SETTLE_BATCH batches) before the warm-up: the
    device's clocks come up under load over ~20 ms and the first replay of each
    graph shape pays a one-time cost; without this a 5-step warm-up leaves
    both inside a 20-step timed run.  A fixed count, so that every
    rank of a sharded run replays the same steps."""
    for s0 in range(0, n - n % SETTLE_BATCH, SETTLE_BATCH):
        run(s0, ctl[s0:s0 + SETTLE_BATCH], want_results=False)
    return n - n % SETTLE_BATCH


def timed_runs(filt, ctl, warmup, steps, barrier_sync, ag=None, settle_steps=0):
    """Every step graph captured first (graph_capture_ms, never inside a timed
    run), `settle_steps` untimed steps (settle), `warmup` untimed steps, `steps`
    timed steps between barrier + synchronize, then a kernel-timing pass over
    `steps` more steps (HIP events on the filter's stream around every launch).
    ctl holds settle_steps + warmup + 2 steps rows.  With an Agreement (the
    sharded mode) a rank's failure is caught, every rank still reaches every
    barrier, and the ranks agree on it at the next checkpoint."""
    call = ag.attempt if ag is not None else (lambda fn, *a, **kw: fn(*a, **kw))
    cap_ms = call(filt.prepare_graphs)
    s0 = call(settle, filt.run, ctl, settle_steps) if settle_steps else 0
    s0 = s0 or 0                                   # (a failed attempt returns None)
    ctl = ctl[s0:]
    if warmup:
        call(filt.run, s0, ctl[:warmup], want_results=False)
    if ag is not None:
        ag.checkpoint("warm-up")
    barrier_sync()
    t0 = time.perf_counter()
    out = call(filt.run, s0 + warmup, ctl[warmup:warmup + steps])
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if ag is not None:
        ag.checkpoint("run")
    call(filt.enable_timing, True)
    call(filt.run, s0 + warmup + steps, ctl[warmup + steps:warmup + 2 * steps])
    timing = call(lambda: {k: filt.timing(k) for k in range(4)})
    call(filt.enable_timing, False)
    if ag is not None:
        ag.checkpoint("timing")
    return elapsed, out, timing, cap_ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--likelihood", default="logsum", choices=["product", "logsum"])
    ap.add_argument("--mode", default=None, choices=["replicas", "sharded"],
                    help="sharded (default for N > 1): one filter over N x 2^20 particles "
                         "(BASELINE configs[2]); replicas (default for N = 1): independent filters")
    ap.add_argument("--total-particles", type=int, default=None,
                    help="strong scaling: one filter of this many particles over the N ranks")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--settle-steps", type=int, default=20 * SETTLE_BATCH,
                    help="untimed steps before the warm-up (whole batches of 31: every graph "
                         "shape; device clocks up); reported as settle_steps")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the EKF / EKF-SLAM / graph-SLAM rows (rank 0, N = 1 only)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.mode is None:
        args.mode = "sharded" if world > 1 else "replicas"
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    strong = args.total_particles is not None
    n_total = args.total_particles if strong else world * NP_PER_GPU
    if strong and (n_total % world or (n_total // world) % 8192):
        raise SystemExit("--total-particles: need T / N to be a whole number of 8192-particle buffers")
    n_per_rank = n_total // world
    # SLAM_BENCH_SHARE_GPU=1 (tests on a one-GPU box): every rank on device 0,
    # gloo for the harness, the exchange regions bootstrapped through gloo
    # (RCCL refuses two ranks on one GPU)
    share_gpu = os.environ.get("SLAM_BENCH_SHARE_GPU") == "1"
    if share_gpu:
        local_rank = 0
    dist = None
    if world > 1 or ("MASTER_ADDR" in os.environ and "RANK" in os.environ):   # torch.distributed.run
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl" if torch.cuda.is_available() and not share_gpu else "gloo")
    multi = dist is not None and world > 1
    tdev = "cpu" if share_gpu else f"cuda:{local_rank}"

    def agree(ok):
        if not multi:
            return ok
        import torch
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return int(t.item()) == 1

    from slamhip.pf import DeviceParticleFilter
    settle_steps = args.settle_steps - args.settle_steps % SETTLE_BATCH
    # the NumPy-stream mode refills its word ring once per ~32 requests
    # (kMtRoundsAhead): it is timed over whole refill periods
    ns_steps = max(args.steps, NS_ROUND_STEPS)
    total_steps = settle_steps + args.warmup + max(2 * args.steps, ns_steps)
    lm, zs, (vel, omega, dt) = simulate_world(total_steps)
    ctl = np.tile([vel, omega], (total_steps, 1))

    def barrier_sync():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    exchange_mode = ["peer"]

    def measure_sharded(likelihood, n_global):
        # one filter over n_global particles (BASELINE configs[2]): this rank's
        # shard through slamhip.dist.DistFilter -- the device-resident step
        # (peer-memory exchanges over xGMI inside the step's kernels, no host
        # decision, 8 steps per hipGraph); the exchange regions are bootstrapped
        # over an RCCL communicator created by the library (the 128-byte RCCL id
        # travels through torch.distributed once).  At world = 1 the single
        # shard runs the same kernels in-process.
        from slamhip.dist import Comm, DistFilter
        if os.environ.get("SLAM_BENCH_FAIL_SHARDED") == "1":         # tests: every rank, before setup
            raise ShardedFailure("setup", f"rank {rank}: injected sharded-mode failure")
        fail_rank = os.environ.get("SLAM_BENCH_FAIL_SHARDED_RANK")   # tests: one rank, after setup
        kw = dict(dt=dt, motion="velocity", likelihood=likelihood, seed=1234, device=local_rank)
        ag = Agreement(agree, rank)
        comm = filt = None
        try:
            if not multi:
                filt = DistFilter(n_global, lm, world=1, **kw)
            else:
                if not share_gpu:
                    obj = [ag.attempt(Comm.unique_id) if rank == 0 else None]
                    dist.broadcast_object_list(obj, src=0)
                    ag.checkpoint("rccl id")
                    comm = Comm(obj[0], world, rank, local_rank)       # collective (RCCL init)
                filt = ag.attempt(DistFilter, n_global, lm, world=world, rank=rank, connect=False, **kw)
                ag.checkpoint("shard create")
                blob = ag.attempt(filt.export_handle)
                if share_gpu:
                    blobs = [None] * world
                    dist.all_gather_object(blobs, blob)
                else:
                    blobs = comm.all_gather_bytes(blob if blob is not None else bytes(len_blob(filt)))
                ag.checkpoint("handle exchange")

                def connect():
                    filt.connect(blobs)
                    if os.environ.get("SLAM_BENCH_FAIL_CONNECT_RANK") == str(rank):   # tests
                        raise RuntimeError(f"injected connect failure on rank {rank}")
                mode, why = connect_exchange(
                    ag, connect, (lambda: filt.use_collectives(comm)) if comm is not None else None)
                exchange_mode[0] = mode if why is None else f"{mode} (peer-memory connect failed: {why[1] or 'another rank'})"
                if fail_rank is not None and int(fail_rank) == rank:
                    ag.attempt(_raise, RuntimeError(f"injected failure on rank {rank} after connect"))
                ag.checkpoint("connect done")
            ag.attempt(filt.load_observations, zs)
            ag.checkpoint("load")
            if multi and os.environ.get("SLAM_BENCH_NO_PARITY") != "1":
                sharded_parity(filt, ag, n_global, likelihood, kw)
            return timed_runs(filt, ctl, args.warmup, args.steps, barrier_sync, ag, settle_steps)
        finally:
            if filt is not None:
                filt.close()
            if comm is not None:
                comm.close()

    parity = {}

    def sharded_parity(filt, ag, n_global, likelihood, kw):
        # the run's own evidence that the cross-device step is the filter
        # (VERDICT r5): PARITY_STEPS sharded steps from the initial state, the
        # final state gathered to rank 0 and compared bit for bit with one
        # handle of all n_global particles replaying the same steps there;
        # a mismatch fails the sharded mode on every rank (replicas, reason)
        import torch
        recs = ag.attempt(filt.run, 0, ctl[:PARITY_STEPS])
        st = ag.attempt(filt.get_state)
        ag.checkpoint("parity run")
        local = torch.from_numpy(np.ascontiguousarray(np.stack(st))).to(tdev)
        sizes = [torch.zeros(1, dtype=torch.int64, device=tdev) for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([local.shape[1]], dtype=torch.int64, device=tdev))
        nmax = int(max(int(t.item()) for t in sizes))
        pad = torch.zeros((4, nmax), dtype=torch.float64, device=tdev)
        pad[:, :local.shape[1]] = local
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad)
        if rank == 0:
            def check():
                full = np.concatenate([p[:, :int(n.item())].cpu().numpy() for p, n in zip(parts, sizes)], 1)
                if os.environ.get("SLAM_BENCH_PARITY_INJECT") == "1":          # tests
                    full[0, 12345] = np.nextafter(full[0, 12345], np.inf)
                one = DeviceParticleFilter(n_global, lm, **kw)
                try:
                    one.load_observations(zs)
                    ref = one.run(0, ctl[:PARITY_STEPS])
                    ref_state = one.get_state()
                finally:
                    one.close()
                ok, worst, first = compare_to_single(list(recs), tuple(full), list(ref), ref_state)
                parity.update(steps=PARITY_STEPS, bit_identical=ok, cov_max_rel=worst,
                              first_mismatch=first,
                              reference=f"one handle of {n_global:,} particles on rank 0's GPU, "
                                        "same seed, observations and controls",
                              resample_steps=int(sum(r["resampled"] for r in ref)))
                if not ok:
                    raise RuntimeError(f"sharded run differs from one handle: {first}")
            ag.attempt(check)
        ag.checkpoint("parity")

    def measure(likelihood, n_part=None):
        if args.mode == "sharded":
            return measure_sharded(likelihood, n_total)
        pf = DeviceParticleFilter(n_part or n_per_rank, lm, dt=dt, motion="velocity",
                                  likelihood=likelihood, seed=1234 + rank, device=local_rank)
        try:
            pf.load_observations(zs)
            return timed_runs(pf, ctl, args.warmup, args.steps, barrier_sync, settle_steps=settle_steps)
        finally:
            pf.close()

    def measure_numpy_stream(likelihood):
        # parity mode on the device: NumPy's RandomState stream drawn there
        # (rand / mvn(Q, NP) / mvn(R, NL) per step, bit-identical to the
        # reference's draws) and the observations simulated from the true pose
        pf = DeviceParticleFilter(NP_PER_GPU, lm, dt=dt, motion="velocity",
                                  likelihood=likelihood, seed=1234, device=local_rank)
        try:
            pf.use_numpy_stream(np.random.RandomState(1234))
            pf.load_truth(simulate_world.poses)
            pf.prepare_graphs()
            s0 = settle(pf.run, ctl, settle_steps)
            if args.warmup:
                pf.run(s0, ctl[s0:s0 + args.warmup], want_results=False)
            barrier_sync()
            t0 = time.perf_counter()
            pf.run(s0 + args.warmup, ctl[s0 + args.warmup:s0 + args.warmup + ns_steps])
            barrier_sync()
            return time.perf_counter() - t0, pf.rng_ring_info()
        finally:
            pf.close()

    sharded_error = None
    if args.mode == "sharded" and multi:
        # the sharded exchange needs every rank's GPU reachable over xGMI; if
        # any rank fails, every rank leaves measure_sharded at the same
        # agreement point with ShardedFailure, the ranks share their errors and
        # measure independent replicas instead, and the line says so
        # (config.parallelism, sharded_error)
        try:
            elapsed, out, timing, cap_ms = measure(args.likelihood)
        except ShardedFailure as e:
            phase, mine = e.args
            print(f"bench: sharded mode failed at {phase} ({mine or 'another rank'})", file=sys.stderr)
            errs = [None] * world
            dist.all_gather_object(errs, mine)
            sharded_error = f"{phase}: " + ("; ".join(x for x in errs if x) or "another rank failed")
            args.mode = "replicas"
            elapsed, out, timing, cap_ms = measure(args.likelihood)
    else:
        elapsed, out, timing, cap_ms = measure(args.likelihood)
    fused_ms, fused_n = timing[0]
    red_ms, red_n = timing[1]
    res_ms, res_n = timing[2]
    step_ms, step_n = timing[3]

    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # particles processed per step by the whole job
    n_job = n_total if args.mode == "sharded" else world * n_per_rank
    n_rank = n_total // world if args.mode == "sharded" else n_per_rank
    updates = n_job * NL * args.steps
    value = updates / elapsed
    fused_avg_s = fused_ms / 1e3 / max(fused_n, 1)
    if args.mode == "replicas":
        workload = (f"PF C2: {n_rank:,} particles/GPU x 100 landmarks, velocity motion model, "
                    "systematic resample")
    else:
        workload = (f"PF C3 form: one filter of {n_job:,} particles sharded {n_rank:,}/GPU x 100 "
                    "landmarks, velocity motion model, exact systematic resample across shards; "
                    "global np.sum-order normalisation")
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "particle-observation updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (simulated circular trajectory, 100 landmarks ~ U(-10,10)^2, "
                "on-device Philox noise)",
        "config": {"workload": workload, "particles_per_gpu": n_rank, "particles_total": n_job,
                   "landmarks": NL, "likelihood": args.likelihood,
                   "parallelism": f"{args.mode}{world}"},
        "roofline": fused_roofline(args.likelihood, n_rank, fused_avg_s),
        "breakdown_ms_per_step": {"fused": fused_ms / max(fused_n, 1),
                                  "reduce": red_ms / max(red_n, 1),
                                  "resample": res_ms / max(res_n, 1),
                                  "step_events": step_ms / max(step_n, 1)},
        "graph_capture_ms": cap_ms,
        "settle_steps": settle_steps,
        "resample_steps": int(sum(o["resampled"] for o in out)),
        "ess_near_steps": int(sum(o.get("ess_near", False) for o in out)),
        "closed_form_fallback_waves": int(sum(o.get("dd_waves", 0) for o in out)),
    }
    if world == 1 and args.likelihood != "product" and not strong:
        e2, _, t2, _ = measure("product")
        f2 = t2[0][0] / 1e3 / max(t2[0][1], 1)
        line["alt_modes"] = {"product": {"value": n_rank * NL * args.steps / e2,
                                         "ms_per_step": e2 * 1e3 / args.steps,
                                         "fused_avg_ms": f2 * 1e3,
                                         "roofline": fused_roofline("product", n_rank, f2)}}
        e4, ring = measure_numpy_stream(args.likelihood)
        line["alt_modes"]["numpy_stream"] = {
            "value": NP_PER_GPU * NL * ns_steps / e4, "ms_per_step": e4 * 1e3 / ns_steps,
            "steps": ns_steps, "ring": ring,
            "note": "the reference's own noise stream (MT19937 + polar normals, bit-identical to "
                    "np.random) drawn on the device with the observations simulated there"}
    if world == 1 and args.mode == "replicas" and not strong:
        # the sharded step's kernels on one shard (its overhead over the single handle)
        e3, _, t3, _ = measure_sharded(args.likelihood, NP_PER_GPU)
        line["sharded1"] = {"ms_per_step": e3 * 1e3 / args.steps,
                            "over_single": e3 / elapsed,
                            "fused_avg_ms": t3[0][0] / max(t3[0][1], 1)}
        # strong-scaling reference: one handle of 2^23 particles (BASELINE configs[2]'s
        # total) -- the single-GPU line that `--total-particles 8388608 --gpus N` divides
        e5, o5, t5, _ = measure(args.likelihood, STRONG_TOTAL)
        line["strong_single"] = {"particles": STRONG_TOTAL,
                                 "value": STRONG_TOTAL * NL * args.steps / e5,
                                 "ms_per_step": e5 * 1e3 / args.steps,
                                 "fused_avg_ms": t5[0][0] / max(t5[0][1], 1),
                                 "resample_steps": int(sum(o["resampled"] for o in o5))}
    if rank == 0 and world == 1 and not args.no_secondary and not strong:
        line["secondary"] = secondary(local_rank, cpu=not args.no_cpu_baseline)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not strong:
        line["cpu_baseline"] = cpu_baseline()
        line["cpu_baseline"]["gpu_over_cpu"] = value / line["cpu_baseline"]["value"]
        try:
            vb = cpu_baseline_vectorised()
            vb["gpu_over_cpu"] = value / vb["value"]
        except Exception as e:            # reported, never silently replaced
            vb = {"error": f"{type(e).__name__}: {e}"}
        line["cpu_baseline_vectorised"] = vb
    if parity:
        line["parity_check"] = parity
    if sharded_error is not None:
        line["sharded_error"] = sharded_error
    if args.mode == "sharded" and multi:
        # peer: the kernels' stores into IPC-mapped peer regions over xGMI;
        # rccl: the fallback's all-gathers / grouped send-recv (slam_dist_set_collective)
        line["config"]["exchange"] = exchange_mode[0]
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _raise(e):
    raise e


def len_blob(filt):
    import ctypes as C
    size = C.c_int64(0)
    filt._lib.slam_dist_handle_size(C.byref(size))
    return size.value


if __name__ == "__main__":
    main()
