"""The benchmarked path itself against the oracle: slam_pf_run (hipGraph step
batches, the Philox HOSTNOISE=false instantiation of pf_fused_kernel with the
deferred normalisation, the device-drawn resample offset) checked step by step
against PFOracle.step (particle_filter.py:102-117, motion_model.py:31-62,
:200-237) on the device's own motion normals and offsets.

How the device's noise reaches the oracle: the fused kernel draws particle
2p's normals as the first three and particle 2p + 1's as the last three of
pair_normals(p, rstep = step number, seed) (common.hpp); slam_debug_pair_normals
evaluates that same device function for every pair of a step, and the offset
is restated on the host from the same Philox block (philox_ref.resample_u,
bit-exact integer words).  The step's result never depends on which path made
the normals: the test uses the identical values.

Lockstep (handle A): the batch is one step (run(k, 1): a one-step graph), and
before every step the oracle is re-based on the device's state (particles and
current weights, get_state), so every transition is compared from identical
inputs, the resample steps included (indices bit-exact through
slam_pf_resample_indices on alternate resample steps; on the others the gather
runs from the previous batch's step-end prefix and is checked through the
particles).  Per step:
  * resample decision, status 0, argmax identical; x_est, cov 1e-6 relative
    (cov atol 1e-12) -- north_star's bar;
  * particles |d| <= 1e-12 (|ref| + |v^/w^|) (the turn radius, test_gpu_c2.py);
  * weights: the oracle's likelihood of the device's predicted particles,
    identical zero sets, <= 1e-11 relative (subnormal dips:
    conftest.subnormal_dip_rtol), as test_gpu_c2.py;
  * the step end on the device's own w_un (slam_pf_get_weights_raw): the
    divisor s bit-identical to np.sum(w_un) (particle_filter.py:234) and to the
    record's weight_sum; max_val / argmax bit-identical to numpy's on the
    device's normalised weights; ESS and cov of the device's state (fixed
    device order) to 1e-10 / 1e-8.
Batch machinery (handle B): the same steps replayed as the bench replays them
(8-, 4-, 2- and 1-step graphs, resamples inside a graph, batches that start on
a resample step and reuse the previous batch's prefix) must give records and
a final state bit-identical to handle A's.

Sizes: C2 itself (2^20 x 100, 24 steps, >= 3 resamples); above 2^20, where the
step end adds the finalize's slice pre-pass (pf_finalize.inl), 2^21 + 12,345
and 2^23 particles with 20 landmarks (the oracle's per-particle factors at
2^23 x 100 would need ~13 GB of host memory per step) and ESS_TH = NP / 10 (a
constructor parameter; with 20 landmarks NP / 100 is first crossed after ~8
steps).
"""
import os

import numpy as np
import pytest

import pf_oracle as po
from conftest import subnormal_dip_rtol, weights_match
from philox_ref import resample_u

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))


def _normals(n, rstep, seed):
    import ctypes as C
    from slamhip import _lib
    pairs = (n + 1) // 2
    out = np.empty((pairs, 6))
    _lib.check(_lib.load().slam_debug_pair_normals(0, 0, pairs, rstep, seed,
                                                   out.ctypes.data_as(C.POINTER(C.c_double))),
               "slam_debug_pair_normals")
    return out.reshape(2 * pairs, 3)[:n]


def _turn_radius(p, g):
    """|v^ / w^| of motion_model.py:46-50 for the standard normals g."""
    a1, a2, a3, a4, _, _ = p.alphas
    v, w = p.vel, p.omega
    sv = (a1 * v ** 2) + (a2 * w ** 2)
    sw = (a3 * v ** 2) + (a4 * w ** 2)
    return np.abs((v + sv ** 2 * g[:, 0]) / (w + sw ** 2 * g[:, 1]))


def _dip_tolerance(x, y, th, p, z, w_prev, chunk=1 << 16):
    """conftest.subnormal_dip_rtol of the oracle's factors on the device's
    particles, per particle chunk (memory), and the products themselves."""
    n = x.size
    bn = np.empty(n)
    rt = np.empty(n)
    from concurrent.futures import ThreadPoolExecutor

    def part(lo):
        hi = min(n, lo + chunk)
        F = po.landmark_factors(x[lo:hi], y[lo:hi], th[lo:hi], p.lm, z, p.r)
        bn[lo:hi] = F.prod(axis=1)
        rt[lo:hi] = subnormal_dip_rtol(F, 1e-11, w_prev[lo:hi])

    with ThreadPoolExecutor(THREADS) as ex:
        list(ex.map(part, range(0, n, chunk)))
    return bn, rt


def _inputs(n, nl, steps, lm_seed, obs_seed, ess_th):
    rs = np.random.RandomState(lm_seed)
    lm = rs.uniform(-10, 10, (nl, 2))
    p = po.PFParams(n_particles=n, landmarks=lm, motion="velocity")
    if ess_th is not None:
        p.ess_th = float(ess_th)
    world = po.PFWorld(p)
    np.random.seed(obs_seed)
    zs = []
    for _ in range(steps):
        world.advance()
        zs.append(world.observe())
    return p, np.array(zs), np.tile([p.vel, p.omega], (steps, 1))


def _handle(p, seed):
    from slamhip.pf import DeviceParticleFilter
    return DeviceParticleFilter(p.np, p.lm, dt=p.dt, motion="velocity", likelihood="logsum",
                                alphas=p.alphas, seed=seed, ess_threshold=p.ess_th)


def _check_step_end(d, rd, n):
    """The step end on the device's own weights (module docstring)."""
    x, y, th, w = d.get_state()
    w_un, s = d.get_weights_raw()
    assert s == rd["weight_sum"], (s, rd["weight_sum"])
    assert s == np.sum(w_un.reshape(1, n)), (s, np.sum(w_un.reshape(1, n)))
    np.testing.assert_array_equal(w, po.normalize(w_un))
    assert rd["max_val"] == np.max(w) and rd["max_idx"] == int(np.argmax(w))
    np.testing.assert_array_equal(rd["x_est"], [x[rd["max_idx"]], y[rd["max_idx"]], th[rd["max_idx"]]])
    ess = po.ess_of(w)
    assert abs(rd["ess"] - ess) <= 1e-10 * ess
    np.testing.assert_allclose(rd["cov"], po.weighted_cov(x, y, th, w), rtol=1e-8, atol=1e-14)
    return x, y, th, w


def run_lockstep(n, nl, steps, seed, lm_seed, obs_seed, min_resamples, batches, ess_th=None):
    p, zs, ctl = _inputs(n, nl, steps, lm_seed, obs_seed, ess_th)
    orc = po.PFOracle(p)
    orc.threads = THREADS
    recs, n_res, n_idx = [], 0, 0
    with _handle(p, seed) as a:
        a.load_observations(zs)
        x, y, th, w = a.get_state()
        for k in range(steps):
            orc.x, orc.y, orc.th, orc.w = x, y, th, w          # identical inputs
            g = _normals(n, k, seed)
            res = orc.needs_resample()
            assert a.resample_next == res, k
            u = resample_u(k, seed) if res else None
            ro = orc.step(zs[k], g, None if u is None else u * p.np_recip)
            if res:
                n_res += 1
                if n_res % 2:                                   # alternate: direct indices
                    idx, _ = a.resample_indices(u)
                    np.testing.assert_array_equal(idx, ro["idx"])
                    n_idx += 1
            rd = a.run(k, ctl[k:k + 1])[0]
            recs.append(rd)
            assert rd["status"] == 0, (k, rd["status"])
            assert rd["resampled"] == ro["resampled"], k
            assert rd["max_idx"] == ro["max_idx"], (k, rd["max_idx"], ro["max_idx"])
            np.testing.assert_allclose(rd["x_est"], ro["x_est"], rtol=1e-6)
            np.testing.assert_allclose(rd["cov"], ro["cov"], rtol=1e-6, atol=1e-12)
            x, y, th, w = _check_step_end(a, rd, n)
            rad = _turn_radius(p, g)
            for got, ref in ((x, orc.x), (y, orc.y), (th, orc.th)):
                bad = np.abs(got - ref) > 1e-12 * (np.abs(ref) + rad)
                assert not bad.any(), (k, int(bad.sum()), np.flatnonzero(bad)[:5])
            bn, rtol = _dip_tolerance(x, y, th, p, zs[k], ro["w_prev"])
            worst = weights_match(w, po.normalize(ro["w_prev"] * bn), rtol=rtol)
            assert rd["resample_next"] == (po.ess_of(w) < p.ess_th), k
            print(f"step {k}: resampled {rd['resampled']} ess {rd['ess']:.6g} "
                  f"worst weight rel {worst:.3g}")
        state_a = a.get_state()
    assert n_res >= min_resamples and n_idx >= 1, (n_res, n_idx)

    # handle B: the same steps in the bench's batch shapes
    with _handle(p, seed) as b:
        b.load_observations(zs)
        b.prepare_graphs()
        k, got = 0, []
        for L in batches:
            got += list(b.run(k, ctl[k:k + L]))
            k += L
        assert k == steps
        state_b = b.get_state()
    inside = 0
    for j, (ra, rb) in enumerate(zip(recs, got)):
        for f in ("x_est", "cov", "max_val", "max_idx", "ess", "weight_sum", "resampled",
                  "resample_next", "status"):
            assert np.array_equal(ra[f], rb[f]), (j, f, ra[f], rb[f])
    starts = np.cumsum([0] + list(batches))[:-1]
    inside = sum(1 for j, r in enumerate(recs) if r["resampled"] and j not in starts)
    for u, v in zip(state_a, state_b):
        np.testing.assert_array_equal(u, v)
    print(f"n={n} nl={nl}: {steps} steps, {n_res} resamples ({inside} inside a graph batch), "
          f"batches {batches}")
    return inside


def test_c2_bench_path_lockstep_vs_oracle():
    """C2 (2^20 x 100): 24 one-step graph batches against the oracle, then the
    bench's batch shapes bit-identical to them."""
    inside = run_lockstep(1 << 20, 100, 24, seed=9, lm_seed=21, obs_seed=22, min_resamples=3,
                          batches=(8, 8, 5, 3))
    assert inside >= 1


def test_ragged_above_2p20_lockstep_vs_oracle():
    """2^21 + 12,345 particles (two finalize slices, a ragged last block)."""
    n = (1 << 21) + 12345
    run_lockstep(n, 20, 7, seed=4, lm_seed=23, obs_seed=24, min_resamples=2, batches=(3, 4),
                 ess_th=n / 10)


def test_2p23_single_handle_lockstep_vs_oracle():
    """The single 2^23 handle (C3's reference and the bench's strong_single
    line): eight finalize slices."""
    n = 1 << 23
    run_lockstep(n, 20, 8, seed=11, lm_seed=25, obs_seed=26, min_resamples=2, batches=(3, 4, 1),
                 ess_th=n / 10)
