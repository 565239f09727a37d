"""The device replica of NumPy's RandomState stream against RandomState itself
(the reference's noise source, particle_filter.py:152/:165/:214), and the
particle filter driven by it.  Bar: bit-exact draws and identical states;
the C1 run with device-drawn noise meets the same fixture bars as the
host-noise run (tests/test_gpu_pf.py)."""
import numpy as np
import pytest

from conftest import golden, weights_match

pytestmark = pytest.mark.gpu


def _same_state(a, b):
    np.testing.assert_array_equal(np.asarray(a[1], np.uint32), np.asarray(b[1], np.uint32))
    assert (int(a[2]), int(a[3])) == (int(b[2]), int(b[3]))
    assert np.float64(a[4]).view(np.uint64) == np.float64(b[4]).view(np.uint64)


def _bits(a):
    return np.asarray(a, np.float64).view(np.uint64)


@pytest.mark.parametrize("seed,warm,g", [(0, 0, 1), (1, 3, 2), (2, 1, 3), (3, 0, 1000),
                                         (4, 311, 1501), (5, 312, 6000), (6, 7, 100001),
                                         (7, 0, 3 * (1 << 20) + 200),
                                         # > 4096 emit blocks: the prefix launch (rng_api.hip)
                                         (8, 5, 3 * (1 << 22) + 7),
                                         # odd stream positions: candidates start at every
                                         # word alignment of the ring's 16-byte loads
                                         (9, -311, 20001), (10, -3, 3 * (1 << 20) + 1)])
def test_standard_normal_matches_numpy(seed, warm, g):
    """warm < 0: the state's position set to -warm (an odd word offset)."""
    from slamhip.rng import DeviceRandomState
    rs = np.random.RandomState(seed)
    if warm >= 0:
        rs.random_sample(warm)
    else:
        st = rs.get_state()
        rs.set_state((st[0], st[1], -warm, 0, 0.0))
    with DeviceRandomState(rs, device=0) as d:
        out = d.standard_normal(g)
        ref = rs.standard_normal(g)
        bad = np.flatnonzero(_bits(out) != _bits(ref))
        assert bad.size == 0, (bad[:5], out[bad[:5]], ref[bad[:5]])
        _same_state(d.get_state(), rs.get_state())


def test_interleaved_calls_match_numpy():
    from slamhip.rng import DeviceRandomState
    rs = np.random.RandomState(23)
    with DeviceRandomState(rs, device=0) as d:
        for n_pre, g in [(1, 5), (3, 1), (0, 2), (1, 7), (2, 0), (0, 1), (1, 4), (700, 3001),
                         (1, 1)]:
            if n_pre:
                np.testing.assert_array_equal(d.random_sample(n_pre), rs.random_sample(n_pre))
            if g:
                np.testing.assert_array_equal(_bits(d.standard_normal(g)), _bits(rs.standard_normal(g)))
            _same_state(d.get_state(), rs.get_state())


def test_many_requests_cross_refill_rounds():
    """200 requests of one size: the word ring refills about three times and
    wraps (it holds one round plus one request, rng_api.hip mt_reserve), every
    request bit-exact."""
    from slamhip.rng import DeviceRandomState
    rs = np.random.RandomState(31)
    with DeviceRandomState(rs, device=0) as d:
        for k in range(200):
            out, ref = d.standard_normal(100001), rs.standard_normal(100001)
            bad = np.flatnonzero(_bits(out) != _bits(ref))
            assert bad.size == 0, (k, bad[:5])
        _same_state(d.get_state(), rs.get_state())


def test_bench_size_ring_within_2gb():
    """The 2^20-particle handle's ring (<= 2 GB) still feeds
    64 requests per refill round."""
    from slamhip.pf import DeviceParticleFilter
    lm = np.random.RandomState(2).uniform(-10, 10, (100, 2))
    with DeviceParticleFilter(1 << 20, lm, motion="velocity", likelihood="logsum") as d:
        d.use_numpy_stream(np.random.RandomState(5))
        info = d.rng_ring_info()
    assert info["ring_bytes"] <= 2 << 30, info
    assert info["requests_per_round"] >= 64, info


def _expected_state_after(seed, steps, resampled, n, nl):
    """np.random after the reference's draws: [rand() if resampling] ->
    mvn(Q, n) -> mvn(R, nl) per step (standard_normal counts)."""
    rs = np.random.RandomState(seed)
    for k in range(steps):
        if resampled[k]:
            rs.random_sample()
        rs.standard_normal(3 * n)
        rs.standard_normal(2 * nl)
    return rs.get_state()


@pytest.mark.parametrize("lik", ["product", "logsum"])
def test_c1_end_to_end_device_stream(lik):
    """BASELINE config 1 (500 x 20 x 1000 steps, seed 0) with every draw made on
    the device from NumPy's stream: the fixture's trajectory, and np.random left
    where the reference leaves it."""
    from particle_filter import ParticleFilter
    g = golden("pf_c1")
    np.random.seed(int(g["seed"]))
    n = int(g["n"])
    pf = ParticleFilter(100, n_particles=n, landmarks=g["lm"], likelihood=lik, noise="mt19937")
    steps = len(g["x_est"])
    x_est = np.zeros((steps, 3))
    max_idx = np.zeros(steps, dtype=np.int64)
    res = np.zeros(steps, dtype=bool)
    keep = {int(k): j for j, k in enumerate(g["keep_steps"])}
    for k in range(steps):
        was = pf.dev.resample_next
        _, xt, xe, px, _, mi, mv = pf.main_pf()
        x_est[k], max_idx[k], res[k] = xe[:, 0], mi, was
        np.testing.assert_array_equal(xt[:, 0], g["x_true"][k])
        if k in keep:
            j = keep[k]
            np.testing.assert_allclose(px, g["px_keep"][j], rtol=1e-6, atol=1e-9)
            weights_match(pf.weights, g["pw_keep"][j], rtol=1e-9, floor=1e-290)
    np.testing.assert_array_equal(res, g["resampled"])
    np.testing.assert_array_equal(max_idx, g["max_idx"])
    np.testing.assert_allclose(x_est, g["x_est"], rtol=1e-6, atol=1e-9)
    _same_state(np.random.get_state(),
                _expected_state_after(int(g["seed"]), steps, g["resampled"], n, len(g["lm"])))


@pytest.mark.parametrize("motion", ["linear", "velocity"])
def test_device_stream_matches_host_stream(motion):
    """Device-drawn noise and device-simulated observations give the same
    filter, bit for bit, as host-drawn ones (same seed): sync steps with the
    returned z checked against the host's observation, then a device-resident
    batch (load_truth + run)."""
    from slamhip.pf import DeviceParticleFilter
    from mylib import transform as tf
    n, nl, steps = 20000, 30, 12
    rs = np.random.RandomState(4)
    lm = rs.uniform(-10, 10, (nl, 2))
    r = np.diag([0.3, 0.3]) ** 2
    q = np.diag([0.03, 0.03, np.deg2rad(2.0)]) ** 2
    dt, v, om = 0.1, 1.0, 0.1
    poses = np.zeros((steps, 3))
    x = np.array([10.0, 0.0, np.pi / 2])
    for k in range(steps):
        x = np.array([x[0] + v * dt * np.cos(x[2]), x[1] + v * dt * np.sin(x[2]), x[2] + om * dt])
        poses[k] = x
    kw = dict(motion=motion, likelihood="logsum", ess_threshold=n / 2.0)   # resample often
    host = np.random.RandomState(99)
    st0 = host.get_state()
    ref = []
    with DeviceParticleFilter(n, lm, **kw) as d:
        for k in range(steps):
            u = host.random_sample() if d.resample_next else np.nan
            noise = (host.multivariate_normal([0.0, 0.0, 0.0], q, n) if motion == "linear"
                     else host.standard_normal(3 * n).reshape(n, 3))
            z = tf.world2robot(poses[k].reshape(3, 1), lm) + host.multivariate_normal([0.0, 0.0], r, nl)
            ref.append((d.step((v, om), z, noise, u), z))
    with DeviceParticleFilter(n, lm, **kw) as d:
        d.use_numpy_stream(st0)
        for k in range(steps):
            out = d.step_truth((v, om), poses[k].reshape(3, 1), want_z=True)
            rk, zk = ref[k]
            np.testing.assert_array_equal(_bits(out["z"]), _bits(zk))
            np.testing.assert_array_equal(_bits(out["x_est"]), _bits(rk["x_est"]))
            assert (out["max_idx"], out["resampled"]) == (rk["max_idx"], rk["resampled"])
        _same_state(d.rng_state(), host.get_state())
    assert any(rk["resampled"] for rk, _ in ref)
    with DeviceParticleFilter(n, lm, **kw) as d:
        d.use_numpy_stream(st0)
        d.load_truth(poses)
        outs = d.run(0, np.tile([v, om], (steps, 1)))
        for k in range(steps):
            rk, _ = ref[k]
            np.testing.assert_array_equal(_bits(outs[k]["x_est"]), _bits(rk["x_est"]))
            assert (outs[k]["max_idx"], outs[k]["resampled"]) == (rk["max_idx"], rk["resampled"])
        _same_state(d.rng_state(), host.get_state())
