"""Parity of the HIP particle filter (through the C-ABI) against the oracle and
the reference-generated golden fixtures.  Runs on the GPU box (-m gpu).

Tolerances (stated per test):
  * bit-exact: resampling indices given identical weights and offset, np.sum
    order, linear-model prediction noise addition;
  * one likelihood step from identical inputs (both modes): identical zero sets
    and <= 1e-12 relative on the non-zero weights (SURVEY 8(a) A6;
    conftest.weights_match);
  * multi-step trajectories (weights carried over steps, ulp differences of
    exp/sin/cos compound): identical zero sets, 1e-9 relative above 1e-290 and
    1e-299 absolute below (weights that passed through the subnormal range);
  * pose / covariance: 1e-6 relative (north_star), with identical max_idx.
"""
import numpy as np
import pytest

from conftest import golden, heavy_weights, rle_decode, stage_weights, weights_match

import pf_oracle as po

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def slamhip_pf():
    from slamhip import pf as dpf
    return dpf


@pytest.mark.parametrize("tag,n", [("r500", 500), ("r1000", 1000), ("r8193", 8193),
                                   ("r65536", 65536), ("r1m", 1 << 20)])
def test_resample_indices_bit_exact(slamhip_pf, tag, n):
    g = golden("pf_stages")
    w = stage_weights(tag, n, g[f"{tag}_wseed"])
    ref = rle_decode(g[f"{tag}_idx_vals"], g[f"{tag}_idx_counts"])
    with slamhip_pf.DeviceParticleFilter(n, np.zeros((1, 2))) as d:
        d.set_state(w=w)
        idx, nspec = d.resample_indices(float(g[f"{tag}_u"]))
    np.testing.assert_array_equal(idx, ref)
    assert nspec < n // 4 + 64


@pytest.mark.parametrize("n", [(1 << 20) + 4097, 1500000, (1 << 21) + 12345, 1 << 23,
                               (1 << 24) + 12345])
def test_resample_indices_numpy_above_2p20(slamhip_pf, n):
    """particle_filter.py:212-221 above the fixture sizes, bit-exact: the
    device's exact cumsum -- its one-launch form past 512 workgroups (the
    coalesced workgroup-total scan, 515 and 733 totals), then the two-launch
    form (that scan in one chunk of rounds, in two, and in five with a partial
    one and the tile offsets read from global memory) -- against np.cumsum +
    searchsorted (the oracle's systematic_indices) on the same weights, offset
    u x (1/NP) as particle_filter.py:214 forms it."""
    rs = np.random.RandomState(n % 9973)
    w = heavy_weights(rs, n, zero_frac=0.3)
    w = w / np.sum(w.reshape(1, n))
    u = 0.9 * float(rs.random_sample())
    ref = po.systematic_indices(w, u * (1.0 / n))
    # both forms where the one-launch form is available (set_scan_merged
    # refuses it otherwise), the two-launch form beyond
    for merged in ((True, False) if n < (1 << 21) else (False,)):
        with slamhip_pf.DeviceParticleFilter(n, np.zeros((1, 2))) as d:
            d.set_scan_merged(merged)
            d.set_state(w=w)
            idx, nspec = d.resample_indices(u)
        np.testing.assert_array_equal(idx, ref, err_msg=f"merged={merged}")
        assert 0 < nspec < n // 4


@pytest.mark.parametrize("n", [1, 7, 8, 100, 128, 129, 500, 1000, 8192, 8193, 20000, 100003, 1 << 20])
def test_weight_sum_numpy_order(slamhip_pf, n):
    g = golden("units")
    i = list(g["sum_sizes"]).index(n)
    a = heavy_weights(np.random.RandomState(n), n)
    with slamhip_pf.DeviceParticleFilter(n, np.zeros((1, 2))) as d:
        d.set_state(w=a)
        s = d.weight_sum()
    assert s == g["sum_out"][i]


@pytest.mark.parametrize("n", [(1 << 21) + 12345, 1 << 23])
def test_weight_sum_numpy_order_above_2p20(slamhip_pf, n):
    """np.sum (particle_filter.py:234) beyond the fixture's sizes: numpy itself
    on the same array is the reference (the step end's np.sum at these sizes,
    through the finalize's slice pre-pass, is tests/test_gpu_run_oracle.py)."""
    a = heavy_weights(np.random.RandomState(n % 100003), n)
    with slamhip_pf.DeviceParticleFilter(n, np.zeros((1, 2))) as d:
        d.set_state(w=a)
        s = d.weight_sum()
    assert s == np.sum(a.reshape(1, n))


@pytest.mark.parametrize("lik", ["product", "logsum"])
@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_likelihood_stage(slamhip_pf, tag, lik):
    g = golden("pf_stages")
    px, pw = g[f"lik_{tag}_px"], g[f"lik_{tag}_pw"]
    ref = g[f"lik_{tag}_out"]
    n = pw.size
    with slamhip_pf.DeviceParticleFilter(n, g[f"lik_{tag}_lm"], likelihood=lik) as d:
        d.set_state(px[0], px[1], px[2], pw)
        out = d.update(g[f"lik_{tag}_z"])
        _, _, _, w = d.get_state()
    worst = weights_match(w, ref, rtol=1e-12)
    print(f"likelihood {tag} {lik}: max relative weight error {worst:.3g}")
    assert out["max_idx"] == int(np.argmax(ref))


@pytest.mark.parametrize("lik", ["product", "logsum"])
def test_likelihood_stage_correlated_r(slamhip_pf, lik):
    """particle_filter.py:179-191 with a non-zero R01: sigmaxy = sqrt(R01) reaches
    mlab.bivariate_normal's rho term (the device's has_rho path, exp(-q / d2)).
    Stage "a" inputs; oracle pf_oracle.likelihood (gauss2d, the published
    formula); identical zero sets and <= 1e-12 relative (A6's bar)."""
    g = golden("pf_stages")
    px, pw = g["lik_a_px"], g["lik_a_pw"]
    lm, z = g["lik_a_lm"], g["lik_a_z"]
    r = np.array([[0.09, 0.0025], [0.0025, 0.09]])            # rho = 0.05 / 0.09
    ref, _ = po.likelihood(px[0], px[1], px[2], pw, lm, z, r)
    with slamhip_pf.DeviceParticleFilter(pw.size, lm, r=r, likelihood=lik) as d:
        d.set_state(px[0], px[1], px[2], pw)
        out = d.update(z)
        _, _, _, w = d.get_state()
    worst = weights_match(w, ref, rtol=1e-12)
    print(f"correlated R {lik}: max relative weight error {worst:.3g}")
    assert out["max_idx"] == int(np.argmax(ref))


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_predict_linear_stage(slamhip_pf, tag):
    g = golden("pf_stages")
    px = g[f"pred_{tag}_in"]
    n = px.shape[1]
    p = po.PFParams(n_particles=n)
    np.random.seed(int(g[f"pred_{tag}_seed"]))
    v = np.random.multivariate_normal([0.0, 0.0, 0.0], p.q, n)
    with slamhip_pf.DeviceParticleFilter(n, np.zeros((1, 2))) as d:
        d.set_state(px[0], px[1], px[2])
        d.predict((p.vel, p.omega), v)
        x, y, th, _ = d.get_state()
    np.testing.assert_allclose(np.vstack([x, y, th]), g[f"pred_{tag}_out"], rtol=0, atol=1e-14)


def test_predict_velocity_model(slamhip_pf):
    g = golden("motion")
    poses = g["poses"]
    n = poses.shape[0]
    dt, a1, a2, a3, a4, a5, a6, v, w = g["case1"]
    np.random.seed(int(g["seed1"]))
    gn = np.random.standard_normal(3 * n).reshape(n, 3)
    with slamhip_pf.DeviceParticleFilter(n, np.zeros((1, 2)), dt=dt, motion="velocity",
                                         alphas=(a1, a2, a3, a4, a5, a6)) as d:
        d.set_state(poses[:, 0], poses[:, 1], poses[:, 2])
        d.predict((v, w), gn)
        x, y, th, _ = d.get_state()
    np.testing.assert_allclose(np.stack([x, y, th], axis=1), g["noisy1"], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("lik", ["product", "logsum"])
def test_c1_end_to_end_vs_reference(lik):
    """BASELINE config 1 through the drop-in ParticleFilter: 500 particles x 20
    landmarks x 1000 steps, seed 0, NumPy noise stream."""
    from particle_filter import ParticleFilter
    g = golden("pf_c1")
    np.random.seed(int(g["seed"]))
    pf = ParticleFilter(100, n_particles=int(g["n"]), landmarks=g["lm"], likelihood=lik)
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


def test_step_covariance_vs_oracle(slamhip_pf):
    rs = np.random.RandomState(5)
    n, nl = 3000, 30
    lm = rs.uniform(-10, 10, (nl, 2))
    p = po.PFParams(n_particles=n, landmarks=lm)
    orc = po.PFOracle(p)
    orc.x += rs.normal(size=n) * 0.3
    orc.y += rs.normal(size=n) * 0.3
    with slamhip_pf.DeviceParticleFilter(n, lm) as d:
        d.set_state(orc.x, orc.y, orc.th, orc.w)
        world = po.PFWorld(p)
        np.random.seed(9)
        for k in range(25):
            world.advance()
            ofs_u = np.random.rand() if orc.needs_resample() else None
            assert d.resample_next == (ofs_u is not None)
            noise = np.random.multivariate_normal([0.0, 0.0, 0.0], p.q, n)
            z = world.observe()
            ro = orc.step(z, noise, None if ofs_u is None else ofs_u * p.np_recip)
            rd = d.step((p.vel, p.omega), z, noise, np.nan if ofs_u is None else ofs_u)
            assert rd["max_idx"] == ro["max_idx"]
            np.testing.assert_allclose(rd["x_est"], ro["x_est"], rtol=1e-6)
            np.testing.assert_allclose(rd["cov"], ro["cov"], rtol=1e-6, atol=1e-12)
            ess_after = po.ess_of(orc.w)       # device reports the post-step ESS
            assert abs(rd["ess"] - ess_after) <= 1e-9 * ess_after
            assert rd["resample_next"] == (ess_after < p.ess_th)


def test_never_resampling_filter_degenerate_weights(slamhip_pf):
    """ESS threshold 0: the filter never resamples, the weights degenerate and
    most particles reach weight 0 while their likelihood falls below the
    closed form's range (fast_min_l).  Those skip the exact sequential product
    (0 x any finite likelihood is 0); the weights, zero set included, and the
    estimate still follow the reference step by step."""
    rs = np.random.RandomState(12)
    n, nl = 4000, 30
    lm = rs.uniform(-10, 10, (nl, 2))
    p = po.PFParams(n_particles=n, landmarks=lm)
    p.ess_th = 0.0
    orc = po.PFOracle(p)
    with slamhip_pf.DeviceParticleFilter(n, lm, likelihood="logsum", ess_threshold=0.0) as d:
        world = po.PFWorld(p)
        np.random.seed(4)
        for k in range(30):
            world.advance()
            noise = np.random.multivariate_normal([0.0, 0.0, 0.0], p.q, n)
            z = world.observe()
            ro = orc.step(z, noise, None)
            rd = d.step((p.vel, p.omega), z, noise, np.nan)
            assert not rd["resampled"]
            assert rd["max_idx"] == ro["max_idx"], k
            np.testing.assert_allclose(rd["x_est"], ro["x_est"], rtol=1e-6)
            weights_match(d.get_state()[3], orc.w, rtol=1e-9, floor=1e-290)
        assert np.count_nonzero(orc.w == 0) > n // 2       # the regime the skip serves


@pytest.mark.parametrize("motion", ["linear", "velocity"])
def test_device_rng_run_tracks_truth(slamhip_pf, motion):
    """Device-resident run (bench path): on-device Philox noise, device-decided
    resampling; the estimate must track the simulated truth."""
    rs = np.random.RandomState(1)
    n, nl, steps = 1 << 16, 100, 40
    lm = rs.uniform(-10, 10, (nl, 2))
    p = po.PFParams(n_particles=n, landmarks=lm, motion=motion)
    world = po.PFWorld(p)
    np.random.seed(3)
    zs, xs = [], []
    for _ in range(steps):
        xs.append(world.advance().copy())
        zs.append(world.observe())
    with slamhip_pf.DeviceParticleFilter(n, lm, motion=motion, seed=7) as d:
        d.load_observations(np.array(zs))
        out = d.run(0, np.tile([p.vel, p.omega], (steps, 1)))
    err = np.array([np.hypot(*(o["x_est"][:2] - x[:2])) for o, x in zip(out, xs)])
    assert np.all(np.isfinite(err)) and np.median(err) < 0.5
    assert sum(o["resampled"] for o in out) >= 1


def test_scan_merged_matches_two_launch(slamhip_pf):
    """The one-launch exact cumsum (co-resident grid) and the two-launch form
    must give bit-identical runs: same seed, same resampling decisions."""
    rs = np.random.RandomState(4)
    n, nl, steps = 1 << 20, 100, 24
    lm = rs.uniform(-10, 10, (nl, 2))
    p = po.PFParams(n_particles=n, landmarks=lm, motion="velocity")
    world = po.PFWorld(p)
    np.random.seed(11)
    zs = []
    for _ in range(steps):
        world.advance()
        zs.append(world.observe())
    ctl = np.tile([p.vel, p.omega], (steps, 1))
    outs, states = [], []
    for merged in (True, False):
        with slamhip_pf.DeviceParticleFilter(n, lm, motion="velocity", seed=5) as d:
            d.set_scan_merged(merged)
            d.load_observations(np.array(zs))
            outs.append(d.run(0, ctl))
            states.append(d.get_state())
    assert sum(o["resampled"] for o in outs[0]) >= 1
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a["x_est"], b["x_est"])
        np.testing.assert_array_equal(a["cov"], b["cov"])
        assert a["max_idx"] == b["max_idx"] and a["resampled"] == b["resampled"]
    for a, b in zip(*states):
        np.testing.assert_array_equal(a, b)


def test_resample_decision_by_host_dot_near_threshold(slamhip_pf):
    """particle_filter.py:210-211 decides from `1 / (pw @ pw.T)` (host BLAS
    order).  With the confirmation band widened to every step, each decision is
    re-formed on the host from the device's normalised weights and the device
    follows it: the next step resamples exactly when NumPy's ESS < ESS_TH."""
    rs = np.random.RandomState(2)
    n, nl, steps = 20_000, 20, 12
    lm = rs.uniform(-10, 10, (nl, 2))
    p = po.PFParams(n_particles=n, landmarks=lm)
    world = po.PFWorld(p)
    np.random.seed(5)
    with slamhip_pf.DeviceParticleFilter(n, lm, seed=3) as d:
        d.ESS_CONFIRM_BAND = np.inf
        prev = False
        n_res = 0
        for _ in range(steps):
            world.advance()
            z = world.observe()
            noise = np.random.multivariate_normal([0.0, 0.0, 0.0], p.q, n)
            u = np.random.rand() if d.resample_next else np.nan
            out = d.step((p.vel, p.omega), z, noise, u)
            assert out["resampled"] == prev
            assert out["ess_confirmed"]
            pw = d.get_state()[3]
            ess = float(np.reciprocal(pw @ pw.T))
            assert out["ess_host"] == ess
            assert out["resample_next"] == (ess < d.cfg.ess_threshold)
            assert abs(out["ess"] - ess) <= 1e-12 * ess
            prev = out["resample_next"]
            n_res += prev
        assert n_res >= 1
        # weights placed on the threshold: set_state's decision is NumPy's dot
        w = np.zeros(n)
        k = int(d.cfg.ess_threshold)
        w[:k] = 1.0 / k
        d.set_state(w=w)
        dec = float(np.reciprocal(w @ w.T)) < d.cfg.ess_threshold
        assert d.resample_next == dec
        world.advance()
        out = d.step((p.vel, p.omega), world.observe(),
                     np.random.multivariate_normal([0.0, 0.0, 0.0], p.q, n),
                     np.random.rand() if dec else np.nan)
        assert out["resampled"] == dec


@pytest.mark.parametrize("n", [1 << 20, (1 << 21) + 12345, (1 << 24) + 12345])
def test_step_end_against_numpy_on_the_devices_weights(slamhip_pf, n):
    """The device-resident step end (particle_filter.py:115-117, :210, :234) on
    the device's own w_un: np.sum, max, the first argmax and ESS exact or to
    1e-12, the covariance to 1e-8 against np.cov of the device's state.  One
    size per finalize form: 2^20 the one-workgroup fast kernel, 2^21 + 12,345
    the fast kernel after the slice pre-pass, 2^24 + 12,345 (17 slices, 2,049
    buffers) the general finalize_deferred_kernel."""
    import bench
    lm, zs, (vel, omega, dt) = bench.simulate_world(8)
    ctl = np.tile([vel, omega], (8, 1))
    with slamhip_pf.DeviceParticleFilter(n, lm, dt=dt, motion="velocity", likelihood="logsum",
                                         seed=3) as d:
        d.load_observations(zs)
        recs = d.run(0, ctl[:3])
        w_un, s = d.get_weights_raw()
        x, y, th, w = d.get_state()
    r = recs[len(recs) - 1]
    assert s == np.sum(w_un) and r["weight_sum"] == s
    np.testing.assert_array_equal(w, w_un / s)
    assert r["max_val"] == w.max() and r["max_idx"] == int(np.argmax(w))
    np.testing.assert_array_equal(r["x_est"], [x[r["max_idx"]], y[r["max_idx"]], th[r["max_idx"]]])
    np.testing.assert_allclose(r["ess"], 1.0 / np.dot(w, w), rtol=1e-12)
    np.testing.assert_allclose(r["cov"], po.weighted_cov(x, y, th, w), rtol=1e-8, atol=1e-14)
    assert r["status"] == 0
