"""Pin the oracle (oracle/*.py) against fixtures produced by the reference
itself (tests/golden/make_golden.py).  CPU only.  Bit-exact: the fixtures were
generated on this build container's NumPy/OpenBLAS; on a host whose NumPy picks
a different SIMD exp/BLAS kernel the transcendental-dependent checks fall back
to a 1e-12 relative tolerance (flagged by ``_same_machine``)."""
import numpy as np
import pytest

from conftest import golden, rle_decode, stage_weights

import pf_oracle as po
import ekf_oracle as eo


def _same_machine():
    g = golden("units")
    return np.array_equal(po.gauss2d(g["gdx"], g["gdy"], 0.3, 0.3, 0.0), g["gauss"])


def _eq(a, b, rtol=1e-12):
    if _same_machine():
        np.testing.assert_array_equal(a, b)
    else:
        np.testing.assert_allclose(a, b, rtol=rtol, atol=0)


def test_limit_angle_exact():
    g = golden("units")
    out = np.array([po.wrap_angle(a) for a in g["ang_in"]])
    np.testing.assert_array_equal(out, g["ang_out"])
    np.testing.assert_array_equal(po.wrap_angles(g["ang_in"]), g["ang_out"])


def test_transforms():
    g = golden("units")
    w2r = np.stack([po.to_robot_frame(p, q) for p, q in zip(g["poses"], g["pts"])])
    r2w = np.stack([po.to_world_frame(p, q) for p, q in zip(g["poses"], g["pts"])])
    _eq(w2r, g["w2r"])
    _eq(r2w, g["r2w"])


def test_gauss2d():
    g = golden("units")
    _eq(po.gauss2d(g["gdx"], g["gdy"], 0.3, 0.3, 0.0), g["gauss"])
    assert (g["gauss"][-3:] == 0).sum() >= 1          # an underflowing factor is covered


@pytest.mark.parametrize("i", range(13))
def test_numpy_order_sum(i):
    from conftest import heavy_weights
    g = golden("units")
    n = int(g["sum_sizes"][i])
    a = heavy_weights(np.random.RandomState(n), n)
    assert np.sum(a.reshape(1, n)) == g["sum_out"][i]
    if n <= 100003:
        assert po.numpy_order_sum(a) == g["sum_out"][i]


@pytest.mark.parametrize("tag,n", [("r500", 500), ("r1000", 1000), ("r8193", 8193),
                                   ("r65536", 65536), ("r1m", 1 << 20)])
def test_resample_indices_exact(tag, n):
    g = golden("pf_stages")
    w = stage_weights(tag, n, g[f"{tag}_wseed"])
    idx = po.systematic_indices(w, float(g[f"{tag}_u"]) * (1 / n))
    ref = rle_decode(g[f"{tag}_idx_vals"], g[f"{tag}_idx_counts"])
    np.testing.assert_array_equal(idx, ref)


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_likelihood_stage(tag):
    g = golden("pf_stages")
    px = g[f"lik_{tag}_px"]
    r = np.diag([0.3, 0.3]) ** 2
    w, bn = po.likelihood(px[0], px[1], px[2], g[f"lik_{tag}_pw"], g[f"lik_{tag}_lm"],
                          g[f"lik_{tag}_z"], r)
    _eq(w, g[f"lik_{tag}_out"])
    if tag == "c":
        w2, _ = po.likelihood_loop(px[0], px[1], px[2], g[f"lik_{tag}_pw"],
                                   g[f"lik_{tag}_lm"], g[f"lik_{tag}_z"], r)
        np.testing.assert_array_equal(w, w2)


def test_likelihood_all_underflow_path():
    # case "b" (spread 2 m, observations uniform): exercise NaN -> 1/NP
    g = golden("pf_stages")
    out = g["lik_b_out"]
    assert np.all(out == out[0]) and out[0] == 1 / out.size


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_predict_linear_stage(tag):
    g = golden("pf_stages")
    px = g[f"pred_{tag}_in"]
    n = px.shape[1]
    p = po.PFParams(n_particles=n)
    np.random.seed(int(g[f"pred_{tag}_seed"]))
    v = np.random.multivariate_normal([0.0, 0.0, 0.0], p.q, n)
    xn, yn, tn = po.motion_linear(px[0], px[1], px[2], p.dt, p.vel, p.omega)
    out = np.vstack([xn + v[:, 0], yn + v[:, 1], tn + v[:, 2]])
    _eq(out, g[f"pred_{tag}_out"])


@pytest.mark.parametrize("c", range(3))
def test_motion_model(c):
    g = golden("motion")
    dt, a1, a2, a3, a4, a5, a6, v, w = g[f"case{c}"]
    poses = g["poses"]
    np.random.seed(int(g[f"seed{c}"]))
    gn = np.random.standard_normal(3 * poses.shape[0]).reshape(-1, 3)
    xn, yn, tn = po.motion_velocity(poses[:, 0], poses[:, 1], poses[:, 2], v, w, dt,
                                    (a1, a2, a3, a4, a5, a6), gn)
    _eq(np.stack([xn, yn, tn], axis=1), g[f"noisy{c}"])
    clean = np.array([po.motion_velocity_exact(p, v, w, dt) for p in poses])
    _eq(clean, g[f"clean{c}"])


def test_pf_c1_end_to_end():
    """BASELINE config 1 (500 particles x 20 landmarks x 1000 steps, seed 0)."""
    g = golden("pf_c1")
    p = po.PFParams(n_particles=int(g["n"]), landmarks=g["lm"])
    pf, rows = po.run_reference_order(p, int(g["seed"]), len(g["x_est"]))
    ks = list(g["keep_steps"])
    res_steps = [r["k"] for r in rows if r["resampled"]]
    assert res_steps[:len(g["idx_steps"])] == list(g["idx_steps"])
    np.testing.assert_array_equal(np.array([r["resampled"] for r in rows]), g["resampled"])
    if _same_machine():
        np.testing.assert_array_equal(np.array([r["x_est"] for r in rows]), g["x_est"])
        np.testing.assert_array_equal(np.array([r["max_idx"] for r in rows]), g["max_idx"])
        np.testing.assert_array_equal(np.array([r["max_val"] for r in rows]), g["max_val"])
        np.testing.assert_array_equal(np.array([r["z"] for r in rows]), g["z"])
        np.testing.assert_array_equal(np.array([r["x_true"] for r in rows]), g["x_true"])
        np.testing.assert_array_equal(np.array([r["ess"] for r in rows]), g["ess"])
        for j, k in enumerate(g["idx_steps"]):
            np.testing.assert_array_equal(rows[k]["idx"], g["idx_keep"][j])
    else:
        np.testing.assert_allclose(np.array([r["x_est"] for r in rows]), g["x_est"], rtol=1e-6)
    assert ks[0] == 0


def test_ekf_end_to_end():
    g = golden("ekf")
    rows = eo.run_reference_order(int(g["seed"]), len(g["P"]))
    for key in ["x_true", "x_dr", "z", "x_hat_m", "P", "x_hat"]:
        _eq(np.array([r[key] for r in rows]), g[key])


# ------------------------------------------------------------ graph SLAM
def test_graph_demo_every_iteration_bit_exact():
    import graph_oracle as go
    g = golden("graph")
    n = int(g["demo_n"])
    assert n == 51
    for i in range(n):
        pairs = g[f"demo{i}_pairs"]
        poses = g[f"demo{i}_poses_before"]
        edges = go.edges_from_pairs(pairs)
        blocks = go.linearize(edges, poses)
        _eq(blocks, g[f"demo{i}_edges"])
        times, H, b = go.assemble(edges, blocks)
        _eq(np.array(times), g[f"demo{i}_times"])
        _eq(H, g[f"demo{i}_H"])
        _eq(b[:, 0], g[f"demo{i}_b"])
        stats, after, _, _, _ = go.update_est_pose(edges, poses)
        _eq(stats, g[f"demo{i}_stats"])
        _eq(after, g[f"demo{i}_poses_after"])


def test_graph_t300_pairing_and_gauss_newton_bit_exact():
    import graph_oracle as go
    g = golden("graph")
    pairs = go.pairs_from_halves(g["big_halves"], 9)
    edges = go.edges_from_pairs(pairs)
    n = int(g["big_n"])
    poses = g["big0_poses_before"]
    for i in range(n):
        assert len(edges) == int(g[f"big{i}_n_edges"])
        _eq(poses, g[f"big{i}_poses_before"])
        blocks = go.linearize(edges, poses)
        _eq(blocks[:64], g[f"big{i}_edges_head"])
        _eq(blocks.sum(axis=0), g[f"big{i}_edges_colsum"])
        stats, poses, H, b, times = go.update_est_pose(edges, poses)
        _eq(np.array(times), g[f"big{i}_times"])
        _eq(b, g[f"big{i}_b"])
        _eq(H.sum(axis=0), g[f"big{i}_H_colsum"])
        _eq(H[::7, ::11], g[f"big{i}_H_sample"])
        _eq(stats, g[f"big{i}_stats"])
        _eq(poses, g[f"big{i}_poses_after"])


def test_scan_sensor_fixture():
    """ScanSensor.scan (graph_based_slam.py:128-172) restated: the reference's
    detections, noise-free and noisy observations, bit-exact, from the same
    seeded global stream (tests/golden/make_golden.py gen_scan)."""
    import graph_oracle as go
    g = golden("scan")
    np.random.seed(int(g["seed"]) + 1)
    ids, clean, noisy = [], [], []
    for p in g["poses"]:
        a, b, c = go.scan_sensor(p, g["lm"], 15.0, np.deg2rad(80.0), 0.05, np.deg2rad(2.0),
                                 np.deg2rad(2.0))
        ids.append(a)
        clean.append(b)
        noisy.append(c)
    np.testing.assert_array_equal(np.concatenate(ids), g["ids"])
    np.testing.assert_array_equal(np.concatenate(clean), g["clean"])
    np.testing.assert_array_equal(np.concatenate(noisy), g["noisy"])
