"""The reference's gate on the PCG path (graph_based_slam.py:494-498).

Two modes: cond="estimate" (the LOBPCG estimate of cond alone, det not
formed) and cond="margin" (the default, formerly "certify": the estimate with an early decision
at a factor-100 margin, plus a log-det interval; test_gpu_graph_gate.py).

updateEstPose forms det(H) and cond(H) = numpy's 2-norm condition number and
solves only if 0.1 < det and cond < 1e15.  At config-5 size the dense route is
out of reach; the PCG path estimates cond = lambda_max / lambda_min by LOBPCG on
the block-sparse H on a second stream beside the solve (graph_kernels.inl,
DESIGN 8).  Checked here:
  * T = 300 / 600 (the dense path's regime, solver forced to PCG): the estimate
    within 1 % of numpy's cond of the same H (the dense H exported from the
    device), and within 1 % of the dense path's own Lanczos cond;
  * the gate's decision on a singular H (two components, one not anchored):
    PCG path and dense path both reject, poses unchanged, as the reference
    (numpy's det ~ 0, cond ~ 1e16+);
  * C5 (50,000 poses): lambda_min / lambda_max within 1e-3 of SciPy's LOBPCG /
    ARPACK on the exported BSR H, and the second Gauss-Newton update of the
    edge set warm-started from the first (fewer iterations).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _graph(T, seed=0):
    from slamhip.graph import circle_graph
    return circle_graph(T, n_landmarks=64, seed=seed, odom_noise=0.002)


@pytest.mark.parametrize("T", [300, 600])
def test_cond_estimate_matches_numpy(T):
    from slamhip.graph import DeviceGraph
    init, _, edges = _graph(T)
    dev = DeviceGraph(solver="pcg", pcg_tol=1e-10, cond="estimate")
    den = DeviceGraph(solver="dense")
    try:
        for g in (dev, den):
            g.set_poses(init)
            g.set_edges(edges)
        for it in range(3):
            ok, dsum, det, cond = dev.update()
            ok_d, dsum_d, det_d, cond_d = den.update()
            _, H, _, _ = dev.get_system(dense=True)
            ref = np.linalg.cond(H)                                     # :495
            info = dev.cond_info()
            assert ok and ok_d and np.isnan(det), (ok, ok_d, det, info)
            assert info["status"] == 1, info
            assert abs(cond / ref - 1) < 1e-2, (it, cond, ref, info)
            assert abs(cond / cond_d - 1) < 1e-2, (it, cond, cond_d)
            np.testing.assert_allclose(dsum, dsum_d, rtol=1e-6)
            np.testing.assert_allclose(dev.get_poses(), den.get_poses(), rtol=0, atol=1e-8)
    finally:
        dev.close()
        den.close()


def test_gate_rejects_singular_h_on_both_paths():
    """Edges only inside [0, 150) and [150, 300): the second component has no
    anchor, H is singular (numpy: det ~ 0, cond >= 1e15), the reference prints
    "can Not calculate trajectory!" and leaves the poses (:496, :510)."""
    from slamhip.graph import DeviceGraph
    init, _, edges = _graph(300)
    keep = (edges["time_bfr"] < 150) == (edges["time_aft"] < 150)
    edges = edges[keep]
    assert (edges["time_bfr"] >= 150).any() and (edges["time_aft"] < 150).any()
    for solver in ("pcg", "dense"):
        g = DeviceGraph(solver=solver, pcg_max_iter=4000)
        try:
            g.set_poses(init)
            g.set_edges(edges)
            ok, dsum, det, cond = g.update()
            assert not ok and dsum == 0.0, (solver, ok, dsum, det, cond)
            assert not (cond < 1e15), (solver, cond)
            np.testing.assert_array_equal(g.get_poses(), init)
            if solver == "pcg":
                info = g.cond_info()
                assert info["status"] in (2, 4), info
                st = g.optimize()                     # the GN loop ends, no error
                assert len(st) == 1 and st[0, 0] == 0.0
        finally:
            g.close()


def test_gate_singular_h_numpy_reference():
    """The same singular H through numpy (the reference's own calls) rejects."""
    from slamhip.graph import DeviceGraph
    init, _, edges = _graph(300)
    keep = (edges["time_bfr"] < 150) == (edges["time_aft"] < 150)
    g = DeviceGraph(solver="dense")
    try:
        g.set_poses(init)
        g.set_edges(edges[keep])
        g.update()
        _, H, _, _ = g.get_system(dense=True)
    finally:
        g.close()
    det, cond = np.linalg.det(H), np.linalg.cond(H)
    assert not ((0.1 < det) and (cond < 1e15)), (det, cond)


def test_c5_cond_estimate_matches_scipy():
    import scipy.sparse as sp
    import scipy.sparse.linalg as sla
    from slamhip.graph import DeviceGraph
    init, _, edges = _graph(50000)
    dev = DeviceGraph(solver="pcg", pcg_tol=1e-10, cond="estimate")
    try:
        dev.set_poses(init)
        dev.set_edges(edges)
        infos = []
        for _ in range(2):
            ok, dsum, det, cond = dev.update()
            info = dev.cond_info()
            infos.append(info)
            assert ok and np.isfinite(cond) and 1.0 < cond < 1e15, (ok, cond, info)
            assert info["status"] == 1, info
        rows, cols, vals = dev.get_bsr()
        nt = int(rows.max()) + 1
        H = sp.bsr_matrix((vals, cols, np.searchsorted(rows, np.arange(nt + 1))),
                          shape=(3 * nt, 3 * nt)).tocsr()
    finally:
        dev.close()
    H = 0.5 * (H + H.T)
    lmax = sla.eigsh(H, k=1, which="LA", return_eigenvectors=False, tol=1e-10)[0]
    # lambda_min by SciPy's LOBPCG with the same block-Jacobi preconditioner
    n = H.shape[0]
    D = np.zeros((nt, 3, 3))
    Hc = H.tocoo()
    m = (Hc.row // 3) == (Hc.col // 3)
    np.add.at(D, (Hc.row[m] // 3, Hc.row[m] % 3, Hc.col[m] % 3), Hc.data[m])
    Minv = np.linalg.inv(D)
    M = sla.LinearOperator((n, n), dtype=float,
                           matvec=lambda r: np.einsum("kij,kj->ki", Minv, r.reshape(nt, 3)).ravel())
    X = np.random.RandomState(1).standard_normal((n, 4))
    lmin = sla.lobpcg(H, X, M=M, largest=False, tol=1e-12, maxiter=400)[0].min()
    last = infos[-1]
    assert abs(last["lambda_max"] / lmax - 1) < 1e-3, (last, lmax)
    assert abs(last["lambda_min"] / lmin - 1) < 1e-3, (last, lmin)
    # the second update of the edge set starts from the first one's vectors
    assert infos[1]["iterations"] < infos[0]["iterations"], infos


@pytest.mark.parametrize("solver", ["pcg", "dense"])
def test_gate_anchor_removed_matches_numpy_cond(solver):
    """the anchor (:475) removed leaves H with the gauge null space
    (singular up to rounding), where lambda_min converges slowest.  is_calc of
    both paths equals the reference's decision from numpy's exact det / cond
    of the same H (:494-496)."""
    from slamhip.graph import DeviceGraph
    init, _, edges = _graph(300)
    g = DeviceGraph(solver=solver, anchor=0.0, pcg_max_iter=4000)
    try:
        g.set_poses(init)
        g.set_edges(edges)
        ok, dsum, det, cond = g.update()
        _, H, _, _ = g.get_system(dense=True)
        info = g.cond_info() if solver == "pcg" else None
    finally:
        g.close()
    ref = bool((0.1 < np.linalg.det(H)) and (np.linalg.cond(H) < 1e15))
    assert bool(ok) == ref, (solver, ok, ref, det, cond, np.linalg.cond(H), info)
    assert not ref


def test_gate_rejects_unconverged_estimate():
    """An estimate stopped at cond_max_iter (status 3) only bounds cond from
    below, so it cannot pass the gate: is_calc 0 and the poses unchanged, on
    the well-conditioned T = 300 graph whose converged estimate passes."""
    from slamhip.graph import DeviceGraph
    init, _, edges = _graph(300)
    g = DeviceGraph(solver="pcg", cond_max_iter=20, cond="estimate")
    try:
        g.set_poses(init)
        g.set_edges(edges)
        ok, dsum, det, cond = g.update()
        info = g.cond_info()
        assert info["status"] == 3, info
        assert not ok and dsum == 0.0, (ok, dsum, cond, info)
        np.testing.assert_array_equal(g.get_poses(), init)
    finally:
        g.close()
