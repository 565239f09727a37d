import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-robot_simu_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """When GPU tests run, bring up PyTorch's HIP runtime before libslam_hip
    touches the device (the torch-based shard tests share the process)."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass
    yield


@pytest.fixture(scope="session")
def c2_trajectory():
    """The oracle's C2 trajectory (BASELINE configs[1]: 2^20 particles x 100
    landmarks, velocity model, 8 steps with resamples): per step the input
    state, the injected normals / observations / offset and the oracle's
    outputs.  Shared by tests/test_gpu_c2.py and tests/test_gpu_zz_order.py."""
    import pf_oracle as po
    n, nl, n_steps = 1 << 20, 100, 8
    rs = np.random.RandomState(1)
    lm = rs.uniform(-10, 10, (nl, 2))
    p = po.PFParams(n_particles=n, landmarks=lm, motion="velocity")
    orc, world = po.PFOracle(p), po.PFWorld(p)
    np.random.seed(2)
    steps = []
    for _ in range(n_steps):
        world.advance()
        state = (orc.x.copy(), orc.y.copy(), orc.th.copy(), orc.w.copy())
        u = np.random.rand() if orc.needs_resample() else None
        g = np.random.standard_normal(3 * n).reshape(n, 3)
        z = world.observe()
        out = orc.step(z, g, None if u is None else u * p.np_recip)
        steps.append(dict(state=state, u=u, g=g, z=z, out=out,
                          post=(orc.x.copy(), orc.y.copy(), orc.th.copy(), orc.w.copy()),
                          resample_next=orc.needs_resample()))
    assert sum(s["out"]["resampled"] for s in steps) >= 1
    return p, steps


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def heavy_weights(rs, n, zero_frac=0.0):
    """Same generator as tests/golden/make_golden.py (multiplications only)."""
    u = rs.random_sample(n)
    v = rs.random_sample(n)
    w = u * u
    w = w * w
    w = w * w
    w = w * w * v
    if zero_frac > 0:
        w[rs.random_sample(n) < zero_frac] = 0.0
    return w


def stage_weights(tag, n, wseed):
    w = heavy_weights(np.random.RandomState(int(wseed)), n,
                      zero_frac=0.5 if tag in ("r8193", "r1m") else 0.0)
    if tag in ("r8193", "r1m"):
        w[:64] = 0.0
    return w / np.sum(w.reshape(1, n))


def rle_decode(vals, counts):
    return np.repeat(vals.astype(np.int64), counts)


DBL_MIN = np.finfo(np.float64).tiny


def weights_match(w, ref, rtol=1e-12, floor=DBL_MIN):
    """SURVEY 8(a) A6 bar for likelihood weights: identical zero sets, <= rtol
    relative on weights >= floor, and within 2 units of 2^-1074 below it (the
    subnormal grid both sides round onto).  A multi-step trajectory passes a
    larger floor with the absolute bound rtol * floor below it: weights that
    went through the subnormal range in an earlier step carry that step's
    precision loss -- the reference's own arithmetic.  rtol may be per element
    (see subnormal_dip_rtol).  Returns the worst relative error seen."""
    w, ref = np.asarray(w), np.asarray(ref)
    zw, zr = w == 0, ref == 0
    assert np.array_equal(zw, zr), f"zero sets differ at {np.flatnonzero(zw != zr)[:8]}"
    nz = ~zr
    normal = nz & (np.abs(ref) >= floor)
    rt = np.broadcast_to(np.asarray(rtol, dtype=np.float64), ref.shape)
    rel = np.abs(w[normal] - ref[normal]) / np.abs(ref[normal])
    worst = float(rel.max()) if rel.size else 0.0
    if rel.size and np.any(rel > rt[normal]):
        i = int(np.argmax(rel / rt[normal]))
        raise AssertionError(f"max relative weight error {rel[i]:.3g} > {rt[normal][i]:.3g} "
                             f"(element {np.flatnonzero(normal)[i]})")
    sub = nz & ~normal
    if sub.any():
        atol = 2 * 2.0 ** -1074 if floor <= DBL_MIN else rt[sub] * floor
        # a per-element rtol above the bar (a subnormal dip) bounds these too
        atol = np.maximum(atol, rt[sub] * np.abs(ref[sub]))
        assert np.all(np.abs(w[sub] - ref[sub]) <= atol)
    return worst


def subnormal_dip_rtol(factors, rtol, w_prev=None):
    """Per-particle weight tolerance for a sequential product (particle_filter.py:
    192) whose partial products dip below DBL_MIN and climb back: from the dip
    on the product carries the subnormal grid's absolute quantum, so one ulp of
    difference in any factor there (exp within 1 ulp) moves the result by up to
    ~2^-1074 / (smallest partial product) relative -- the reference's own
    precision loss.  w_prev: the previous weights, whose product with the
    likelihood (particle_filter.py:194, before normalising) is one more partial
    product.  rtol elsewhere."""
    cp = np.cumprod(factors, axis=1)
    dip = cp.min(axis=1)
    if w_prev is not None:
        dip = np.minimum(dip, w_prev * cp[:, -1])
    del cp
    out = np.full(dip.shape, float(rtol))
    low = (dip > 0) & (dip < DBL_MIN)
    out[low] = np.maximum(rtol, 4 * 2.0 ** -1074 / dip[low])
    return out
