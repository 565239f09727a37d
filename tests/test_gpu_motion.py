"""MotionModel (motion_model.py:14-86) on the GPU against the reference's own
outputs (tests/golden/motion.npz: three noise settings, 300 poses each, noisy
from a seeded global RNG and noise-free).

  * the drop-in ``motion_model.MotionModel``: one (3, 1) call per pose, the
    NumPy stream drawn by the drop-in in the reference's order, and the same
    300 calls as one (3, 300) batch;
  * the particle filter's fused predict (velocity model) on the same poses and
    normals.
Tolerance: 1e-12 (relative and absolute) -- sin/cos within an ulp of NumPy's.
"""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

CASES = [0, 1, 2]


@pytest.mark.parametrize("c", CASES)
def test_dropin_motion_model_per_call(c):
    from motion_model import MotionModel
    g = golden("motion")
    dt, a1, a2, a3, a4, a5, a6, v, w = g[f"case{c}"]
    m = MotionModel(dt, a1, a2, a3, a4, a5, a6)
    np.random.seed(int(g[f"seed{c}"]))
    noisy = np.stack([m.moveWithNoise(p.reshape(3, 1), v, w)[:, 0] for p in g["poses"]])
    clean = np.stack([m.moveWithoutNoise(p.reshape(3, 1), v, w)[:, 0] for p in g["poses"]])
    np.testing.assert_allclose(noisy, g[f"noisy{c}"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(clean, g[f"clean{c}"], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("c", CASES)
def test_dropin_motion_model_batch(c):
    from motion_model import MotionModel
    g = golden("motion")
    dt, a1, a2, a3, a4, a5, a6, v, w = g[f"case{c}"]
    m = MotionModel(dt, a1, a2, a3, a4, a5, a6)
    np.random.seed(int(g[f"seed{c}"]))
    noisy = m.moveWithNoise(g["poses"].T, v, w)
    out = m.moveWithoutNoise(g["poses"].T, v, w)
    assert noisy.shape == (3, 300) and out.shape == (3, 300)
    np.testing.assert_allclose(noisy.T, g[f"noisy{c}"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(out.T, g[f"clean{c}"], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("c", CASES)
def test_pf_velocity_predict_all_cases(c):
    from slamhip.pf import DeviceParticleFilter
    g = golden("motion")
    poses = g["poses"]
    n = poses.shape[0]
    dt, a1, a2, a3, a4, a5, a6, v, w = g[f"case{c}"]
    np.random.seed(int(g[f"seed{c}"]))
    gn = np.random.standard_normal(3 * n).reshape(n, 3)
    with DeviceParticleFilter(n, np.zeros((1, 2)), dt=dt, motion="velocity",
                              alphas=(a1, a2, a3, a4, a5, a6)) as d:
        d.set_state(poses[:, 0], poses[:, 1], poses[:, 2])
        d.predict((v, w), gn)
        x, y, th, _ = d.get_state()
    np.testing.assert_allclose(np.stack([x, y, th], axis=1), g[f"noisy{c}"], rtol=1e-12, atol=1e-12)
