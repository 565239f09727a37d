"""ErrorEllipse.calc_error_ellipse on the GPU (csrc/ellipse_api.hip) against
the reference's own outputs (tests/golden/ellipse.npz) and the host module at
batch size.  Axis lengths bit-exact (LAPACK's eigenvalues, NaN where the
reference's sqrt of a negative eigenvalue is NaN); angles within 2e-15 rad
(device atan2)."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _check(dev, ref):
    np.testing.assert_array_equal(dev[0], ref[:, 0])
    np.testing.assert_array_equal(dev[1], ref[:, 1])
    np.testing.assert_allclose(dev[2], ref[:, 2], rtol=0, atol=2e-15)


@pytest.mark.parametrize("p,key", [(99.0, "out99"), (95.0, "out95")])
def test_device_ellipse_matches_reference_fixture(p, key):
    from mylib.error_ellipse import ErrorEllipse
    g = golden("ellipse")
    with np.errstate(invalid="ignore"):
        _check(ErrorEllipse(p).calc_error_ellipse_device(g["covs"]), g[key])


def test_device_ellipse_batch_matches_host():
    from mylib.error_ellipse import ErrorEllipse
    rs = np.random.RandomState(4)
    A = rs.normal(size=(200000, 2, 2)) * rs.uniform(1e-3, 1e3, (200000, 1, 1))
    covs = A @ A.transpose(0, 2, 1)
    for col in (False, True):
        ee = ErrorEllipse(90.0, column_vectors=col)
        ref = np.column_stack(ee.calc_error_ellipse_batch(covs))
        _check(ee.calc_error_ellipse_device(covs), ref)
