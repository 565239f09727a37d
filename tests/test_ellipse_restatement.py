"""The 2x2 symmetric eigen-decomposition the error-ellipse kernel restates
(oracle/ellipse_oracle.py, mirroring csrc/ellipse_api.hip) against
np.linalg.eigh (LAPACK dsyevd), bit-exact: the fixture covariances of
mylib/error_ellipse.py (degenerate, diagonal, equal eigenvalues, zero) and
random SPD / indefinite matrices."""
import numpy as np

from conftest import golden
import ellipse_oracle as eo


def test_dsyevd_2x2_restatement_bit_exact():
    covs = list(golden("ellipse")["covs"])
    rs = np.random.RandomState(0)
    for _ in range(3000):
        A = rs.normal(size=(2, 2)) * rs.uniform(1e-3, 1e3)
        covs.append(A @ A.T)
        B = rs.normal(size=(2, 2))
        covs.append(B + B.T)
    covs += [np.diag([1.0, 1.0]), np.array([[1.0, 1e-300], [1e-300, 1.0]]),
             np.array([[2.0, 1e-17], [1e-17, 1.0]])]
    for A in covs:
        w, Z = np.linalg.eigh(A)
        w2, Z2 = eo.eig2(A)
        np.testing.assert_array_equal(w, w2)
        np.testing.assert_array_equal(Z, Z2)
