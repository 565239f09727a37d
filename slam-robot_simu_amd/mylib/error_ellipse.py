"""Error-ellipse parameters with the semantics of the reference's
mylib/error_ellipse.py:15-68 (reporting helper).

Host-side NumPy, like the reference module; nothing here is on the estimator's
device path.  The drop-ins' callers (animation front-ends, user code) draw the
pose / landmark covariances returned by ``step()`` with it.

Differences from the reference, none of which changes a result:
  * no matplotlib / scipy import: the chi-squared table lookup restates
    ``scipy.interpolate.interp1d(p, square_x)`` (linear kind, sorted knots,
    ``searchsorted`` left bracket clipped to [1, n-1], slope * (x - x_lo) + y_lo,
    ValueError outside the table) so the interpolated value is the same double;
  * ``calc_error_ellipse_batch`` runs the same computation over an (N, 2, 2)
    stack (``np.linalg.eigh`` loops the same LAPACK routine per matrix).

The reference takes the eigenvector as ``vec[idxmax]`` -- a ROW of the
eigenvector matrix, not the column eigh returns (error_ellipse.py:51).  That
quirk is kept by default so the angles match the reference's plots;
``column_vectors=True`` gives the mathematically usual major-axis angle.
"""
import numpy as np

# upper cumulative percentage points [%] (2 degrees of freedom) and their
# chi-squared values: the table of error_ellipse.py:24-33
_P = np.array([99.9, 99.5, 99, 98.5, 98, 97.5, 97, 96, 95, 94, 93, 92, 91, 90, 85, 80, 75, 70,
               65, 60, 55, 50, 45, 40, 35, 30, 25, 20, 15, 10, 9, 8, 7, 6, 5, 4, 3, 2.5, 2, 1.5,
               1, 0.5, 0], dtype=np.float64)
_CHI2 = np.array([13.81551056, 10.59663473, 9.210340372, 8.399410156, 7.824046011, 7.377758908,
                  7.013115795, 6.43775165, 5.991464547, 5.626821434, 5.318520074, 5.051457289,
                  4.815891217, 4.605170186, 3.79423997, 3.218875825, 2.772588722, 2.407945609,
                  2.099644249, 1.832581464, 1.597015392, 1.386294361, 1.195674002, 1.021651248,
                  0.861565832, 0.713349888, 0.575364145, 0.446287103, 0.325037859, 0.210721031,
                  0.188621359, 0.166763218, 0.145141386, 0.123750807, 0.102586589, 0.081643989,
                  0.060918415, 0.050635616, 0.040405415, 0.030227276, 0.020100672, 0.010025084,
                  0], dtype=np.float64)
_ORDER = np.argsort(_P, kind="mergesort")
_XS = _P[_ORDER]
_YS = _CHI2[_ORDER]


def chi_squared(p):
    """Linear interpolation of the chi-squared table at percentage point(s) p
    (error_ellipse.py:36-37).  Raises ValueError outside [0, 99.9] like
    interp1d's default bounds check."""
    x = np.asarray(p, dtype=np.float64)
    flat = np.atleast_1d(x).ravel()
    if np.any(flat < _XS[0]) or np.any(flat > _XS[-1]):
        raise ValueError("A value in x_new is outside the interpolation range.")
    hi = np.clip(np.searchsorted(_XS, flat, side="left"), 1, len(_XS) - 1)
    lo = hi - 1
    slope = (_YS[hi] - _YS[lo]) / (_XS[hi] - _XS[lo])
    y = slope * (flat - _XS[lo]) + _YS[lo]
    return y.reshape(x.shape) if x.ndim else np.float64(y[0])


class ErrorEllipse(object):
    """Same constructor and methods as the reference's ErrorEllipse
    (error_ellipse.py:15-68)."""

    def __init__(self, p, column_vectors=False):
        self.p = _P.copy()
        self.square_x = _CHI2.copy()
        self.chi_squared_distribution = chi_squared
        self.__chi = chi_squared(p)
        self._column = bool(column_vectors)

    def calc_error_ellipse(self, sigma):
        """(major axis length, minor axis length, angle [rad]) of the ellipse
        of the 2x2 covariance sigma (error_ellipse.py:39-55)."""
        val, vec = np.linalg.eigh(sigma)
        idxmax = np.argmax(val)
        idxmin = np.argmin(val)
        vecmax = vec[:, idxmax] if self._column else vec[idxmax]
        ang_rad = np.arctan2(vecmax[1], vecmax[0])
        l = np.sqrt(val[idxmax] * self.__chi) * 2
        y = np.sqrt(val[idxmin] * self.__chi) * 2
        return l, y, ang_rad

    def calc_error_ellipse_batch(self, sigmas):
        """calc_error_ellipse over an (N, 2, 2) stack: three (N,) arrays."""
        s = np.asarray(sigmas, dtype=np.float64)
        if s.ndim != 3 or s.shape[1:] != (2, 2):
            raise ValueError("sigmas must have shape (N, 2, 2)")
        val, vec = np.linalg.eigh(s)
        rows = np.arange(len(s))
        idxmax = np.argmax(val, axis=1)
        idxmin = np.argmin(val, axis=1)
        vecmax = vec[rows, :, idxmax] if self._column else vec[rows, idxmax, :]
        ang = np.arctan2(vecmax[:, 1], vecmax[:, 0])
        l = np.sqrt(val[rows, idxmax] * self.__chi) * 2
        y = np.sqrt(val[rows, idxmin] * self.__chi) * 2
        return l, y, ang

    def calc_chi(self, p, sigma):
        """Major axis length at percentage point p (error_ellipse.py:57-68)."""
        chi = chi_squared(p)
        val, vec = np.linalg.eigh(sigma)
        idxmax = np.argmax(val)
        return np.sqrt(val[idxmax] * chi) * 2
