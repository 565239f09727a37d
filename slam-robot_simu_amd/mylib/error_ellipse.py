"""Error-ellipse parameters with the semantics of the reference's
mylib/error_ellipse.py:15-68 (reporting helper).

Host-side NumPy, like the reference module, plus ``calc_error_ellipse_device``
for a batch of covariances on the GPU (csrc/ellipse_api.hip).  The drop-ins' callers (animation front-ends, user code) draw the
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

# (upper cumulative percentage point [%], chi-squared value) for 2 degrees of
# freedom, ascending: the table of error_ellipse.py:24-33 (its literal values,
# not -2 ln(1 - p/100), so the lookup returns the reference's doubles)
_TABLE = (
    (0.0, 0.0), (0.5, 0.010025084), (1.0, 0.020100672),
    (1.5, 0.030227276), (2.0, 0.040405415), (2.5, 0.050635616),
    (3.0, 0.060918415), (4.0, 0.081643989), (5.0, 0.102586589),
    (6.0, 0.123750807), (7.0, 0.145141386), (8.0, 0.166763218),
    (9.0, 0.188621359), (10.0, 0.210721031), (15.0, 0.325037859),
    (20.0, 0.446287103), (25.0, 0.575364145), (30.0, 0.713349888),
    (35.0, 0.861565832), (40.0, 1.021651248), (45.0, 1.195674002),
    (50.0, 1.386294361), (55.0, 1.597015392), (60.0, 1.832581464),
    (65.0, 2.099644249), (70.0, 2.407945609), (75.0, 2.772588722),
    (80.0, 3.218875825), (85.0, 3.79423997), (90.0, 4.605170186),
    (91.0, 4.815891217), (92.0, 5.051457289), (93.0, 5.318520074),
    (94.0, 5.626821434), (95.0, 5.991464547), (96.0, 6.43775165),
    (97.0, 7.013115795), (97.5, 7.377758908), (98.0, 7.824046011),
    (98.5, 8.399410156), (99.0, 9.210340372), (99.5, 10.59663473),
    (99.9, 13.81551056),
)
_XS = np.array([t[0] for t in _TABLE], dtype=np.float64)
_YS = np.array([t[1] for t in _TABLE], dtype=np.float64)


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
        self.p = _XS[::-1].copy()            # the reference's (descending) order
        self.square_x = _YS[::-1].copy()
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

    def calc_error_ellipse_device(self, sigmas, device=0):
        """calc_error_ellipse_batch on the GPU (csrc/ellipse_api.hip: dsyevd's
        2x2 path restated, LAPACK's eigen-decomposition doubles): three (N,)
        arrays."""
        import ctypes as C
        from slamhip import _lib
        from slamhip._lib import check
        s = np.ascontiguousarray(sigmas, dtype=np.float64)
        if s.ndim != 3 or s.shape[1:] != (2, 2):
            raise ValueError("sigmas must have shape (N, 2, 2)")
        out = np.empty((len(s), 3))
        dp = C.POINTER(C.c_double)
        check(_lib.load().slam_error_ellipse(len(s), s.ctypes.data_as(dp), float(self.__chi),
                                             int(self._column), out.ctypes.data_as(dp), int(device)),
              "slam_error_ellipse")
        return out[:, 0], out[:, 1], out[:, 2]

    def calc_chi(self, p, sigma):
        """Major axis length at percentage point p (error_ellipse.py:57-68)."""
        chi = chi_squared(p)
        val, vec = np.linalg.eigh(sigma)
        idxmax = np.argmax(val)
        return np.sqrt(val[idxmax] * chi) * 2
