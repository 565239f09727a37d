"""RunResults (slamhip.pf): the records of a device-resident batch compare
element-wise with any sequence of record dicts, whichever path built them
(the C array of slam_pf_run, or the confirm_ess path's dicts) -- ADVICE r4.
Host logic only (no GPU)."""
import numpy as np


def _records(k):
    from slamhip._lib import PFResult
    res = (PFResult * k)()
    for i in range(k):
        res[i].max_idx = 10 * i
        res[i].max_val = 0.5 + i
        res[i].x_est[:] = [1.0 * i, 2.0, 3.0]
        res[i].cov[:] = [float(j) for j in range(9)]
        res[i].resampled = i % 2
    return res


def test_run_results_equality_and_slices():
    from slamhip.pf import RunResults
    a = RunResults(_records(3))
    b = RunResults(_records(3))
    assert a == b and not (a != b)
    assert a == list(b)                              # against plain dicts
    assert a == RunResults.from_dicts(list(b))       # the confirm_ess form
    c = _records(3)
    c[2].max_idx = 7
    assert a != RunResults(c)
    assert a != RunResults(_records(2))
    assert len(a[1:]) == 2 and a[1]["max_idx"] == 10
    assert a.records.shape == (3,)
    d = RunResults.from_dicts(list(b))
    assert len(d) == 3 and d[2]["resampled"] is False
    np.testing.assert_array_equal(d[1]["x_est"], [1.0, 2.0, 3.0])


def test_run_results_nan_fields_compare_equal():
    """A degenerate step's NaN covariance / ESS: two identical runs still
    compare equal, and a NaN against a number does not."""
    from slamhip.pf import RunResults
    a, b = _records(2), _records(2)
    for r in (a, b):
        r[1].cov[4] = float("nan")
        r[1].ess = float("nan")
    assert RunResults(a) == RunResults(b)
    b[1].ess = 1.0
    assert RunResults(a) != RunResults(b)
