"""bench.compare_to_single (host logic of the sharded run's parity check, no
GPU): identical records and state pass; a one-ulp particle difference, a
different argmax or resample decision, or a covariance beyond 1e-7 fail and are
named in first_mismatch."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _recs(k, rs):
    out = []
    for j in range(k):
        c = rs.normal(size=(3, 3))
        out.append({"resampled": bool(j % 3 == 1), "resample_next": bool(j % 3 == 0),
                    "max_idx": 10 * j + 1, "max_val": 0.5 / (j + 1), "weight_sum": 1e-30 * (j + 2),
                    "x_est": rs.normal(size=3), "cov": c @ c.T})
    return out


def test_compare_to_single():
    import bench
    rs = np.random.RandomState(0)
    ref = _recs(8, rs)
    state = tuple(rs.normal(size=1000) for _ in range(4))
    copy = lambda recs: [{k: (np.array(v) if isinstance(v, np.ndarray) else v) for k, v in r.items()}
                         for r in recs]
    ok, worst, first = bench.compare_to_single(copy(ref), state, ref, state)
    assert ok and worst == 0.0 and first is None
    s2 = tuple(a.copy() for a in state)
    s2[2][17] = np.nextafter(s2[2][17], np.inf)
    ok, _, first = bench.compare_to_single(copy(ref), s2, ref, state)
    assert not ok and first.startswith("final th[17]")
    r2 = copy(ref)
    r2[5]["max_idx"] += 1
    ok, _, first = bench.compare_to_single(r2, state, ref, state)
    assert not ok and first.startswith("step 5: max_idx")
    r3 = copy(ref)
    r3[3]["cov"] = r3[3]["cov"] * (1 + 1e-9)                  # within the covariance bar
    ok, worst, first = bench.compare_to_single(r3, state, ref, state)
    assert ok and 0 < worst <= 1e-8
    r3[3]["cov"] = ref[3]["cov"] * (1 + 1e-6)
    ok, worst, first = bench.compare_to_single(r3, state, ref, state)
    assert not ok and first.startswith("cov relative difference")
