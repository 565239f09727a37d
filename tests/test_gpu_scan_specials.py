"""The exact cumsum's approximate prefixes stay accurate enough that the
classification does its work (particle_filter.py:212).

The lean exact cumsum decides each element from an approximate prefix with a
relative margin; an element whose prefix misses the margin becomes a special
(folded sequentially), and a classification the fold cannot reconcile falls
back to a sequential pass (record status bit 1).  Either way the indices stay
exact -- the lockstep tests cannot see a prefix gone bad -- so this test reads
the records: a resample step must not fall back, and its specials stay a few
dozen.  Round 6 regression: an exclusive wave scan formed as `inclusive - own`
loses a small prefix ahead of a large element (unbounded relative error); in
the bench's device NumPy-stream run (velocity model, 2^20 x 100, RandomState
1234) one step fell back and took 108 ms.  Runs that workload's steps
(`bench.simulate_world`, the bench's settle + warm-up + timed steps).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _records(dpf, bench, mode):
    lm, zs, (vel, omega, dt) = bench.simulate_world(760)
    ctl = np.tile([vel, omega], (760, 1))
    pf = dpf.DeviceParticleFilter(bench.NP_PER_GPU, lm, dt=dt, motion="velocity",
                                  likelihood="logsum", seed=1234)
    try:
        if mode == "numpy":
            pf.use_numpy_stream(np.random.RandomState(1234))
            pf.load_truth(bench.simulate_world.poses)
        else:
            pf.load_observations(zs)
        out = []
        for s0 in range(0, 760, 40):
            out.extend(pf.run(s0, ctl[s0:s0 + 40]))
        return out
    finally:
        pf.close()


@pytest.mark.parametrize("mode", ["numpy", "philox"])
def test_resample_steps_classify_without_fallback(mode):
    import bench
    from slamhip import pf as dpf
    recs = _records(dpf, bench, mode)
    res = [r for r in recs if r["resampled"]]
    assert len(res) >= 20, len(res)
    fell_back = [i for i, r in enumerate(recs) if r["status"] & 2]
    assert not fell_back, f"exact-scan fallback at steps {fell_back[:10]}"
    worst = max(r["n_special"] for r in res)
    assert worst < 4096, worst
