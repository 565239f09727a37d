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


def test_resample_indices_leaves_the_next_gather_alone():
    """slam_pf_resample_indices runs the exact cumsum's expand pass too, which
    writes run marks; they must not reach the next step's gather.  Round 6
    (test_gpu_zz_order's IndexError, and most likely round 3's C2 miss): the
    stand-alone scan read its offset from StepIO slot ctr[0], which the
    previous step end had advanced past the staged slot 0 -- out of bounds on a
    handle without loaded observations, a NaN (the device offset) here -- and
    its marks carried the current generation, so an earlier run start from a
    larger offset won the gather's running max.  Two handles take the same
    steps (offset 0 on resampling steps); one also asks for the indices first:
    every record and the final state must be identical."""
    import bench
    from slamhip import pf as dpf
    n = 1 << 16
    lm, zs, (vel, omega, dt) = bench.simulate_world(40)
    ctl = np.tile([vel, omega], (40, 1))
    rs = np.random.RandomState(7)
    hs = [dpf.DeviceParticleFilter(n, lm, dt=dt, motion="velocity", likelihood="logsum", seed=9)
          for _ in range(2)]
    try:
        for h in hs:
            h.load_observations(zs)                    # every offset slot NaN
            h.run(0, ctl[:2])
        resampled = 0
        for k in range(2, 16):
            g = rs.standard_normal((n, 3))
            recs = []
            for i, h in enumerate(hs):
                u = 0.0 if h.resample_next else float("nan")
                if i == 1 and h.resample_next:
                    h.resample_indices(u)
                recs.append(h.step(ctl[k], zs[k], g, u))
            a, b = recs
            resampled += int(a["resampled"])
            for f in ("resampled", "max_idx", "max_val", "weight_sum", "status"):
                assert a[f] == b[f], (k, f, a[f], b[f])
            np.testing.assert_array_equal(a["x_est"], b["x_est"], err_msg=f"step {k}")
        assert resampled >= 3, resampled
        sa, sb = hs[0].get_state(), hs[1].get_state()
        for u, v in zip(sa, sb):
            np.testing.assert_array_equal(u, v)
    finally:
        for h in hs:
            h.close()
