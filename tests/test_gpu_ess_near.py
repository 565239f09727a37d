"""The resample decision at the ESS threshold (particle_filter.py:210-211).

The reference decides `1 / (pw @ pw.T) < ESS_TH` with its BLAS's summation
order; the device sums the same squares in a fixed order of its own, a few ulp
apart.  Every step result carries `ess_near` (the device's ESS within the band
of ESS_TH); the drop-in's per-step calls and `run(confirm_ess=True)` then
re-form the decision on the host with the reference's own expression.

The weights are placed exactly at the threshold: NP = 12,800 (ESS_TH = 128),
128 particles of weight 1/128 and the rest 0, every particle at the same pose
and no motion noise, so the likelihood is one common factor and the
normalised weights stay at 1/128 up to the rounding of np.sum -- the ESS lands
within a few ulp of ESS_TH, on either side.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, M = 12800, 128
# a wide observation noise keeps the common likelihood factor far from
# underflow (all-zero weights would become 1/NP, particle_filter.py:236)
R = np.diag([100.0, 100.0]) ** 2


def _placed(pf):
    w = np.zeros(N)
    w[np.random.RandomState(5).choice(N, M, replace=False)] = 1.0 / M
    pf.set_state(x=np.full(N, 10.0), y=np.zeros(N), th=np.full(N, np.pi / 2), w=w)
    return w


def _host_decision(pf):
    pw = pf.get_state()[3]
    return bool(1.0 / float(pw @ pw.T) < pf.cfg.ess_threshold), pw


@pytest.mark.parametrize("likelihood", ["product", "logsum"])
def test_step_flags_and_confirms_at_threshold(likelihood):
    from slamhip.pf import DeviceParticleFilter
    lm = np.random.RandomState(1).uniform(-10, 10, (20, 2))
    z = np.random.RandomState(2).normal(0, 1, (20, 2))
    with DeviceParticleFilter(N, lm, r=R, likelihood=likelihood) as pf:
        _placed(pf)
        assert pf.cfg.ess_threshold == 128.0
        out = pf.step((1.0, 0.1), z, noise=np.zeros((N, 3)))
        assert abs(out["ess"] / 128.0 - 1) < 1e-12, out["ess"]
        assert out["ess_near"], out["ess"]
        assert out["ess_confirmed"]
        host, pw = _host_decision(pf)
        assert out["resample_next"] == host
        assert out["ess_host"] == 1.0 / float(pw @ pw.T)
        # the device takes the host's decision into the next step
        out2 = pf.step((1.0, 0.1), z, noise=np.zeros((N, 3)))
        assert out2["resampled"] == host


def test_run_flags_and_confirmed_replay():
    """slam_pf_run (the device-resident batch): the flag in every result, and
    confirm_ess=True re-forms each flagged decision before the next step."""
    from slamhip.pf import DeviceParticleFilter
    lm = np.random.RandomState(1).uniform(-10, 10, (20, 2))
    zs = np.random.RandomState(3).normal(0, 1, (4, 20, 2))
    ctl = np.tile([1.0, 0.1], (4, 1))
    for confirm in (False, True):
        with DeviceParticleFilter(N, lm, r=R, motion="velocity", likelihood="logsum",
                                  alphas=(0.0,) * 6) as pf:
            _placed(pf)
            pf.load_observations(zs)
            res = pf.run(0, ctl[:1], confirm_ess=confirm)
            assert res[0]["ess_near"], res[0]["ess"]
            host, _ = _host_decision(pf)
            if confirm:
                assert res[0]["ess_confirmed"] and res[0]["resample_next"] == host
            else:
                assert "ess_confirmed" not in res[0]
            nxt = pf.run(1, ctl[1:2], confirm_ess=confirm)
            assert nxt[0]["resampled"] == res[0]["resample_next"]


def test_band_controls_the_flag():
    from slamhip.pf import DeviceParticleFilter
    lm = np.random.RandomState(1).uniform(-10, 10, (20, 2))
    zs = np.random.RandomState(3).normal(0, 1, (6, 20, 2))
    ctl = np.tile([1.0, 0.1], (6, 1))
    with DeviceParticleFilter(N, lm, r=R, motion="velocity", likelihood="logsum", seed=4) as pf:
        pf.load_observations(zs)
        pf.set_ess_band(1e6)                 # every step inside the band
        assert all(r["ess_near"] for r in pf.run(0, ctl[:3]))
        pf.set_ess_band(0.0)
        assert not any(r["ess_near"] for r in pf.run(3, ctl[3:]) if r["ess"] != 128.0)
