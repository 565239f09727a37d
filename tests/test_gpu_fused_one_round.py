"""The one-round fused kernel (pf_fused4.inl: four particles per lane, 1,024
per block) against the two-particle kernel it replaces (pf_fused_kernel),
through the C-ABI (slam_pf_set_fused_one_round).  Both evaluate each particle
pair with the same arithmetic (particle_filter.py:156-198, motion_model.py:31-62)
and sum the block partials in the same order, so every step record (x_est,
max_idx, max_val, weight_sum, ess, cov) and the final particles and weights
must be BIT-identical -- including resample steps (the run-mark gather,
particle_filter.py:216-221), partial last blocks and odd tile counts.  The
parity of the kernel against the oracle itself is test_gpu_c2.py /
test_gpu_pf.py (which now run the one-round kernel)."""
import numpy as np
import pytest

import pf_oracle as po

pytestmark = pytest.mark.gpu

FIELDS = ("max_idx", "max_val", "weight_sum", "ess", "resampled", "resample_next", "status",
          "n_special")


def _world(n, nl, steps, seed, motion):
    rs = np.random.RandomState(seed)
    lm = rs.uniform(-10, 10, (nl, 2))
    p = po.PFParams(n_particles=n, landmarks=lm, motion=motion)
    world = po.PFWorld(p)
    np.random.seed(seed + 100)
    zs = []
    for _ in range(steps):
        world.advance()
        zs.append(world.observe())
    return p, lm, np.array(zs)


def _same(ra, rb):
    for k, (a, b) in enumerate(zip(ra, rb)):
        for f in FIELDS:
            assert a[f] == b[f], (k, f, a[f], b[f])
        np.testing.assert_array_equal(a["x_est"], b["x_est"], err_msg=f"step {k}")
        np.testing.assert_array_equal(a["cov"], b["cov"], err_msg=f"step {k}")


@pytest.mark.parametrize("n,nl,lik", [(1 << 20, 100, "logsum"), (1 << 20, 100, "product"),
                                       (300_001, 100, "logsum"), (4_600, 20, "logsum"),
                                       (4_600, 20, "product")])
def test_one_round_matches_pair_kernel_device_rng(n, nl, lik):
    """Device-resident batches (graph replays, device Philox noise, velocity
    model): identical records and state."""
    from slamhip.pf import DeviceParticleFilter
    steps = 24
    p, lm, zs = _world(n, nl, steps, 3, "velocity")
    ctl = np.tile([p.vel, p.omega], (steps, 1))
    outs, states = [], []
    for one in (True, False):
        with DeviceParticleFilter(n, lm, motion="velocity", likelihood=lik, seed=9) as d:
            d.set_fused_one_round(one)
            d.load_observations(zs)
            outs.append(list(d.run(0, ctl)))
            states.append(d.get_state())
    assert sum(o["resampled"] for o in outs[0]) >= 2
    _same(*outs)
    for a, b in zip(*states):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("motion", ["linear", "velocity"])
def test_one_round_matches_pair_kernel_host_noise(motion):
    """Synchronous steps with host-injected noise (the parity path of the
    drop-in), 12,345 particles (a partial last block), resample offsets from
    the host."""
    from slamhip.pf import DeviceParticleFilter
    n, nl, steps = 12_345, 20, 16
    p, lm, zs = _world(n, nl, steps, 5, motion)
    rs = np.random.RandomState(7)
    noises = [rs.standard_normal((n, 3)) * (0.05 if motion == "linear" else 1.0)
              for _ in range(steps)]
    us = rs.random_sample(steps)
    outs, states = [], []
    for one in (True, False):
        with DeviceParticleFilter(n, lm, motion=motion) as d:
            d.set_fused_one_round(one)
            r = []
            for k in range(steps):
                u = us[k] if d.resample_next else float("nan")
                r.append(d.step((p.vel, p.omega), zs[k], noises[k], u))
            outs.append(r)
            states.append(d.get_state())
    assert sum(o["resampled"] for o in outs[0]) >= 1
    _same(*outs)
    for a, b in zip(*states):
        np.testing.assert_array_equal(a, b)
