"""Sharded particle filter on the GPU: several HIP shards of one filter in one
process (slamhip.shard.LocalComm, the same orchestration the multi-GPU run
uses with torch.distributed/RCCL) must reproduce the single-handle filter
over the same particles bit for bit: resampling decisions, argmax index,
estimate and every weight."""
import numpy as np
import pytest

import pf_oracle as po

pytestmark = pytest.mark.gpu


def _world(n_global, nl, steps, seed, motion="linear"):
    rs = np.random.RandomState(seed)
    lm = rs.uniform(-10, 10, (nl, 2))
    p = po.PFParams(n_particles=n_global, landmarks=lm, motion=motion)
    world = po.PFWorld(p)
    np.random.seed(seed + 1)
    zs = []
    for _ in range(steps):
        world.advance()
        zs.append(world.observe())
    return lm, zs, p


@pytest.mark.parametrize("world,n_local,nl,motion,host_noise", [
    (2, 16384, 20, "linear", True),
    (4, 65536, 100, "velocity", False),
    (3, 8192, 5, "linear", False),
])
def test_local_shards_match_single_handle(world, n_local, nl, motion, host_noise):
    from slamhip.pf import DeviceParticleFilter
    from slamhip.shard import DeviceShard, LocalComm, ShardedFilter
    n_global = world * n_local
    steps = 30
    lm, zs, p = _world(n_global, nl, steps, 21, motion)
    single = DeviceParticleFilter(n_global, lm, motion=motion, seed=5)
    shards = [DeviceShard(n_local, n_global, r * n_local, lm, motion=motion, seed=5)
              for r in range(world)]
    filt = ShardedFilter(shards, list(range(world)), LocalComm(world), n_global)
    rs = np.random.RandomState(77)
    n_res = 0
    try:
        for k in range(steps):
            assert single.resample_next == filt.resample_next
            u = rs.random_sample() if single.resample_next else float("nan")
            if not host_noise:
                u = float("nan")                    # device RNG offset on both sides
            noise = None
            if host_noise:
                noise = (np.random.multivariate_normal([0, 0, 0], p.q, n_global)
                         if motion == "linear" else rs.standard_normal((n_global, 3)))
            a = single.step((p.vel, p.omega), zs[k], noise, u)
            b = filt.step((p.vel, p.omega), zs[k], noise, u)
            n_res += a["resampled"]
            assert a["resampled"] == b["resampled"], k
            assert a["max_idx"] == b["max_idx"], (k, a["max_idx"], b["max_idx"])
            np.testing.assert_array_equal(a["x_est"], b["x_est"])
            assert a["max_val"] == b["max_val"]
            assert a["weight_sum"] == b["weight_sum"]
            np.testing.assert_allclose(a["cov"], b["cov"], rtol=1e-7, atol=1e-13)
            assert abs(a["ess"] - b["ess"]) <= 1e-9 * a["ess"]
        xs, ys, ts, ws = single.get_state()
        xg, yg, tg, wg = filt.get_state()
        np.testing.assert_array_equal(ws, wg)
        np.testing.assert_array_equal(xs, xg)
        np.testing.assert_array_equal(ts, tg)
        assert n_res >= 2
    finally:
        single.close()
        filt.close()
