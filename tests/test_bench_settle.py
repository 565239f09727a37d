"""bench.settle / timed_runs step bookkeeping (host logic, no GPU): the settle
phase replays whole 31-step batches from step 0, and the warm-up, the timed run
and the timing pass follow it on consecutive step indices."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


class Rec:
    def __init__(self):
        self.calls = []

    def prepare_graphs(self):
        return 0.5

    def run(self, first, ctl, want_results=True):
        self.calls.append((first, len(ctl), want_results))
        return [{"resampled": 0}] * len(ctl) if want_results else None

    def enable_timing(self, on):
        pass

    def timing(self, k):
        return (0.0, 0)


def test_settle_whole_batches():
    r = Rec()
    ctl = np.zeros((100, 2))
    assert bench.settle(r.run, ctl, 65) == 62
    assert r.calls == [(0, 31, False), (31, 31, False)]
    assert bench.settle(Rec().run, ctl, 30) == 0


def test_timed_runs_step_indices_after_settle():
    r = Rec()
    settle, warm, steps = 62, 5, 20
    ctl = np.zeros((settle + warm + 2 * steps, 2))
    elapsed, out, timing, cap = bench.timed_runs(r, ctl, warm, steps, lambda: None,
                                                 settle_steps=settle)
    assert cap == 0.5 and len(out) == steps
    assert r.calls == [(0, 31, False), (31, 31, False), (62, 5, False), (67, 20, True), (87, 20, True)]
