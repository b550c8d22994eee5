"""bench.py's overlap choice for multi-rank sym runs (CPU, fake engine): the gated launch is
kept only when it gives the ungated schedule's bits on every rank and is no slower in the
alternating race."""
from __future__ import annotations

import importlib.util
import os
import time
from types import SimpleNamespace

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


class FakeEngine:
    """Steps cost `ms[overlap]` of wall time; state depends on the overlap only if `differ`."""

    def __init__(self, ms, differ=False):
        self.ms, self.differ, self.ov, self.k = ms, differ, 0, 0
        self.layout = SimpleNamespace(real_local=slice(0, 4))

    def set_overlap(self, ov):
        self.ov = ov

    def init_ics(self, *_):
        self.k = 0

    def step(self, n):
        time.sleep(self.ms[self.ov] * 1e-3 * n)
        self.k += n

    def sync(self):
        pass

    def state(self):
        v = np.full((4, 3), float(self.k) + (0.5 * self.ov if self.differ else 0.0))
        return SimpleNamespace(pos=v, vel=v)


class OneRank:
    @staticmethod
    def allreduce_sum(dist, x):
        return x

    @staticmethod
    def allreduce_max(dist, x):
        return x

    @staticmethod
    def barrier(dist):
        pass


def test_gated_kept_when_equal_and_faster():
    b = _bench()
    cfg = SimpleNamespace(n=1 << 16, seed=1)
    mode, verdict = b.overlap_self_check(FakeEngine({0: 6.0, 3: 2.0}), cfg, None, OneRank)
    assert mode == 3 and "bitwise" in verdict and "overlap 3" in verdict


def test_ungated_kept_when_faster():
    b = _bench()
    cfg = SimpleNamespace(n=1 << 16, seed=1)
    mode, verdict = b.overlap_self_check(FakeEngine({0: 2.0, 3: 6.0}), cfg, None, OneRank)
    assert mode == 0 and verdict.endswith("overlap 0")


def test_ungated_kept_when_bits_differ():
    b = _bench()
    cfg = SimpleNamespace(n=1 << 16, seed=1)
    mode, verdict = b.overlap_self_check(FakeEngine({0: 6.0, 3: 2.0}, differ=True), cfg, None,
                                         OneRank)
    assert mode == 0 and "differed" in verdict
