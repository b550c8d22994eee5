"""Newton-3 symmetric schedule (mode=sym, csrc/hip/nbody_sym.hip) on the GPU.

Reference: cuda.cu:53-60 evaluates each pair once (j > i) and scatters +F/-F into both
bodies (cuda.cu:43-49) with a data race; pyspark.py:80-84 does the same
pair reduction on the driver. The sym schedule keeps the pair-once saving race-free; these
tests pin its accuracy against the fp64 oracle, its determinism, graph replay, and bitwise
independence of the rank count (virtual ranks, P | 8).
"""
import numpy as np
import pytest

from gravsim.config import SimConfig
from gravsim.models import initial_conditions as ic
from gravsim.ops import oracle

from test_gpu_kernels import assert_close_sum, quantized_ref

pytestmark = pytest.mark.gpu


def _engine(n, **kw):
    from gravsim.runtime.engines import HipEngine

    return HipEngine(SimConfig(n=n, dtype="fp32", device="gpu", mode="sym", **kw))


@pytest.mark.parametrize("n", [3, 1000, 2049, 16384, 20000])
def test_sym_step_path_accel_matches_oracle(hip, n):
    b = ic.solar_random(n, seed=11 + n)
    ref, _, absref = quantized_ref(b.pos, b.mass, "fp32")
    e = _engine(n)
    try:
        assert e.native_layout["mode"] == 3
        e.load(b)
        got = e.accel(step_path=True)[:n, :3]
    finally:
        e.close()
    assert_close_sum(got, ref, absref, "fp32")


def test_sym_newton3_momentum(hip):
    """Pairs are evaluated once with exactly opposite terms: sum m_i a_i ~ 0 to rounding."""
    b = ic.random_cube(30000, seed=4)
    e = _engine(b.n)
    try:
        e.load(b)
        a = e.accel(step_path=True)[: b.n, :3]
    finally:
        e.close()
    f = (b.mass[:, None] * a).sum(0)
    scale = (b.mass[:, None] * np.abs(a)).sum(0)
    assert np.all(np.abs(f) <= 1e-5 * scale)


def test_sym_steps_match_oracle(hip):
    b = ic.solar_random(700, seed=5)
    e = _engine(b.n, dt=3600.0)
    e.load(b)
    e.step(20)
    got = e.state()
    e.close()
    x, v, _ = oracle.simulate(b.pos, b.vel, b.mass, 3600.0, 20)
    assert np.abs(got.pos - x).max() / np.abs(x).max() < 1e-5
    assert np.abs(got.vel - v).max() / np.abs(v).max() < 1e-4


def test_sym_close_to_split(hip):
    """Same step through the one-sided split schedule: equal to fp32 rounding."""
    b = ic.solar_random(40000, seed=8)
    outs = {}
    for mode in ("sym", "split"):
        from gravsim.runtime.engines import HipEngine

        e = HipEngine(SimConfig(n=b.n, dtype="fp32", device="gpu", mode=mode))
        e.load(b)
        e.step(3)
        outs[mode] = e.state().pos
        e.close()
    rel = np.abs(outs["sym"] - outs["split"]).max() / np.abs(outs["split"]).max()
    assert rel < 1e-6


def test_sym_determinism_and_graph(hip):
    res = []
    for graph in (True, True, False):
        e = _engine(50000, graph=graph)
        e.init_ics("solar+random", 21)
        e.step(5)
        res.append(e.state().pos)
        e.close()
    assert np.array_equal(res[0], res[1])
    assert np.array_equal(res[0], res[2])


@pytest.mark.parametrize("P", [2, 4, 8])
def test_sym_virtual_ranks_bitwise(hip, P):
    """P shards (all-gather + group-sum exchange by device copies) == 1 rank, bitwise."""
    from gravsim.runtime.engines import VirtualGroup

    cfg = SimConfig(n=40000, dtype="fp32", device="gpu", mode="sym")
    g = VirtualGroup(cfg, P)
    g.init_ics("solar+random", 9)
    g.step(4)
    got = g.state()
    g.close()
    one = VirtualGroup(cfg, 1)
    one.init_ics("solar+random", 9)
    one.step(4)
    ref = one.state()
    one.close()
    assert np.array_equal(got.pos, ref.pos)
    assert np.array_equal(got.vel, ref.vel)


def test_sym_exact_cutoff_falls_back(hip):
    """A sym layout whose cutoff resolves to the exact select runs the split schedule."""
    from gravsim.runtime.engines import HipEngine

    b = ic.solar_random(2000, seed=1)
    outs = []
    for mode in ("sym", "split"):
        e = HipEngine(SimConfig(n=b.n, dtype="fp32", device="gpu", mode=mode, cutoff=1e3))
        e.load(b)
        assert e.force_mode()["exact"]
        e.step(2)
        outs.append(e.state().pos)
        e.close()
    assert np.array_equal(outs[0], outs[1])
