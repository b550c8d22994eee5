"""GPU numerics of the gfx950 force/step kernels against the fp64 oracle.

Tile-edge sizes, both j-source variants (LDS-DMA tiles / SGPR scalar cache), both schedules
(fused / split), fp32 and fp64, random data. Determinism and schedule-independence are
bitwise; accuracy is relative to max |a| (fp32 ~1e-6, fp64 ~1e-13).
"""
import numpy as np
import pytest

from gravsim.config import SimConfig
from gravsim.models import initial_conditions as ic
from gravsim.models.initial_conditions import BodySet
from gravsim.ops import oracle
from gravsim.ops.force import cpu_accelerations

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 3, 63, 64, 65, 1000, 4097]


EPS = {"fp32": 2.0 ** -24, "fp64": 2.0 ** -53}


def quantized_ref(pos, mass, dtype, **kw):
    """Oracle on the inputs as the kernel sees them (positions and mu = G m rounded to dtype),
    so the check measures kernel arithmetic, not input quantisation."""
    from gravsim.config import G_SI

    T = np.float32 if dtype == "fp32" else np.float64
    p = np.asarray(pos).astype(T).astype(np.float64)
    mu = (G_SI * np.asarray(mass, dtype=np.float64)).astype(T).astype(np.float64)
    return oracle.accelerations(p, mu, G=1.0, with_potential=True, with_abs=True, **kw)


def assert_close_sum(got, ref, absref, dtype, c=128.0):
    """|got - ref| <= c * eps * sum_j |term_ij| (+ tiny): rounding of a sum of terms."""
    err = np.abs(got - ref)
    bound = c * EPS[dtype] * absref + 1e-300
    worst = (err / bound).max()
    assert worst <= 1.0, f"error {worst:.2f}x over the rounding bound"


def _engine(n, dtype="fp32", **kw):
    from gravsim.runtime.engines import HipEngine

    return HipEngine(SimConfig(n=n, dtype=dtype, device="gpu", **kw))


def _accel(bodies, dtype, **kw):
    eng = _engine(bodies.n, dtype, **kw)
    try:
        eng.load(bodies)
        return eng.accel()[: bodies.n]
    finally:
        eng.close()


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("kernel", ["lds", "smem"])
def test_accel_matches_oracle(hip, n, dtype, kernel):
    b = ic.solar_random(n, seed=7 + n)
    ref, phi, absref = quantized_ref(b.pos, b.mass, dtype)
    got = _accel(b, dtype, kernel=kernel)
    assert_close_sum(got[:, :3], ref, absref, dtype)
    if n > 1:  # phi is a sum of positive terms: sum |terms| = |phi|
        assert_close_sum(got[:, 3], phi, np.abs(phi), dtype)


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("kernel", ["lds", "smem"])
def test_step_path_accel_matches_oracle(hip, n, dtype, kernel):
    """The integrator's own force path (fp32: explicit 2-vector loop; fp64: direct r^-3
    refinement; fast cutoff core) on tile-edge sizes, against the fp64 oracle."""
    from gravsim.runtime.engines import HipEngine

    b = ic.solar_random(n, seed=3 + n)
    ref, _, absref = quantized_ref(b.pos, b.mass, dtype)
    e = HipEngine(SimConfig(n=n, dtype=dtype, device="gpu", kernel=kernel))
    try:
        e.load(b)
        got = e.accel(step_path=True)[:n, :3]
    finally:
        e.close()
    assert_close_sum(got, ref, absref, dtype)


@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
def test_variants_and_schedules_bitwise(hip, dtype):
    """LDS vs SMEM and fused vs split, every ipl: identical bits (canonical chunk order)."""
    b = ic.random_cube(5000, seed=3)
    outs = []
    for kernel in ("lds", "smem"):
        for mode in ("fused", "split"):
            for ipl in (1, 2, 4):
                eng = _engine(b.n, dtype, kernel=kernel, mode=mode, ipl=ipl)
                eng.load(b)
                eng.step(3)
                outs.append(eng.state().pos)
                eng.close()
    for o in outs[1:]:
        assert np.array_equal(o, outs[0])


def test_determinism_two_runs(hip):
    res = []
    for _ in range(2):
        eng = _engine(9000, "fp32")
        eng.init_ics("solar+random", 11)
        eng.step(5)
        res.append(eng.state().pos)
        eng.close()
    assert np.array_equal(res[0], res[1])


def test_device_ics_match_host(hip):
    for fam in ("solar+random", "random"):
        eng = _engine(3000, "fp64")
        eng.init_ics(fam, 1234)
        got = eng.state()
        eng.close()
        ref = ic.make(fam, 3000, 1234)
        assert np.array_equal(got.pos, ref.pos)
        assert np.array_equal(got.mass, ref.mass)
        assert np.array_equal(got.vel, ref.vel)


@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
def test_steps_match_oracle(hip, dtype):
    b = ic.solar_random(700, seed=5)
    eng = _engine(b.n, dtype, dt=3600.0)
    eng.load(b)
    eng.step(20)
    got = eng.state()
    eng.close()
    x, v, _ = oracle.simulate(b.pos, b.vel, b.mass, 3600.0, 20)
    tol = 1e-5 if dtype == "fp32" else 1e-12
    assert np.abs(got.pos - x).max() / np.abs(x).max() < tol
    assert np.abs(got.vel - v).max() / np.abs(v).max() < tol * 10


def test_graph_replay_equals_eager(hip):
    outs = []
    for graph in (True, False):
        eng = _engine(6000, "fp32", graph=graph)
        eng.init_ics("solar+random", 2)
        eng.step(7)
        outs.append(eng.state().pos)
        eng.close()
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("P", [2, 3, 4])
@pytest.mark.parametrize("mode", ["fused", "split"])
def test_virtual_ranks_bitwise(hip, P, mode):
    """P shards with the RCCL schedule (overlapped own-chunk partials) == 1 rank, bitwise."""
    from gravsim.runtime.engines import VirtualGroup

    n = 5000
    cfg = SimConfig(n=n, dtype="fp32", device="gpu", mode=mode, chunk=1024)
    g = VirtualGroup(cfg, P)
    g.init_ics("solar+random", 9)
    g.step(6)
    got = g.state()
    g.close()
    one = VirtualGroup(cfg, 1)
    one.init_ics("solar+random", 9)
    one.step(6)
    ref = one.state()
    one.close()
    assert np.array_equal(got.pos, ref.pos)
    assert np.array_equal(got.vel, ref.vel)


@pytest.mark.parametrize("P,dtype", [(2, "fp32"), (3, "fp64"), (5, "fp32")])
def test_virtual_ranks_ring_bitwise(hip, P, dtype):
    """Ring pass (P-1 neighbour transfers, each slice computed on arrival on alternating
    streams) over P virtual shards == the 1-rank all-gather run, bitwise."""
    from gravsim.runtime.engines import VirtualGroup

    cfg = SimConfig(n=5000, dtype=dtype, device="gpu", chunk=1024, strategy="ring")
    g = VirtualGroup(cfg, P)
    g.init_ics("solar+random", 9)
    g.step(5)
    got = g.state()
    g.close()
    one = VirtualGroup(cfg.replace(strategy="allgather"), 1)
    one.init_ics("solar+random", 9)
    one.step(5)
    ref = one.state()
    one.close()
    assert np.array_equal(got.pos, ref.pos)
    assert np.array_equal(got.vel, ref.vel)


def test_fp32_no_overflow_heavy_masses(hip):
    """D1: G*m_i*m_j overflows fp32 in the reference; mu = G*m per body does not."""
    rng = np.random.default_rng(0)
    n = 512
    pos = rng.uniform(-3e11, 3e11, (n, 3))
    mass = rng.uniform(1e24, 1e25, n)
    mass[0] = 1.989e30
    b = BodySet(pos, np.zeros((n, 3)), mass)
    got = _accel(b, "fp32")
    assert np.isfinite(got).all()
    ref, _, absref = quantized_ref(pos, mass, "fp32")
    assert_close_sum(got[:, :3], ref, absref, "fp32")


def test_gpu_matches_cpu_engine_fp64(hip):
    b = ic.solar_random(3000, seed=21)
    got = _accel(b, "fp64")
    a, phi = cpu_accelerations(b.pos, b.mass, dtype="fp64")
    assert np.abs(got[:, :3] - a).max() / np.abs(a).max() < 1e-13


def test_nonfinite_guard(hip):
    b = ic.solar_random(100, seed=1)
    b.pos[5] = np.nan
    eng = _engine(b.n, "fp32")
    eng.load(b)
    assert eng.nonfinite() > 0
    eng.close()


@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("kernel", ["lds", "smem"])
def test_fast_cutoff_bit_identical_to_exact(hip, dtype, kernel):
    """The fast path (cutoff inside an overflow-safe core, no select) equals the hard-cutoff
    select bit for bit on the reference ICs (all separations >> the ~mm core)."""
    outs = {}
    for mode in ("exact", "fast"):
        eng = _engine(6000, dtype, cutoff_mode=mode, kernel=kernel, ipl=2 if dtype == "fp64" else 8)
        eng.init_ics("solar+random", 77)
        fm = eng.force_mode()
        assert fm["exact"] == (mode == "exact")
        eng.step(4)
        outs[mode] = eng.state()
        eng.close()
    assert np.array_equal(outs["fast"].pos, outs["exact"].pos)
    assert np.array_equal(outs["fast"].vel, outs["exact"].vel)


def test_auto_cutoff_mode_resolution(hip):
    eng = _engine(100, "fp32")
    eng.init_ics("solar+random", 1)
    fm = eng.force_mode()
    assert not fm["exact"] and 1e-13 < fm["eps2"] < 1e-10  # default 1e-10 m cutoff -> fast
    eng.close()
    eng = _engine(100, "fp32", cutoff=1e3)  # a 1 km cutoff needs the exact select
    eng.init_ics("solar+random", 1)
    assert eng.force_mode()["exact"]
    eng.close()
    # fp64: the fast path softens at the cutoff scale (bit-identical above ~1 cm)
    eng = _engine(100, "fp64")
    eng.init_ics("solar+random", 1)
    fm = eng.force_mode()
    assert not fm["exact"] and fm["eps2"] == pytest.approx(1e-20)
    eng.close()
    eng = _engine(100, "fp64", cutoff=1e3)
    eng.init_ics("solar+random", 1)
    assert eng.force_mode()["exact"]
    eng.close()


def test_fast_path_self_term_zero_with_coincident_bodies(hip):
    """Coincident distinct bodies: the reference gives them zero mutual force (r < cutoff)."""
    pos = np.array([[1e11, 0, 0], [1e11, 0, 0], [-1e11, 0, 0]])
    mass = np.array([1e25, 1e25, 1e30])
    b = BodySet(pos, np.zeros((3, 3)), mass)
    eng = _engine(3, "fp32", cutoff_mode="fast")
    eng.load(b)
    eng.step(1)
    got = eng.state()
    eng.close()
    x, v, _ = oracle.simulate(pos, np.zeros((3, 3)), mass, 3600.0, 1)
    assert np.isfinite(got.pos).all()
    assert np.allclose(got.vel, v, rtol=1e-5, atol=1e-12)


def _clustered(n, seed=5, center=(3.0e11, 2.0e11, -1.0e11), radius=1.0e9):
    rng = np.random.default_rng(seed)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    pos = np.asarray(center) + d * (radius * rng.random(n) ** (1 / 3))[:, None]
    return BodySet(pos, np.zeros((n, 3)), 10 ** rng.uniform(22, 24, n))


@pytest.mark.parametrize("ics", ["clustered", "solar+random"])
def test_mfma_variant_vs_oracle(hip, ics):
    """Experimental MFMA kernel (r^2 as a 16x16x4 f32 GEMM on re-centred coordinates) vs the
    fp64 oracle: a cluster 1e9 m wide, 3.7e11 m from the origin, would cancel completely
    without re-centring (|x|^2 ~ 1e23 m^2 vs r^2 ~ 1e16). Bounds are from the measured
    errors in profiles/r1_mfma_probe.jsonl, with margin; the VALU kernel is far tighter.
    Without re-centring the median error of the cluster case would be O(1)."""
    from gravsim.config import G_SI
    from gravsim.runtime.engines import HipEngine

    b = _clustered(4096) if ics == "clustered" else ic.solar_random(4096, 3)
    p = b.pos.astype(np.float32).astype(np.float64)
    mu = (G_SI * b.mass).astype(np.float32).astype(np.float64)
    ref = oracle.accelerations(p, mu, G=1.0)
    e = HipEngine(SimConfig(n=b.n, dtype="fp32", device="gpu", kernel="mfma"))
    assert e.native_layout["kernel"] == 3 and e.native_layout["mode"] == 2
    e.load(b)
    a = e.accel(step_path=True)[: b.n, :3]
    e.close()
    rel = np.linalg.norm(a - ref, axis=1) / np.linalg.norm(ref, axis=1)
    assert np.isfinite(a).all()
    # Median and 90th percentile only: the tail is the expanded form's cancellation for close
    # pairs (p99 ~ 1e-3, max ~ 1e-2), the reason the variant is not the default.
    assert np.median(rel) < 2e-5
    assert np.quantile(rel, 0.9) < 1e-3


def test_mfma_variant_deterministic_and_rank_count_independent(hip):
    """Same i-blocks and re-centring origin for every P: P virtual shards == 1 rank, bitwise,
    and two runs agree (fixed in-lane order + fixed xor butterfly, no atomics)."""
    from gravsim.runtime.engines import VirtualGroup

    cfg = SimConfig(n=6000, dtype="fp32", device="gpu", chunk=1024, kernel="mfma")
    outs = []
    for P in (1, 3, 1):
        g = VirtualGroup(cfg, P)
        g.init_ics("solar+random", 2)
        g.step(4)
        outs.append(g.state())
        g.close()
    for o in outs[1:]:
        assert np.array_equal(o.pos, outs[0].pos) and np.array_equal(o.vel, outs[0].vel)
    assert np.isfinite(outs[0].pos).all()


def test_fused_engine_allocates_partials_on_demand(hip):
    """A single-rank fused Stepper skips the per-chunk partial buffer; an accel query
    allocates it lazily and matches the split engine bit for bit."""
    b = ic.solar_random(3000, 4)
    got = {m: _accel(b, "fp32", mode=m, chunk=1024) for m in ("fused", "split")}
    assert np.array_equal(got["fused"], got["split"])
