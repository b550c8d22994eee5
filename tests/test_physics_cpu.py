"""Physics of the oracle and the native CPU engine (no GPU).

Pair-law identities (mpi.c:59-73), the KD integrator (mpi.c:206-215), the reference defects
the new design must not reproduce, and CPU engine vs oracle parity.
"""
import numpy as np
import pytest

from gravsim.config import G_SI, SimConfig
from gravsim.models import initial_conditions as ic
from gravsim.models.diagnostics import energy, momentum
from gravsim.models.initial_conditions import BodySet
from gravsim.ops import oracle
from gravsim.ops.force import cpu_accelerations
from gravsim.runtime.engines import CpuEngine


def test_two_body_force_law():
    pos = np.array([[0.0, 0, 0], [3.0e10, 4.0e10, 0]])
    mass = np.array([2e30, 5e24])
    a = oracle.accelerations(pos, mass)
    r = 5e10
    assert np.allclose(a[0], G_SI * mass[1] / r ** 2 * np.array([0.6, 0.8, 0]), rtol=1e-14)
    assert np.allclose(a[1], -G_SI * mass[0] / r ** 2 * np.array([0.6, 0.8, 0]), rtol=1e-14)


def test_newton_third_law_momentum_conserved():
    b = ic.solar_random(500, 2)
    a = oracle.accelerations(b.pos, b.mass)
    f = (b.mass[:, None] * a).sum(0)
    scale = (b.mass[:, None] * np.abs(a)).sum(0)
    assert np.all(np.abs(f) < 1e-12 * scale)


def test_cutoff_and_self_exclusion():
    pos = np.array([[0.0, 0, 0], [5e-11, 0, 0], [1.0, 0, 0]])
    mass = np.array([1e30, 1e30, 1.0])
    a = oracle.accelerations(pos, mass)
    # bodies 0,1 closer than 1e-10 m do not interact (mpi.c:64-66); self terms excluded
    assert a[0][0] == pytest.approx(G_SI * 1.0 / 1.0, rel=1e-12)
    a_cpu, _ = cpu_accelerations(pos, mass)
    assert np.allclose(a_cpu, a, rtol=1e-14)


@pytest.mark.parametrize("dtype,tol", [("fp64", 1e-14), ("fp32", 2e-6)])
def test_cpu_engine_matches_oracle(dtype, tol):
    b = ic.solar_random(1500, 8)
    ref, phi = oracle.accelerations(b.pos, b.mass, with_potential=True)
    a, p = cpu_accelerations(b.pos, b.mass, dtype=dtype)
    assert np.abs(a - ref).max() <= tol * np.abs(ref).max()
    assert np.abs(p - phi).max() <= tol * np.abs(phi).max()


def test_fp32_heavy_masses_do_not_overflow():
    """D1: cuda.cu's G*m_i*m_j overflows fp32 (81% of random pairs); mu_j = G m_j does not."""
    b = ic.solar_random(400, 6)
    gmm = np.float32(G_SI) * b.mass[3:200].astype(np.float32)[:, None] * \
        b.mass[3:200].astype(np.float32)[None, :]
    assert (~np.isfinite(gmm)).mean() > 0.5  # the reference's product overflows
    a, _ = cpu_accelerations(b.pos, b.mass, dtype="fp32")
    assert np.isfinite(a).all()


def test_kepler_orbit_closes_and_energy_bounded():
    """Sun+Earth, one year of 3600 s steps: KD (symplectic) closes the orbit, bounded energy."""
    b = ic.kepler()
    year = 365.25 * 86400
    steps = int(round(year / 3600))
    e0 = energy(b.pos, b.vel, b.mass)
    x, v = b.pos.copy(), b.vel.copy()
    es = []
    for s in range(steps):
        x, v = oracle.step(x, v, b.mass, 3600.0)
        if s % 500 == 0:
            es.append(energy(x, v, b.mass))
    rel = (x[1] - x[0]) - (b.pos[1] - b.pos[0])
    assert np.linalg.norm(rel) / 1.496e11 < 2e-3
    assert max(abs(e - e0) for e in es) / abs(e0) < 1e-4


def test_momentum_conserved_over_steps_cpu_engine():
    cfg = SimConfig(n=300, dtype="fp64", device="cpu", dt=3600.0)
    eng = CpuEngine(cfg)
    eng.init_ics("solar+random", 4)
    b0 = eng.state()
    p0 = momentum(b0.vel, b0.mass)
    eng.step(50)
    b1 = eng.state()
    p1 = momentum(b1.vel, b1.mass)
    scale = np.abs(b0.mass[:, None] * b0.vel).sum(0).max()
    assert np.abs(p1 - p0).max() < 1e-12 * scale


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_cpu_engine_steps_match_oracle(dtype):
    b = ic.solar_random(600, 12)
    cfg = SimConfig(n=b.n, dtype=dtype, device="cpu")
    eng = CpuEngine(cfg)
    eng.load(b)
    eng.step(25)
    got = eng.state()
    x, v, _ = oracle.simulate(b.pos, b.vel, b.mass, cfg.dt, 25)
    tol = 1e-12 if dtype == "fp64" else 2e-5
    assert np.abs(got.pos - x).max() / np.abs(x).max() < tol


def test_reference_gauss_seidel_depends_on_world_size():
    """D6: mpi.c's in-place update gives P-dependent results; the Jacobi oracle does not."""
    b = ic.solar_random(8, 1)
    outs = [oracle.gauss_seidel_step(b.pos, b.vel, b.mass, 3600.0, P)[0] for P in (1, 2, 8)]
    assert not np.array_equal(outs[0], outs[1])
    jac, _ = oracle.step(b.pos, b.vel, b.mass, 3600.0)
    assert np.allclose(outs[2], jac, rtol=1e-14, atol=0)  # P = N is Jacobi


def test_softening_removes_singularity():
    pos = np.array([[0.0, 0, 0], [1e-12, 0, 0]])
    mass = np.array([1e30, 1e30])
    a = oracle.accelerations(pos, mass, cutoff=0.0, softening=1e6)
    assert np.isfinite(a).all() and abs(a[0, 0]) < G_SI * 1e30 / 1e12
    a2, _ = cpu_accelerations(pos, mass, cutoff=0.0, softening=1e6)
    assert np.allclose(a, a2, rtol=1e-13)


def test_energy_drift_small_random_system():
    b = ic.plummer(200, 3)
    e0 = energy(b.pos, b.vel, b.mass)
    x, v, _ = oracle.simulate(b.pos, b.vel, b.mass, 3600.0, 100)
    assert abs(energy(x, v, b.mass) - e0) / abs(e0) < 1e-3


def test_bodyset_copy():
    b = BodySet(np.zeros((2, 3)), np.zeros((2, 3)), np.ones(2))
    c = b.copy()
    c.pos[0, 0] = 1
    assert b.pos[0, 0] == 0


def test_leapfrog_is_second_order_kd_first_order():
    """Quarter-orbit energy error of a circular Kepler orbit: kick-drift (symplectic Euler)
    scales ~dt^2, leapfrog (KDK) much faster (~dt^4 here) and is orders of magnitude smaller."""
    b = ic.kepler()
    e0 = energy(b.pos, b.vel, b.mass)
    errs = {}
    for integ in ("kd", "leapfrog"):
        for dt in (14400.0, 7200.0):
            steps = int(round(365.25 * 86400 / dt / 4))  # a quarter orbit
            x, v, _ = oracle.simulate(b.pos, b.vel, b.mass, dt, steps, integrator=integ)
            errs[(integ, dt)] = abs(energy(x, v, b.mass) - e0) / abs(e0)
    r_kd = errs[("kd", 14400.0)] / errs[("kd", 7200.0)]
    r_lf = errs[("leapfrog", 14400.0)] / errs[("leapfrog", 7200.0)]
    assert 3.0 < r_kd < 5.0 and r_lf > 8.0
    assert errs[("leapfrog", 7200.0)] < errs[("kd", 7200.0)] * 1e-4


@pytest.mark.parametrize("dtype", ["fp64"])
def test_leapfrog_driver_matches_oracle_kdk(dtype, tmp_path):
    """The driver's staggered-velocity leapfrog equals the textbook KDK update."""
    from gravsim.runtime.simulation import Simulation

    cfg = SimConfig(n=400, steps=12, dtype=dtype, device="cpu", integrator="leapfrog")
    sim = Simulation(cfg)
    b0 = ic.solar_random(400, cfg.seed)
    sim.run()
    got = sim.global_state()
    x, v, _ = oracle.simulate(b0.pos, b0.vel, b0.mass, cfg.dt, 12, integrator="leapfrog")
    assert np.abs(got.pos - x).max() / np.abs(x).max() < 1e-12
    assert np.abs(got.vel - v).max() / np.abs(v).max() < 1e-10
    # checkpoint keeps the staggered velocities: resume is bit-exact
    path = str(tmp_path / "c.gsck")
    sim.save_checkpoint(path)
    sim.run(3)
    ref = sim.global_state()
    sim2 = Simulation(cfg.replace(resume=path))
    sim2.run(3)
    got2 = sim2.global_state()
    assert np.array_equal(got2.pos, ref.pos) and np.array_equal(got2.vel, ref.vel)
