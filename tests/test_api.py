"""pyspark.py-compatible object API (Particle, create_solar_system, generate_random_particles,
SparkGravitySimulator.calculate_forces / update / run_simulation) on the native CPU engine."""
import numpy as np

from gravsim.api import (GravitySimulator, Particle, SparkGravitySimulator, create_solar_system,
                         generate_random_particles)
from gravsim.models import initial_conditions as ic
from gravsim.ops import oracle


def test_particle_roundtrip_and_solar_system():
    s = create_solar_system()
    assert len(s) == 3 and s[0].mass == 1.989e30 and s[1].velocity[1] == 29.78e3
    d = s[2].to_dict()
    assert Particle.from_dict(d).to_dict() == d


def test_random_particles_match_model_and_ranges():
    ps = generate_random_particles(50, seed=7)
    ref = ic.solar_random(53, 7)
    assert np.array_equal(np.array([p.position for p in ps]), ref.pos[3:])
    assert all(1e23 <= p.mass < 1e25 for p in ps)


def test_spark_style_run_simulation(capsys):
    particles = create_solar_system() + generate_random_particles(37, seed=1)
    sim = SparkGravitySimulator(particles, dt=3600, cores=2, memory="4g", device="cpu")
    forces = sim.calculate_forces()
    b = ic.solar_random(40, 1)
    a = oracle.accelerations(b.pos, b.mass)
    assert np.allclose(np.array(forces), b.mass[:, None] * a, rtol=1e-12)
    traj = sim.run_simulation(5)
    assert len(traj) == 40 and len(traj[0]) == 5 and len(traj[0][0]) == 3
    x, _, _ = oracle.simulate(b.pos, b.vel, b.mass, 3600.0, 5)
    assert np.allclose(np.array([t[-1] for t in traj]), x, rtol=1e-12)
    assert "Step 0/5" in capsys.readouterr().out
    sim.update()
    assert len(sim.particles_data) == 40
    sim.close()
    assert GravitySimulator is SparkGravitySimulator


def test_calculate_force_between_pair_law():
    """The reference's scalar pair force (pyspark.py:32-42): G m1 m2 / r^2 along r, equal and
    opposite, zero inside the 1e-10 m cutoff; m1 times the oracle's acceleration of body 1."""
    from gravsim.api import calculate_force_between
    from gravsim.config import G_SI

    s = [p.to_dict() for p in create_solar_system()]
    f = np.array(calculate_force_between(s[1], s[0]))  # Earth pulled toward the Sun
    r = 1.496e11
    assert f[1] == 0.0 and f[2] == 0.0 and f[0] < 0
    assert np.isclose(-f[0], G_SI * 1.989e30 * 5.972e24 / r**2, rtol=1e-15)
    assert np.allclose(calculate_force_between(s[0], s[1]), -f, rtol=1e-15)
    pos = np.array([p["position"] for p in s[:2]])
    acc = oracle.accelerations(pos, np.array([p["mass"] for p in s[:2]]))
    assert np.allclose(f, s[1]["mass"] * acc[1], rtol=1e-12)
    near = dict(s[1], position=[1.496e11 + 5e-11, 0.0, 0.0])
    assert calculate_force_between(s[1], near) == [0.0, 0.0, 0.0]
