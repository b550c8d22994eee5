"""Object API with the reference's names, backed by the native engines.

pyspark.py is the only reference program with a programmatic surface. This module offers the
same names, so code written against it ports by changing the import:

  Particle (pyspark.py:10-29)             -> Particle (dataclass, to_dict / from_dict)
  create_solar_system() (pyspark.py:124-141)
  generate_random_particles(n) (:144-149) -> seeded counter RNG (``seed=``), same ranges
  calculate_force_between(p1, p2, G) (:32-42) -> the pair force on p1 from p2 (dicts, a list)
  SparkGravitySimulator(particles, dt, cores, memory) (:45-57)
      .calculate_forces() (:59-86)        -> per-body force vectors F_i = m_i a_i (list)
      .update() (:88-102)                 -> one kick-drift step
      .run_simulation(steps) (:104-121)   -> per-body position trajectories (list of tuples)

``GravitySimulator`` is the same class under a neutral name. It runs on the MI355X Stepper
(``device="gpu"``) or the native CPU engine (``device="cpu"``). ``cores`` maps to CPU threads;
``memory`` is accepted and ignored (there is no JVM).

Differences by design: forces come from i-owned direct sums (no O(N²) pair list and no driver
reduction), every step uses start-of-step positions, and the RNG is seeded.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from .config import G_SI, SimConfig
from .models import initial_conditions as ic
from .models.initial_conditions import BodySet


@dataclass
class Particle:
    position: np.ndarray
    velocity: np.ndarray
    mass: float

    def to_dict(self) -> dict:
        return {"position": np.asarray(self.position, float).tolist(),
                "velocity": np.asarray(self.velocity, float).tolist(),
                "mass": float(self.mass)}

    @staticmethod
    def from_dict(d: dict) -> "Particle":
        return Particle(position=np.array(d["position"], float),
                        velocity=np.array(d["velocity"], float), mass=float(d["mass"]))


def calculate_force_between(p1_data: dict, p2_data: dict, G: float = G_SI,
                            cutoff: float = 1e-10) -> List[float]:
    """Force on body 1 from body 2 (the dict form of Particle.to_dict), as a 3-list:
    G m1 m2 (x2 - x1) / r^3, or zeros closer than `cutoff` (pyspark.py:32-42, mpi.c:59-73).
    A scalar helper for code written against the reference; the engines never call it."""
    d = np.asarray(p2_data["position"], float) - np.asarray(p1_data["position"], float)
    r = float(np.sqrt(d @ d))
    if r < cutoff:
        return [0.0, 0.0, 0.0]
    return (G * float(p1_data["mass"]) * float(p2_data["mass"]) / (r * r * r) * d).tolist()


def create_solar_system() -> List[Particle]:
    """Sun, Earth, Mars (pyspark.py:124-141, cuda.cu:81-96, mpi.c:75-95)."""
    return [Particle(np.array([x, 0.0, 0.0]), np.array([0.0, vy, 0.0]), m)
            for _, x, vy, m in ic.SOLAR]


def generate_random_particles(num_particles: int, seed: int = 0,
                              first_index: int = 3) -> List[Particle]:
    """Uniform bodies (pyspark.py:144-149 ranges) from the seeded counter RNG; body indices
    start at `first_index`, so create_solar_system() + this equals the solar+random model."""
    idx = np.arange(first_index, first_index + num_particles, dtype=np.int64)
    pos, vel, mass = ic.uniform_bodies(seed, idx)
    return [Particle(pos[i], vel[i], float(mass[i])) for i in range(num_particles)]


def _bodies(particles: Sequence) -> BodySet:
    ps = [p if isinstance(p, Particle) else Particle.from_dict(p) for p in particles]
    return BodySet(np.array([p.position for p in ps], float).reshape(-1, 3),
                   np.array([p.velocity for p in ps], float).reshape(-1, 3),
                   np.array([p.mass for p in ps], float))


class GravitySimulator:
    G = G_SI

    def __init__(self, particles: Sequence, dt: float = 0.01, cores: int = 0,
                 memory: str = "", device: str = "auto", dtype: str = "fp64",
                 cutoff: float = 1e-10, softening: float = 0.0, progress: bool = True):
        from .runtime.engines import CpuEngine, HipEngine, gpu_available

        b = _bodies(particles)
        self.num_particles = b.n
        self.dt = float(dt)
        self.progress = progress
        use_gpu = device == "gpu" or (device == "auto" and gpu_available())
        self.cfg = SimConfig(n=b.n, dt=self.dt, dtype=dtype, device="gpu" if use_gpu else "cpu",
                             G=self.G, cutoff=cutoff, softening=softening,
                             threads=int(cores or 0)).validate()
        self.engine = HipEngine(self.cfg) if use_gpu else CpuEngine(self.cfg)
        self.engine.load(b)
        self._mass = b.mass

    @property
    def particles_data(self) -> List[dict]:
        b = self.engine.state()
        return [{"position": b.pos[i].tolist(), "velocity": b.vel[i].tolist(),
                 "mass": float(b.mass[i])} for i in range(self.num_particles)]

    def calculate_forces(self) -> List[np.ndarray]:
        """Net gravitational force on every body for the current positions (N)."""
        a = self.engine.accel()[: self.num_particles, :3]
        return list(self._mass[:, None] * a)

    def update(self) -> None:
        """One kick-drift step (pyspark.py:88-102)."""
        self.engine.step(1)

    def run_simulation(self, steps: int) -> List[List[Tuple[float, float, float]]]:
        trajectories: List[List[Tuple[float, float, float]]] = [[] for _ in
                                                                 range(self.num_particles)]
        t0 = time.time()
        for step in range(steps):
            if self.progress and step % 100 == 0:
                print(f"Step {step}/{steps}")
            self.engine.step(1)
            pos = self.engine.state().pos
            for i in range(self.num_particles):
                trajectories[i].append(tuple(float(c) for c in pos[i]))
        if self.progress:
            print(f"Simulation took {time.time() - t0:.2f} seconds")
        return trajectories

    def close(self) -> None:
        self.engine.close()


SparkGravitySimulator = GravitySimulator
