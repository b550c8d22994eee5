"""Initial-condition families ("models").

The reference has exactly one model: Sun, Earth, Mars plus uniform-random bodies, generated
three times with three unseeded RNGs (cuda.cu:81-96,127-138; mpi.c:75-105;
pyspark.py:124-149). Here every family is a pure function of (seed, body index) built on a
counter-based SplitMix64 hash, so

* any rank can generate any slice without communication (replaces MPI_Bcast, mpi.c:182);
* runs are reproducible (fixes D11) and identical for every world size;
* the NumPy version below is bit-for-bit equal to the C++/HIP version in
  csrc/include/gs_common.h (`gs::ic_body`), which the GPU init kernel uses.

Families:
  solar+random  Sun/Earth/Mars then U[-3e11,3e11]^3 m, U[-3e4,3e4]^3 m/s, U[1e23,1e25] kg
  random        the uniform bodies only (no solar bodies)
  plummer       Plummer sphere in virial equilibrium (host-generated)
  kepler        Sun + Earth on a circular orbit (host-generated; orbit-closure tests)
  cold          uniform-density sphere at rest (host-generated; cold collapse)
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..config import G_SI

POS_LO, POS_HI = -3e11, 3e11
VEL_LO, VEL_HI = -3e4, 3e4
MASS_LO, MASS_HI = 1e23, 1e25

# (position x, velocity y, mass) of the reference solar bodies (cuda.cu:82-93, mpi.c:79-93,
# pyspark.py:126-141).
SOLAR = (
    ("Sun", 0.0, 0.0, 1.989e30),
    ("Earth", 1.496e11, 29.78e3, 5.972e24),
    ("Mars", 2.279e11, 24.077e3, 6.39e23),
)

DEVICE_IC_IDS = {"solar+random": 0, "random": 1}
FAMILIES = ("solar+random", "random", "plummer", "kepler", "cold")

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_GOLD = np.uint64(0x9E3779B97F4A7C15)
_KEY = np.uint64(0xD1B54A32D192ED03)


def mix64(z):
    """SplitMix64 finaliser on uint64 arrays (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = np.asarray(z, dtype=np.uint64) + _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def uniform01(seed: int, body, stream: int) -> np.ndarray:
    """U[0,1) doubles for (seed, body index array, stream) — matches gs::uniform01."""
    key = mix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ _KEY)
    with np.errstate(over="ignore"):
        ctr = np.asarray(body, dtype=np.uint64) * np.uint64(16) + np.uint64(stream)
    h = mix64(key ^ ctr)
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def _affine(lo: float, hi: float, u: np.ndarray) -> np.ndarray:
    return lo + (hi - lo) * u  # two roundings, no FMA: same as gs::affine


@dataclass
class BodySet:
    """Global fp64 state of a body set (SI units)."""

    pos: np.ndarray   # (n, 3) m
    vel: np.ndarray   # (n, 3) m/s
    mass: np.ndarray  # (n,) kg

    @property
    def n(self) -> int:
        return int(self.mass.shape[0])

    def copy(self) -> "BodySet":
        return BodySet(self.pos.copy(), self.vel.copy(), self.mass.copy())


def uniform_bodies(seed: int, idx: np.ndarray):
    idx = np.asarray(idx, dtype=np.int64)
    pos = np.stack([_affine(POS_LO, POS_HI, uniform01(seed, idx, d)) for d in range(3)], axis=1)
    vel = np.stack([_affine(VEL_LO, VEL_HI, uniform01(seed, idx, 3 + d)) for d in range(3)],
                   axis=1)
    mass = _affine(MASS_LO, MASS_HI, uniform01(seed, idx, 6))
    return pos, vel, mass


def solar_random(n: int, seed: int, begin: int = 0, end: int | None = None) -> BodySet:
    """Bodies [begin, end) of the reference model (solar bodies at indices 0-2)."""
    end = n if end is None else min(end, n)
    idx = np.arange(begin, end, dtype=np.int64)
    pos, vel, mass = uniform_bodies(seed, idx)
    for k, (_, x, vy, m) in enumerate(SOLAR):
        sel = idx == k
        if sel.any():
            pos[sel] = (x, 0.0, 0.0)
            vel[sel] = (0.0, vy, 0.0)
            mass[sel] = m
    return BodySet(pos, vel, mass)


def random_cube(n: int, seed: int, begin: int = 0, end: int | None = None) -> BodySet:
    end = n if end is None else min(end, n)
    pos, vel, mass = uniform_bodies(seed, np.arange(begin, end, dtype=np.int64))
    return BodySet(pos, vel, mass)


def plummer(n: int, seed: int, total_mass: float = 2e30, scale: float = 1.5e11,
            G: float = G_SI) -> BodySet:
    """Plummer sphere (Aarseth, Henon & Wielen 1974 sampling), equal masses, zero net momentum."""
    idx = np.arange(n, dtype=np.int64)
    u = [uniform01(seed, idx, s) for s in range(8)]
    # radius from the cumulative mass profile, truncated at 0.999 of the mass
    m = np.clip(u[0], 1e-10, 0.999)
    r = scale / np.sqrt(m ** (-2.0 / 3.0) - 1.0)
    cost = 2.0 * u[1] - 1.0
    phi = 2.0 * np.pi * u[2]
    sint = np.sqrt(1.0 - cost ** 2)
    pos = np.stack([r * sint * np.cos(phi), r * sint * np.sin(phi), r * cost], axis=1)
    # speed by von Neumann rejection on g(q) = q^2 (1 - q^2)^3.5, drawn from counter streams
    q = np.empty(n)
    todo = np.ones(n, dtype=bool)
    attempt = 0
    while todo.any():
        a = uniform01(seed + 1000003 * (attempt + 1), idx, 0)
        b = uniform01(seed + 1000003 * (attempt + 1), idx, 1)
        ok = todo & (0.1 * b < a ** 2 * (1.0 - a ** 2) ** 3.5)
        q[ok] = a[ok]
        todo &= ~ok
        attempt += 1
    vesc = np.sqrt(2.0 * G * total_mass) * (r ** 2 + scale ** 2) ** -0.25
    v = q * vesc
    cost = 2.0 * u[3] - 1.0
    phi = 2.0 * np.pi * u[4]
    sint = np.sqrt(1.0 - cost ** 2)
    vel = np.stack([v * sint * np.cos(phi), v * sint * np.sin(phi), v * cost], axis=1)
    mass = np.full(n, total_mass / n)
    pos -= (mass[:, None] * pos).sum(0) / mass.sum()
    vel -= (mass[:, None] * vel).sum(0) / mass.sum()
    return BodySet(pos, vel, mass)


def kepler(n: int = 2, seed: int = 0, G: float = G_SI) -> BodySet:
    """Sun + Earth on a circular orbit about their barycentre (n must be 2)."""
    if n != 2:
        raise ValueError("kepler model has exactly 2 bodies")
    ms, me, a = SOLAR[0][3], SOLAR[1][3], SOLAR[1][1]
    mt = ms + me
    v = np.sqrt(G * mt / a)
    pos = np.array([[-a * me / mt, 0.0, 0.0], [a * ms / mt, 0.0, 0.0]])
    vel = np.array([[0.0, -v * me / mt, 0.0], [0.0, v * ms / mt, 0.0]])
    return BodySet(pos, vel, np.array([ms, me]))


def cold_sphere(n: int, seed: int, radius: float = 3e11, total_mass: float = 2e30) -> BodySet:
    idx = np.arange(n, dtype=np.int64)
    r = radius * np.cbrt(uniform01(seed, idx, 0))
    cost = 2.0 * uniform01(seed, idx, 1) - 1.0
    phi = 2.0 * np.pi * uniform01(seed, idx, 2)
    sint = np.sqrt(1.0 - cost ** 2)
    pos = np.stack([r * sint * np.cos(phi), r * sint * np.sin(phi), r * cost], axis=1)
    return BodySet(pos, np.zeros((n, 3)), np.full(n, total_mass / n))


def make(family: str, n: int, seed: int, G: float = G_SI) -> BodySet:
    """Full global body set of a family."""
    if family == "solar+random":
        return solar_random(n, seed)
    if family == "random":
        return random_cube(n, seed)
    if family == "plummer":
        return plummer(n, seed, G=G)
    if family == "kepler":
        return kepler(n, seed, G=G)
    if family == "cold":
        return cold_sphere(n, seed)
    raise ValueError(f"unknown IC family {family!r}; choose from {FAMILIES}")
