"""Conserved-quantity diagnostics (not present in the reference, which only prints positions).

Used by the tests (Newton-3 momentum conservation, symplectic energy behaviour) and by the
driver's optional per-run summary.
"""
from __future__ import annotations

import numpy as np

from ..config import G_SI


def momentum(vel: np.ndarray, mass: np.ndarray) -> np.ndarray:
    return (np.asarray(mass)[:, None] * np.asarray(vel)).sum(0)


def center_of_mass(pos: np.ndarray, mass: np.ndarray) -> np.ndarray:
    m = np.asarray(mass)
    return (m[:, None] * np.asarray(pos)).sum(0) / m.sum()


def kinetic_energy(vel, mass) -> float:
    return float(0.5 * (np.asarray(mass) * (np.asarray(vel) ** 2).sum(1)).sum())


def potential_energy(pos, mass, G: float = G_SI, cutoff: float = 1e-10, softening: float = 0.0,
                     phi: np.ndarray | None = None) -> float:
    """U = 1/2 sum_i m_i phi_i with phi_i = -sum_j G m_j / r_ij (same cutoff as the force)."""
    if phi is None:
        from ..ops.oracle import accelerations

        _, phi = accelerations(pos, mass, G, cutoff, softening, with_potential=True)
    return float(0.5 * (np.asarray(mass) * phi).sum())


def energy(pos, vel, mass, G: float = G_SI, cutoff: float = 1e-10, softening: float = 0.0,
           phi: np.ndarray | None = None) -> float:
    return kinetic_energy(vel, mass) + potential_energy(pos, mass, G, cutoff, softening, phi)
