"""NumPy fp64 oracle: the intended physics of the reference, as one vectorised function.

    a_i = sum_{j : |x_j - x_i| >= r_cut} G m_j (x_j - x_i) / |x_j - x_i|^3      (mpi.c:59-73)
    v <- v + a dt ;  x <- x + v dt                                             (mpi.c:206-215)

with every acceleration of a step evaluated from the positions at the start of that step
(synchronous / Jacobi). This is NOT the reference output — cuda.cu overflows in fp32 and
never refreshes its device positions, and mpi.c updates in place — but the physics all three
programs intend. Optional Plummer softening eps: r^2 -> r^2 + eps^2.
"""
from __future__ import annotations

import os

import numpy as np

from ..config import G_SI


def accelerations(pos: np.ndarray, mass: np.ndarray, G: float = G_SI, cutoff: float = 1e-10,
                  softening: float = 0.0, block: int = 256, with_potential: bool = False,
                  with_abs: bool = False):
    """Direct-sum accelerations (n, 3) in fp64; optionally the potential phi (n,) too.

    with_abs also returns sum_j |term_ij| per component (n, 3): the scale against which a
    floating-point sum of the terms should be judged (error <= c * eps * sum |terms|)."""
    pos = np.asarray(pos, dtype=np.float64)
    mu = G * np.asarray(mass, dtype=np.float64)
    n = pos.shape[0]
    acc = np.zeros((n, 3))
    absacc = np.zeros((n, 3))
    phi = np.zeros(n)
    cut2 = cutoff * cutoff
    eps2 = softening * softening

    def rows(i0: int) -> None:
        i1 = min(n, i0 + block)
        d = pos[None, :, :] - pos[i0:i1, None, :]            # (b, n, 3)  x_j - x_i
        r2 = (d * d).sum(-1) + eps2
        ok = r2 >= cut2
        inv = np.zeros_like(r2)
        inv[ok] = 1.0 / np.sqrt(r2[ok])
        mi = mu[None, :] * inv
        s = mi * inv * inv
        acc[i0:i1] = (s[:, :, None] * d).sum(1)
        if with_abs:
            absacc[i0:i1] = (s[:, :, None] * np.abs(d)).sum(1)
        phi[i0:i1] = -mi.sum(1)

    starts = range(0, n, block)
    if n * n >= 1 << 24 and len(starts) > 1:
        # Row blocks are independent (each writes its own rows; same bits in any order) and
        # NumPy releases the GIL inside these array operations: a few threads cut the
        # oracle's wall time on the large reference sums the tests use.
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
            list(ex.map(rows, starts))
    else:
        for i0 in starts:
            rows(i0)
    out = (acc,)
    if with_potential:
        out += (phi,)
    if with_abs:
        out += (absacc,)
    return out if len(out) > 1 else acc


def step(pos, vel, mass, dt, G=G_SI, cutoff=1e-10, softening=0.0):
    """One synchronous kick-drift step; returns new (pos, vel)."""
    a = accelerations(pos, mass, G, cutoff, softening)
    v = vel + a * dt
    x = pos + v * dt
    return x, v


def simulate(pos, vel, mass, dt, steps, G=G_SI, cutoff=1e-10, softening=0.0, record_every=0,
             integrator="kd"):
    """Run `steps` steps. Returns (pos, vel, trajectory list of positions if record_every).

    integrator "leapfrog": kick-drift-kick, v_{1/2} = v_0 + a_0 dt/2, x_1 = x_0 + v_{1/2} dt,
    v_1 = v_{1/2} + a_1 dt/2 (velocities returned synchronized)."""
    x = np.array(pos, dtype=np.float64, copy=True)
    v = np.array(vel, dtype=np.float64, copy=True)
    traj = []
    if integrator == "leapfrog":
        a = accelerations(x, mass, G, cutoff, softening)
        for s in range(steps):
            v = v + 0.5 * dt * a
            x = x + v * dt
            a = accelerations(x, mass, G, cutoff, softening)
            v = v + 0.5 * dt * a
            if record_every and (s + 1) % record_every == 0:
                traj.append(x.copy())
        return x, v, traj
    for s in range(steps):
        x, v = step(x, v, mass, dt, G, cutoff, softening)
        if record_every and (s + 1) % record_every == 0:
            traj.append(x.copy())
    return x, v, traj


def gauss_seidel_step(pos, vel, mass, dt, nranks, G=G_SI, cutoff=1e-10):
    """Emulation of mpi.c's in-place update inside each rank's block (mpi.c:196-216, D6).

    Kept only to document the defect in tests: results depend on `nranks`.
    """
    x = np.array(pos, dtype=np.float64, copy=True)
    v = np.array(vel, dtype=np.float64, copy=True)
    n = x.shape[0]
    base, rem = divmod(n, nranks)
    snapshot = x.copy()  # what other ranks hold until the Allgatherv
    new_x = x.copy()
    for r in range(nranks):
        start = r * base + min(r, rem)
        cnt = base + (1 if r < rem else 0)
        local = snapshot.copy()
        for i in range(start, start + cnt):
            d = local - local[i]
            r2 = (d * d).sum(1)
            ok = r2 >= cutoff * cutoff
            ok[i] = False
            inv = np.zeros(n)
            inv[ok] = 1.0 / np.sqrt(r2[ok])
            a = ((G * mass * inv ** 3)[:, None] * d).sum(0)
            v[i] = v[i] + a * dt
            local[i] = local[i] + v[i] * dt
            new_x[i] = local[i]
    return new_x, v
