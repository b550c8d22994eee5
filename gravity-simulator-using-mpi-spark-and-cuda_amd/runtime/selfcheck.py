"""Pre-run self-check of the multi-rank sym schedule's gated launch (bench.py and the CLI).

The default multi-rank step (overlap 3) starts the rank-local force units before the RCCL
all-gather has landed and lets each remote unit test a gate flag the comm stream sets
(csrc/hip/nbody_sym.hip gate_open_or_defer). Its correctness rests on a system-scope
acquire of rows written by peer GPUs over xGMI, which a one-GPU box never exercises. So
before a multi-rank run commits to it, both schedules run the same few steps from the same
initial state on every rank; they evaluate the same units into the same slots, so their bits
must agree (docs/DESIGN.md §7). If they do not, the run uses the ungated schedule (overlap 0,
which waits for the gather) and says so. The reference's per-step exchange has no such
question: it blocks in MPI_Allgatherv + MPI_Barrier (mpi.c:227-236).
"""
from __future__ import annotations

import time
from typing import Callable


def gated_self_check(eng, dist, comm, reload: Callable[[], None], steps: int = 2,
                     race: int = 0) -> tuple[int, str, float]:
    """Run `steps` steps with the ungated (0) and the gated (3) schedule from `reload()`'s state
    on every rank and compare the bits. With race > 0 and equal bits, keep the faster one in an
    alternating race of `race` steps per turn (slowest rank's wall). Returns (overlap mode,
    verdict, seconds per step of the last timed steps: the run's step-time estimate). The
    caller reloads its own initial state afterwards."""
    import numpy as np

    out, per_step = [], 0.0
    for ov in (0, 3):
        eng.set_overlap(ov)
        reload()
        eng.sync()
        t0 = time.perf_counter()
        eng.step(steps)
        eng.sync()
        per_step = comm.allreduce_max(dist, (time.perf_counter() - t0) / max(steps, 1))
        b = eng.state()
        own = eng.layout.real_local
        out.append((b.pos[own.start:own.stop].copy(), b.vel[own.start:own.stop].copy()))
    same = all(np.array_equal(x, y) for x, y in zip(out[0], out[1]))
    bad = comm.allreduce_sum(dist, 0.0 if same else 1.0)
    if bad:
        eng.set_overlap(0)
        return 0, (f"gated launch differed from the ungated one on {int(bad)} rank(s) after "
                   f"{steps} steps: overlap 0"), per_step
    if race <= 0:
        eng.set_overlap(3)
        return 3, f"gated == ungated bitwise after {steps} steps on every rank: overlap 3", \
            per_step
    # Same bits either way, so keep whichever is faster on THIS node's interconnect (the
    # gated launch won under modeled comm, but real RCCL kernels compete for CUs
    # differently): alternating untimed races, slowest rank's wall per mode.
    wall = {0: 0.0, 3: 0.0}
    for ov in (0, 3, 0, 3):
        eng.set_overlap(ov)
        eng.step(1)
        eng.sync()
        comm.barrier(dist)
        t0 = time.perf_counter()
        eng.step(race)
        eng.sync()
        wall[ov] += comm.allreduce_max(dist, time.perf_counter() - t0)
    ms = {ov: 1e3 * w / (2 * race) for ov, w in wall.items()}
    pick = 3 if ms[3] <= ms[0] else 0
    eng.set_overlap(pick)
    return pick, (f"gated == ungated bitwise after {steps} steps on every rank; race "
                  f"{ms[0]:.3f} ms ungated vs {ms[3]:.3f} ms gated per step: overlap {pick}"), \
        min(ms.values()) * 1e-3
