"""Text logs and final-state dumps in the reference's three formats.

mpi   (canonical, mpi.c:110-138,242-262):
        gravity_logs_mpi/mpi_c_simulation_%Y%m%d_%H%M%S.txt, header, stats, every particle as
        "Particle %d: (%e, %e, %e)", "Simulation completed successfully".
spark (pyspark.py:153-163,181-200):
        gravity_logs_spark/simulation_log_%Y%m%d_%H%M%S.txt; every line is also printed; one
        block per configuration of a sweep; positions as Python tuple reprs.
cuda  (cuda.cu:99-117,140-175):
        gravity_logs_spark/simulation_log_<epoch>.txt with start/step/took/completed lines;
        the first 10 final positions go to stdout only, fixed with 14 decimals. Unlike the
        reference (D13) the directory is created.
"""
from __future__ import annotations

import datetime
import os
import time
from typing import Iterable, Optional, TextIO

import numpy as np


def _stamp(now: Optional[datetime.datetime] = None) -> str:
    return (now or datetime.datetime.now()).strftime("%Y%m%d_%H%M%S")


class RunLog:
    """Writes one run's log in a reference format. `path` is None when file logging is off."""

    def __init__(self, fmt: str, log_dir: Optional[str], echo: bool = True,
                 now: Optional[datetime.datetime] = None, stdout: Optional[TextIO] = None):
        self.fmt = fmt
        self.echo = echo
        self.stdout = stdout
        self.path: Optional[str] = None
        self.stamp = _stamp(now)
        if fmt != "none" and log_dir is not None:
            sub = {"mpi": "gravity_logs_mpi", "spark": "gravity_logs_spark",
                   "cuda": "gravity_logs_spark"}[fmt]
            d = os.path.join(log_dir, sub)
            os.makedirs(d, mode=0o700, exist_ok=True)  # mpi.c:112-118 uses 0700
            if fmt == "mpi":
                name = f"mpi_c_simulation_{self.stamp}.txt"
            elif fmt == "spark":
                name = f"simulation_log_{self.stamp}.txt"
            else:
                name = f"simulation_log_{int(time.time())}.txt"
            self.path = os.path.join(d, name)
            if fmt == "mpi":
                open(self.path, "w").close()

    # -- primitives -----------------------------------------------------------------------
    def _file(self, text: str) -> None:
        if self.path:
            with open(self.path, "a") as f:
                f.write(text)

    def _out(self, text: str) -> None:
        if self.echo:
            import sys

            (self.stdout or sys.stdout).write(text)
            (self.stdout or sys.stdout).flush()

    def line(self, msg: str) -> None:
        """log_print: stdout + file (pyspark.py:160-163, cuda.cu:113-117)."""
        self._out(msg + "\n")
        self._file(msg + "\n")

    # -- run phases -----------------------------------------------------------------------
    def header(self, nranks: int, n: int, steps: int, dt: float, cores: int = 0) -> None:
        if self.fmt == "mpi":
            self._file(f"Starting MPI C gravity simulation at {self.stamp}\n"
                       f"Number of processes: {nranks}\n"
                       f"Number of particles: {n}\n"
                       f"Steps: {steps}\n"
                       f"Timestep: {dt:f} seconds\n\n")
        elif self.fmt == "spark":
            self.line(f"\nStarting gravity simulation with {cores or nranks} cores and {n} particles")
            self.line("Configuration:")
            self.line(f"- Number of steps: {steps}")
            self.line(f"- Time step: {dt:g} seconds ({dt / 3600:g} hour)")
        elif self.fmt == "cuda":
            self.line("Starting gravity simulation")

    def progress(self, step: int, steps: int) -> None:
        if self.fmt == "cuda":
            self.line(f"Step {step}")
        else:
            self._out(f"Step {step}/{steps}\n")  # mpi.c:192-193, pyspark.py:109-110

    def stats(self, total_s: float, steps: int) -> None:
        per = total_s / steps if steps else 0.0
        if self.fmt == "mpi":
            self._file("\nPerformance Statistics:\n"
                       f"Total execution time: {total_s:.2f} seconds\n"
                       f"Average time per step: {per:.4f} seconds\n")
        elif self.fmt == "spark":
            self._out(f"Simulation took {total_s:.2f} seconds\n")  # pyspark.py:118
            self.line("\nPerformance Statistics:")
            self.line(f"Total execution time: {total_s:.2f} seconds")
            self.line(f"Average time per step: {per:.4f} seconds")
        elif self.fmt == "cuda":
            self.line(f"Simulation took {total_s:f} seconds")

    def positions(self, pos: np.ndarray, limit_stdout: int = 10) -> None:
        n = pos.shape[0]
        if self.fmt == "mpi":
            lines = "".join(f"Particle {i}: ({p[0]:e}, {p[1]:e}, {p[2]:e})\n"
                            for i, p in enumerate(pos))
            self._file("\nFinal positions:\n" + lines)
        elif self.fmt == "spark":
            self.line("\nFinal positions:")
            for i, p in enumerate(pos):
                self.line(f"Particle {i}: {tuple(float(c) for c in p)}")
        elif self.fmt == "cuda":
            k = min(limit_stdout, n)
            self._out(f"\nFinal positions of first {k} out of {n} particles:\n")
            for i in range(k):
                p = pos[i]
                self._out(f"Particle {i}: ({p[0]:.14f}, {p[1]:.14f}, {p[2]:.14f})\n")

    def completed(self) -> None:
        if self.fmt == "mpi":
            self._file("\nSimulation completed successfully\n")
        elif self.fmt == "spark":
            self.line("\nSimulation completed successfully")
        elif self.fmt == "cuda":
            self.line("Simulation completed successfully")


def format_positions_mpi(pos: Iterable) -> str:
    return "".join(f"Particle {i}: ({p[0]:e}, {p[1]:e}, {p[2]:e})\n" for i, p in enumerate(pos))
