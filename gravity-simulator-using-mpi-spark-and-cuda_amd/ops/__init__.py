"""Operators: gravitational accelerations and kick-drift steps.

Three implementations of the same math (reference: cuda.cu:32-78, mpi.c:59-73,196-216,
pyspark.py:32-42,59-102):
  * `oracle`  — NumPy fp64, vectorised, synchronous (Jacobi) update: the correctness oracle.
  * `cpu`     — native C++/OpenMP engine (libgravsim_cpu.so), canonical chunk order.
  * `hip`     — gfx950 HIP kernels behind the native Stepper (libgravsim_hip.so).
"""
from . import oracle  # noqa: F401
from .force import accelerations, cpu_accelerations  # noqa: F401
