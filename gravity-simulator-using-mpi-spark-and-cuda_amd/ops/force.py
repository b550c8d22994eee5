"""Stateless force entry points (one-shot accelerations of a body set).

The reference computes forces three ways: a racy upper-triangle CUDA kernel with Newton-3
scatter (cuda.cu:32-60), a full-row C loop (mpi.c:196-205), and a Spark pair map with a
driver-side reduction (pyspark.py:59-86). All three are replaced by i-owned full-row sums.
"""
from __future__ import annotations

import numpy as np

from ..config import G_SI, SimConfig
from ..models.initial_conditions import BodySet
from ..parallel.partition import layout
from . import _native, oracle


def cpu_accelerations(pos, mass, dtype: str = "fp64", G: float = G_SI, cutoff: float = 1e-10,
                      softening: float = 0.0, chunk: int = 0):
    """Native C++ engine: returns (acc (n,3), phi (n,)) as float64 arrays."""
    lib = _native.cpu_lib()
    n = int(np.asarray(mass).shape[0])
    L = layout(n, 0, 1, chunk)
    T = np.float64 if dtype == "fp64" else np.float32
    X = np.zeros((L.n_pad, 4), T)
    X[:n, :3] = pos
    X[:n, 3] = G * np.asarray(mass, dtype=np.float64)
    out = np.zeros((n, 4), T)
    fn = lib.gs_cpu_accel_f64 if dtype == "fp64" else lib.gs_cpu_accel_f32
    ptr = _native.dptr if dtype == "fp64" else _native.fptr
    _native.check(lib, fn(ptr(X), n, 0, n, L.chunk, T(cutoff * cutoff), T(softening ** 2),
                          ptr(out)), "cpu accel")
    out = out.astype(np.float64)
    return out[:, :3], out[:, 3]


def hip_accelerations(pos, mass, dtype: str = "fp32", G: float = G_SI, cutoff: float = 1e-10,
                      softening: float = 0.0, kernel: str = "auto", ipl: int = 0,
                      chunk: int = 0, mode: str = "auto"):
    """gfx950 kernels: returns (acc (n,3), phi (n,)). Raises if the HIP path is unavailable."""
    from ..runtime.engines import HipEngine

    n = int(np.asarray(mass).shape[0])
    cfg = SimConfig(n=n, dtype=dtype, G=G, cutoff=cutoff, softening=softening, kernel=kernel,
                    ipl=ipl, chunk=chunk, mode=mode, device="gpu")
    eng = HipEngine(cfg)
    try:
        eng.load(BodySet(np.asarray(pos, np.float64), np.zeros((n, 3)),
                         np.asarray(mass, np.float64)))
        a = eng.accel()[:n]
    finally:
        eng.close()
    return a[:, :3], a[:, 3]


def accelerations(pos, mass, device: str = "cpu", **kw):
    """Dispatch: device in {"oracle", "cpu", "gpu"}."""
    if device == "oracle":
        kw.pop("dtype", None)
        return oracle.accelerations(pos, mass, with_potential=True, **kw)
    if device == "cpu":
        return cpu_accelerations(pos, mass, **kw)
    if device == "gpu":
        return hip_accelerations(pos, mass, **kw)
    raise ValueError(f"unknown device {device!r}")
