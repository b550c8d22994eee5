"""Accuracy and speed of the experimental MFMA kernel vs the VALU kernel (MI355X).

For each IC family: per-body relative error of the step-path accelerations against the fp64
oracle on fp32-rounded inputs, for kernel=mfma and kernel=smem; then ms/step at N = 1M.
    python bench/mfma_probe.py
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def clustered(n, seed=5, center=(3.0e11, 2.0e11, -1.0e11), radius=1.0e9):
    from gravsim.models.initial_conditions import BodySet

    rng = np.random.default_rng(seed)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = radius * rng.random(n) ** (1 / 3)
    pos = np.asarray(center) + d * r[:, None]
    return BodySet(pos, np.zeros((n, 3)), 10 ** rng.uniform(22, 24, n))


def main() -> int:
    import torch  # noqa: F401

    import gravsim  # noqa: F401
    from gravsim.config import G_SI, SimConfig
    from gravsim.models import initial_conditions as ic
    from gravsim.ops import oracle
    from gravsim.runtime.engines import HipEngine

    cases = {"clustered_far": clustered(8192), "solar+random": ic.solar_random(8192, 3),
             "plummer": ic.plummer(8192, 3)}
    for name, b in cases.items():
        p = b.pos.astype(np.float32).astype(np.float64)
        mu = (G_SI * b.mass).astype(np.float32).astype(np.float64)
        ref = oracle.accelerations(p, mu, G=1.0)
        nref = np.linalg.norm(ref, axis=1)
        row = {"ics": name, "n": b.n}
        for kernel in ("mfma", "smem"):
            e = HipEngine(SimConfig(n=b.n, dtype="fp32", device="gpu", kernel=kernel))
            e.load(b)
            a = e.accel(step_path=True)[: b.n, :3]
            e.close()
            rel = np.linalg.norm(a - ref, axis=1) / nref
            row[kernel] = {"median_rel": float(np.median(rel)), "p99_rel": float(np.quantile(rel, 0.99)),
                           "max_rel": float(rel.max()),
                           "frob_rel": float(np.linalg.norm(a - ref) / np.linalg.norm(ref))}
        print(json.dumps(row), flush=True)
    for kernel in ("mfma", "smem"):
        e = HipEngine(SimConfig(n=1 << 20, dtype="fp32", device="gpu", kernel=kernel))
        e.init_ics("solar+random", 1)
        e.step(2)
        e.sync()
        t0 = time.perf_counter()
        e.step(4)
        e.sync()
        ms = (time.perf_counter() - t0) / 4 * 1e3
        print(json.dumps({"kernel": kernel, "n": 1 << 20, "ms_per_step": ms,
                          "effective_interactions_per_s": (1 << 20) ** 2 / (ms * 1e-3),
                          "layout": e.native_layout}), flush=True)
        e.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
