"""Per-body error of the sym step path against the fp64 oracle (sizing the smoke / scale gates).
    python scripts/accel_err.py [--n 4096] [--dtype fp32]
Prints one JSON line: max / median per-body relative error |a - a_ref| / |a_ref| and the
worst ratio |a - a_ref| / (eps * sum_j |term_ij|) (the rounding-bound constant needed)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--dtype", default="fp32")
    a = ap.parse_args()
    import gravsim  # noqa: F401
    from gravsim.config import G_SI, SimConfig
    from gravsim.ops import oracle
    from gravsim.runtime.engines import HipEngine

    cfg = SimConfig(n=a.n, dtype=a.dtype, device="gpu", mode="sym").validate()
    eng = HipEngine(cfg, device=0)
    try:
        eng.init_ics("solar+random", cfg.seed)
        b = eng.state()
        got = eng.accel(step_path=True)[: a.n, :3]
    finally:
        eng.close()
    T = np.float32 if a.dtype == "fp32" else np.float64
    p = b.pos.astype(T).astype(np.float64)
    mu = (G_SI * b.mass).astype(T).astype(np.float64)
    ref, _, absref = oracle.accelerations(p, mu, G=1.0, with_potential=True, with_abs=True)
    err = np.linalg.norm(got - ref, axis=1)
    rel = err / np.linalg.norm(ref, axis=1)
    eps = 2.0 ** -24 if a.dtype == "fp32" else 2.0 ** -53
    ratio = (np.abs(got - ref) / (eps * absref + 1e-300)).max()
    print(json.dumps({"n": a.n, "dtype": a.dtype, "rel_max": float(rel.max()),
                      "rel_median": float(np.median(rel)), "rel_p99": float(np.quantile(rel, 0.99)),
                      "bound_ratio_max": float(ratio)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
