"""Where the KD energy drift of the benchmark run comes from.

bench.py reports energy_rel_drift ~0.88 over its 25 steps at N = 1M (fp32, dt = 3600 s) and
attributes it to close passages that the first-order kick-drift step (mpi.c:206-215) cannot
resolve. This script checks that claim on the GPU:

1. the same ICs (bench.py's seed) are stepped `--steps` times in fp32 AND fp64; the relative
   drift of the total energy (kinetic + exact-cutoff potential) must agree between the two if
   it is physics of the integrator rather than rounding or a kernel bug that bites only in
   one precision;
2. per-body energies e_i = m_i v_i^2 / 2 + m_i phi_i / 2 (they sum to E) before and after:
   the bodies with the largest |de_i| and the share of the net dE they carry;
3. those bodies are re-stepped one step at a time from the ICs: their nearest neighbour
   distance at every step against |v| dt, the distance they move in one step (a close
   encounter the step cannot resolve has d_min << |v| dt).

    python scripts/energy_drift.py --n 1048576 --steps 25 --json profiles/r4_energy_drift_1m.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def per_body_energy(eng, G: float) -> tuple[np.ndarray, np.ndarray]:
    """(e_i, phi_i) of every body (one rank): m v^2 / 2 + m phi / 2 with the exact-cutoff
    potential of the engine's diagnostic force pass."""
    b = eng.state()
    a4 = eng.accel()[: len(b.mass)]
    m = b.mass
    return 0.5 * m * (b.vel * b.vel).sum(1) + 0.5 * m * a4[:, 3], a4[:, 3]


def nearest(pos: np.ndarray, idx: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Distance to, and index of, the nearest other body for bodies idx (exact, O(k N))."""
    d = np.empty(len(idx))
    j = np.empty(len(idx), dtype=np.int64)
    for k, i in enumerate(idx):
        r = np.linalg.norm(pos - pos[i], axis=1)
        r[i] = np.inf
        j[k] = int(np.argmin(r))
        d[k] = r[j[k]]
    return d, j


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--dt", type=float, default=3600.0)
    ap.add_argument("--dtypes", default="fp32,fp64")
    ap.add_argument("--top", type=int, default=16, help="bodies traced step by step")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.runtime.engines import HipEngine

    out = {"n": a.n, "steps": a.steps, "dt": a.dt, "runs": {}}
    de_ref = None
    for dt_name in a.dtypes.split(","):
        cfg = SimConfig(n=a.n, dtype=dt_name, device="gpu", dt=a.dt).validate()
        eng = HipEngine(cfg, device=0)
        t0 = time.time()
        eng.init_ics("solar+random", cfg.seed)
        e0, _ = per_body_energy(eng, cfg.G)
        eng.step(a.steps)
        eng.sync()
        e1, _ = per_body_energy(eng, cfg.G)
        b1 = eng.state()
        eng.close()
        E0, E1 = float(e0.sum()), float(e1.sum())
        de = e1 - e0
        order = np.argsort(-np.abs(de))
        cum = np.cumsum(de[order])
        dE = E1 - E0
        # fewest bodies whose summed de reaches 90 % of the net dE
        k90 = int(np.argmax(np.abs(cum) >= 0.9 * abs(dE))) + 1 if dE != 0 else 0
        run = {"energy_start": E0, "energy_end": E1, "energy_rel_drift": abs(dE) / abs(E0),
               "net_dE": dE, "sum_abs_de": float(np.abs(de).sum()),
               "bodies_for_90pct_of_dE": k90,
               "top_bodies": [{"body": int(i), "de": float(de[i]),
                               "share_of_dE": float(de[i] / dE) if dE else None,
                               "mass": float(b1.mass[i])} for i in order[:a.top]],
               "wall_s": round(time.time() - t0, 1)}
        out["runs"][dt_name] = run
        if de_ref is None:
            de_ref = (order[:a.top].copy(), dt_name)
        print(json.dumps({k: v for k, v in run.items() if k != "top_bodies"}), flush=True)

    # step-by-step trace of the fp32 run's top bodies (and the fp64 run's, if different)
    top = np.unique(np.concatenate([np.array([t["body"] for t in r["top_bodies"]])
                                    for r in out["runs"].values()]))
    cfg = SimConfig(n=a.n, dtype=a.dtypes.split(",")[0], device="gpu", dt=a.dt).validate()
    eng = HipEngine(cfg, device=0)
    eng.init_ics("solar+random", cfg.seed)
    trace = {int(i): {"d_min": np.inf, "step_of_d_min": -1, "partner": -1,
                      "v_dt_at_d_min": None} for i in top}
    for s in range(a.steps + 1):
        b = eng.state()
        d, j = nearest(b.pos, top)
        speed = np.linalg.norm(b.vel[top], axis=1)
        for k, i in enumerate(top):
            t = trace[int(i)]
            if d[k] < t["d_min"]:
                t.update(d_min=float(d[k]), step_of_d_min=s, partner=int(j[k]),
                         v_dt_at_d_min=float(speed[k] * a.dt))
        if s < a.steps:
            eng.step(1)
            eng.sync()
    eng.close()
    for i, t in trace.items():
        t["d_min_over_v_dt"] = t["d_min"] / t["v_dt_at_d_min"] if t["v_dt_at_d_min"] else None
    out["trace"] = trace
    r32 = out["runs"].get("fp32")
    r64 = out["runs"].get("fp64")
    if r32 and r64:
        out["fp32_vs_fp64_drift_ratio"] = r32["energy_rel_drift"] / r64["energy_rel_drift"]
        shared = {t["body"] for t in r32["top_bodies"][:8]} & {t["body"] for t in r64["top_bodies"][:8]}
        out["top8_bodies_shared"] = sorted(shared)
    close = [t for t in trace.values() if t["d_min_over_v_dt"] is not None]
    out["summary"] = {
        "traced": len(close),
        "median_d_min_over_v_dt": float(np.median([t["d_min_over_v_dt"] for t in close]))
        if close else None,
        "partners": sorted({t["partner"] for t in close})}
    print(json.dumps({k: v for k, v in out.items() if k not in ("runs", "trace")}), flush=True)
    if a.json:
        os.makedirs(os.path.dirname(os.path.abspath(a.json)), exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1, default=float)
    return 0


if __name__ == "__main__":
    sys.exit(main())
