"""Workgroup timeline of one sym force launch: where a step's force time goes beyond the
units' own work (dispatch ramp, the final partial wave, per-XCD imbalance).

The force kernel, built with its probe (SymArgs.utrace) and run with GRAVSIM_UNIT_TRACE=1,
stamps every unit with s_memrealtime (100 MHz) at start and end plus the hardware ids of
the CU that ran it. This script runs one rank of a P-rank sym run on one GPU (the per-rank
emulation of bench/rank_shape.py, collectives free) and reports, per configuration:

  span_ms      first unit start -> last unit end
  busy_frac    sum of unit durations / (resident slots x span): 1.0 is a perfectly packed launch
  ramp_ms      until 90 % of the slots are busy
  tail_ms      from the last moment 90 % of the slots were busy to the end
  shell_ms / diag_ms  median unit durations (shell segment, diagonal part)
  xcd_end_ms   per XCD, when its last unit ended (relative to the launch start)

    python bench/unit_timeline.py --n 1048576 --ranks 1,8
    python bench/unit_timeline.py --n 1048576 --ranks 8 --env GRAVSIM_SYM_OVERLAP=0,3
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TICK_MS = 1e-5  # s_memrealtime runs at 100 MHz


def analyse(tr: np.ndarray, S: int, slots_per_cu: int = 2) -> dict:
    """Summary of one launch's trace rows {start, end, hw ids, row << 32 | segment}."""
    t = tr[tr[:, 0] > 0]
    if len(t) == 0:
        return {"units": 0}
    t0 = t[:, 0].astype(np.int64)
    t1 = t[:, 1].astype(np.int64)
    base = int(t0.min())
    t0 -= base
    t1 -= base
    hw = (t[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    xcc = (t[:, 2] >> np.uint64(32)).astype(np.int64) & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    cus = len(set(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist())))
    seg = (t[:, 3] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    dur = t1 - t0
    span = int(t1.max())
    slots = slots_per_cu * cus
    # active units over time (event sweep)
    ev = np.concatenate([np.stack([t0, np.ones_like(t0)], 1), np.stack([t1, -np.ones_like(t1)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    active = np.cumsum(ev[:, 1])
    hi = active >= 0.9 * slots
    ramp = int(ev[np.argmax(hi), 0]) if hi.any() else span
    tail_start = int(ev[len(hi) - 1 - np.argmax(hi[::-1]), 0]) if hi.any() else 0
    shell = dur[seg < S]
    diag = dur[seg >= S]
    xcd_end = {int(x): round(float(t1[xcc == x].max()) * TICK_MS, 3) for x in sorted(set(xcc.tolist()))}
    # units running at once on one CU (expected: the resident workgroups per CU)
    cu_key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    conc = []
    for k in np.unique(cu_key):
        m = cu_key == k
        e = np.concatenate([np.stack([t0[m], np.ones(m.sum(), np.int64)], 1),
                            np.stack([t1[m], -np.ones(m.sum(), np.int64)], 1)])
        e = e[np.lexsort((e[:, 1], e[:, 0]))]
        conc.append(int(np.cumsum(e[:, 1]).max()))
    return {
        "units": int(len(t)), "cus_seen": cus, "slots": slots,
        "span_ms": round(span * TICK_MS, 3),
        "busy_frac": round(float(dur.sum()) / (slots * span), 4),
        "ramp_ms": round(ramp * TICK_MS, 3),
        "tail_ms": round((span - tail_start) * TICK_MS, 3),
        "shell_ms": round(statistics.median(shell.tolist()) * TICK_MS, 4) if len(shell) else None,
        "shell_p90_ms": round(float(np.percentile(shell, 90)) * TICK_MS, 4) if len(shell) else None,
        "diag_ms": round(statistics.median(diag.tolist()) * TICK_MS, 4) if len(diag) else None,
        "n_shell": int(len(shell)), "n_diag": int(len(diag)),
        "xcd_end_ms": xcd_end,
        "max_units_per_cu": max(conc), "median_max_units_per_cu": float(np.median(conc)),
        "xcd_units": {int(x): int((xcc == x).sum()) for x in sorted(set(xcc.tolist()))},
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--ranks", default="1,8")
    ap.add_argument("--rank", type=int, default=-1, help="emulated rank (default: the last)")
    ap.add_argument("--steps", type=int, default=2, help="steps before the traced one")
    ap.add_argument("--env", action="append", default=[],
                    help="VAR=v1,v2 axis set while the engine is created (repeatable)")
    ap.add_argument("--out", default=None, help="also save the raw traces here (.npz)")
    a = ap.parse_args()
    # (set here, not at import: tests import analyse() and must not inherit these)
    os.environ["GRAVSIM_EMULATE_RANK"] = "1"
    os.environ["GRAVSIM_UNIT_TRACE"] = "1"
    import torch  # noqa: F401

    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.runtime.engines import HipEngine

    axes = [[("P", int(p)) for p in a.ranks.split(",")]]
    for e in a.env:
        k, vs = e.split("=", 1)
        axes.append([(k, v) for v in vs.split(",")])
    raw = {}
    for combo in itertools.product(*axes):
        c = dict(combo)
        P = c.pop("P")
        saved = {k: os.environ.get(k) for k in c}
        os.environ.update(c)
        cfg = SimConfig(n=a.n, dtype=a.dtype, device="gpu", mode="sym")
        r = (a.rank if a.rank >= 0 else P - 1) if P > 1 else 0
        eng = HipEngine(cfg, r, P)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        eng.init_ics("solar+random", cfg.seed)
        eng.step(a.steps)
        eng.sync()
        eng.unit_trace()  # drop the warm-up launches
        eng.step(1)
        eng.sync()
        tr = eng.unit_trace()
        S = _sym_S(eng, a.n)
        res = analyse(tr, S)
        print(json.dumps(dict(n=a.n, dtype=a.dtype, P=P, rank=r, **c, **res)), flush=True)
        raw[f"P{P}_" + "_".join(f"{k}{v}" for k, v in c.items())] = tr
        eng.close()
    if a.out:
        np.savez_compressed(a.out, **raw)
    return 0


def _sym_S(eng, n: int) -> int:
    import ctypes

    from gravsim.ops import _native

    vals = [ctypes.c_int32() for _ in range(5)]  # NC, H, L, S, D
    _native.check(eng.lib, eng.lib.gs_sym_geometry(eng.native_layout["n_pad"],
                                                   *[ctypes.byref(v) for v in vals]), "geometry")
    return vals[3].value


if __name__ == "__main__":
    sys.exit(main())
