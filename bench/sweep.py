"""Kernel/schedule sweep in ONE process (interleaved rounds, §5.4 rule 24 of the HIP guide).

    python bench/sweep.py --n 1048576 --steps 3 --rounds 2 --grid "kernel=lds,smem;ipl=1,2,4;mode=fused,split"
    python bench/sweep.py --n 65536 --grid "mode=sym;env.GRAVSIM_SYM_BAND_MB=1540,0"
Axes named env.<VAR> set that environment variable while the engine is created (the native
stepper reads its A/B knobs at creation). Prints one JSON line per (config, round) and a
summary sorted by median ms/step.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--grid", default="kernel=lds,smem;ipl=1,2,4;mode=fused,split")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch  # noqa: F401

    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.runtime.engines import HipEngine

    axes = []
    for part in a.grid.split(";"):
        k, vs = part.split("=")
        conv = int if k in ("ipl", "chunk", "split_groups") else str
        axes.append([(k, conv(v)) for v in vs.split(",")])
    combos = [dict(c) for c in itertools.product(*axes)]
    engines = []
    for c in combos:
        env = {k[4:]: v for k, v in c.items() if k.startswith("env.")}
        kw = {k: v for k, v in c.items() if not k.startswith("env.")}
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        cfg = SimConfig(n=a.n, dtype=a.dtype, device="gpu", **kw)
        e = HipEngine(cfg)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        e.init_ics("solar+random", cfg.seed)
        e.step(1)
        e.sync()
        engines.append(e)
    res = {i: [] for i in range(len(combos))}
    out = open(a.out, "a") if a.out else None
    for r in range(a.rounds):
        for i, (c, e) in enumerate(zip(combos, engines)):
            e.sync()
            t0 = time.perf_counter()
            e.step(a.steps)
            e.sync()
            ms = 1e3 * (time.perf_counter() - t0) / a.steps
            res[i].append(ms)
            line = json.dumps(dict(round=r, n=a.n, dtype=a.dtype, ms=ms,
                                   inter_per_s=a.n * a.n / (ms * 1e-3), layout=e.native_layout, **c))
            print(line, flush=True)
            if out:
                out.write(line + "\n")
    print("== summary (median ms/step)")
    for i in sorted(res, key=lambda i: statistics.median(res[i])):
        m = statistics.median(res[i])
        print(f"{m:10.3f} ms  {a.n * a.n / (m * 1e-3):.3e} int/s  {combos[i]}  "
              f"mode={engines[i].native_layout['mode']} groups={engines[i].native_layout['split_groups']}")
    for e in engines:
        e.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
