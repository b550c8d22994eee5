"""Per-GPU step time of ONE rank of a P-rank run, measured on one GPU.

Runs rank r's exact launch shapes (local chunks + remote chunks on two compute streams +
reduce/integrate) with the all-gather treated as done (GRAVSIM_EMULATE_RANK=1), so
ms/step ~ what each GPU of a P-GPU node spends on compute per step; the RCCL all-gather is
overlapped with the local chunks in the real run. Predicted strong-scaling efficiency =
ms(P=1) / (P * ms(P)).  Not physics: remote slices hold stale positions.
    python bench/rank_shape.py --n 1048576 --ranks 1,2,4,8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["GRAVSIM_EMULATE_RANK"] = "1"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--ipl", default="0", help="comma list")
    ap.add_argument("--kernel", default="auto", help="comma list")
    ap.add_argument("--strategy", default="allgather", help="comma list: allgather,ring")
    ap.add_argument("--mode", default="auto", help="comma list: auto,split,sym")
    a = ap.parse_args()
    import torch  # noqa: F401

    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.runtime.engines import HipEngine

    base = None
    import itertools

    grid = list(itertools.product([int(x) for x in a.ranks.split(",")],
                                  [int(x) for x in a.ipl.split(",")], a.kernel.split(","),
                                  a.strategy.split(","), a.mode.split(",")))
    for P, ipl, kernel, strategy, mode in grid:
        cfg = SimConfig(n=a.n, dtype=a.dtype, device="gpu", ipl=ipl, kernel=kernel,
                        strategy=strategy, mode=mode)
        r = P - 1 if P > 1 else 0  # a rank with its own chunks at the end
        e = HipEngine(cfg, r, P)
        e.init_ics("solar+random", cfg.seed)
        e.step(2)
        e.sync()
        t0 = time.perf_counter()
        e.step(a.steps)
        e.sync()
        ms = 1e3 * (time.perf_counter() - t0) / a.steps
        base = base or ms * P
        print(json.dumps(dict(P=P, rank=r, n=a.n, dtype=a.dtype, ipl=ipl, kernel=kernel,
                              strategy=strategy, mode=e.native_layout["mode"], ms_per_step=ms,
                              predicted_efficiency=base / (P * ms),
                              predicted_body_updates_per_s=a.n / (ms * 1e-3),
                              layout=e.native_layout)), flush=True)
        e.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
