"""Schedule-overhead probe: P virtual ranks on ONE GPU (gs_group_step).

The total interaction count is the same for every P, so ms/step(P) / ms/step(1) - 1 is
the cost of the multi-rank schedule itself (per-rank launch shapes, local/remote overlap on
two compute streams, the exchange as device copies) — what the 8-GPU run pays on top of
the RCCL all-gather over xGMI.
    python bench/virtual_scaling.py --n 1048576 --ranks 1,2,4,8 --steps 3
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--dtype", default="fp32")
    a = ap.parse_args()
    import torch  # noqa: F401

    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.runtime.engines import VirtualGroup

    base = None
    for P in [int(x) for x in a.ranks.split(",")]:
        cfg = SimConfig(n=a.n, dtype=a.dtype, device="gpu")
        g = VirtualGroup(cfg, P)
        g.init_ics("solar+random", cfg.seed)
        g.step(2)
        g.sync()
        t0 = time.perf_counter()
        g.step(a.steps)
        g.sync()
        ms = 1e3 * (time.perf_counter() - t0) / a.steps
        base = base or ms
        lay = g.shards[0].native_layout
        print(json.dumps(dict(P=P, n=a.n, ms_per_step=ms, overhead_vs_P1=ms / base - 1,
                              ipl=lay["ipl"], mode=lay["mode"], n_local=lay["n_local"])),
              flush=True)
        g.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
