"""Per-GPU step time of ONE rank of a P-rank run, measured on one GPU.

Runs rank r's exact launch shapes (sym: gather -> force units -> node reduce -> node-sum
exchange beside the row reduce -> finalize; split: local + remote chunks on two compute
streams -> reduce/integrate) under GRAVSIM_EMULATE_RANK=1. The collectives are either free
(--comm-gbps 0, round 1's emulation) or modeled: a comm_model kernel of the collective's
exact byte count on the comm stream that stays resident for latency + bytes / rate
(csrc/hip/comm_model.hip), so the emulated step pays for an xGMI all-gather and exchange
and shows how much of it the schedule hides. Predicted strong-scaling efficiency =
ms(P=1) / (P * ms(P)). Not physics: remote slices hold stale positions.

    python bench/rank_shape.py --n 1048576 --ranks 1,2,4,8 --comm-gbps 0,64 --overlap 0,3

Since round 3 the sym schedule runs every P up to 8 (uneven row blocks for P not dividing
the 256 blocks): --rank all measures every rank of such a run (rank 0 holds the most blocks).
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--ipl", default="0", help="comma list")
    ap.add_argument("--kernel", default="auto", help="comma list")
    ap.add_argument("--strategy", default="allgather", help="comma list: allgather,ring")
    ap.add_argument("--mode", default="auto", help="comma list: auto,split,sym")
    ap.add_argument("--comm-gbps", default="0",
                    help="comma list of modeled per-rank collective rates in GB/s (0: free)")
    ap.add_argument("--comm-us", type=float, default=15.0, help="modeled latency per collective")
    ap.add_argument("--comm-wgs", type=int, default=16, help="workgroups of a modeled collective")
    ap.add_argument("--overlap", default="3", help="comma list of sym overlap modes (0, 3)")
    ap.add_argument("--graph", default="segmented",
                    help="comma list of multi-rank step modes: eager | segmented (the default: "
                         "compute segments as graphs, collectives eager between them) | full "
                         "(collectives captured too)")
    ap.add_argument("--links", action="store_true",
                    help="price the node-sum exchange per xGMI link (GRAVSIM_EMU_LINKS=1: each "
                         "source peer's bytes at --comm-gbps, peers in parallel) instead of all "
                         "of a rank's bytes through one --comm-gbps pipe")
    ap.add_argument("--rank", default="-1",
                    help="emulated rank: an index, -1 the last, 'all' every rank")
    ap.add_argument("--repeat", type=int, default=1, help="run the whole grid this many times "
                    "(alternating configurations, for A/B on a noisy clock)")
    a = ap.parse_args()
    os.environ["GRAVSIM_EMULATE_RANK"] = "1"
    if a.links:
        os.environ["GRAVSIM_EMU_LINKS"] = "1"
    import torch  # noqa: F401

    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.runtime.engines import HipEngine

    base = {}
    grid = list(itertools.product([int(x) for x in a.ranks.split(",")],
                                  [int(x) for x in a.ipl.split(",")], a.kernel.split(","),
                                  a.strategy.split(","), a.mode.split(","),
                                  [float(x) for x in a.comm_gbps.split(",")],
                                  [int(x) for x in a.overlap.split(",")],
                                  a.graph.split(",")))
    runs = []
    for P, *rest in grid:
        ranks = range(P) if a.rank == "all" else \
            [((int(a.rank) if int(a.rank) >= 0 else P - 1) if P > 1 else 0)]
        runs += [(P, r, *rest) for r in ranks]
    for P, r, ipl, kernel, strategy, mode, gbps, ov, gmode in runs * a.repeat:
        # modeled collectives: "GB/s,latency us,workgroups" (stepper.hip GRAVSIM_EMU_COMM)
        os.environ["GRAVSIM_EMU_COMM"] = f"{gbps},{a.comm_us},{a.comm_wgs}"
        cfg = SimConfig(n=a.n, dtype=a.dtype, device="gpu", ipl=ipl, kernel=kernel,
                        strategy=strategy, mode=mode, graph=gmode != "eager",
                        graph_comm=gmode == "full")
        e = HipEngine(cfg, r, P)
        e.set_overlap(ov)
        e.init_ics("solar+random", cfg.seed)
        e.step(2)
        e.sync()
        e.clock()  # (reset: the engine-clock record of the timed steps only)
        t0 = time.perf_counter()
        e.step(a.steps)
        e.sync()
        ms = 1e3 * (time.perf_counter() - t0) / a.steps
        ghz = e.clock()["ghz"] or None
        phase = None
        if P > 1:
            if e.graph_info()["mode"] == "segmented":
                e.step(2 if e.steps_done % 2 == 0 else 1)  # whole plan periods (bench.py)
            e.set_timing(True)
            e.step(4)
            phase = e.phase_stats()
            e.set_timing(False)
        key = (ipl, kernel, strategy, mode, a.dtype)
        # the step in engine-clock cycles (ms x GHz): a prediction that does not depend on the
        # clock the box held during each run (DVFS; r6_clock_normalised_boxes.txt)
        mcyc = ms * ghz if ghz else None
        if P == 1:
            base[key] = (ms, mcyc)
        b, bc = base.get(key, (None, None))
        print(json.dumps(dict(P=P, rank=r, n=a.n, dtype=a.dtype, ipl=ipl, kernel=kernel,
                              strategy=strategy, mode=e.native_layout["mode"], comm_gbps=gbps,
                              exchange_model="per-link" if a.links else "one pipe",
                              comm_us=a.comm_us, overlap=ov, graph=gmode, graph_info=e.graph_info(),
                              ms_per_step=ms, engine_clock_ghz=ghz, step_mcycles=mcyc,
                              predicted_efficiency=(b / (P * ms)) if b else None,
                              predicted_efficiency_cycles=(bc / (P * mcyc)) if bc and mcyc
                              else None,
                              predicted_body_updates_per_s=a.n / (ms * 1e-3), phase=phase,
                              layout=e.native_layout)), flush=True)
        e.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
