"""Where the time of a multi-process RCCL run goes, per rank (one-GPU rehearsal).

    python scripts/rccl_phase_times.py --world 4 --n 20000 [--strategy ring] [--debug]

Spawns `world` ranks on device 0 (one NCCL_HOSTID each: RCCL's socket transport, as
tests/test_rccl_gpu.py) and prints one JSON line per rank with the seconds spent in each
phase: gloo init, engine creation, RCCL communicator init, ICs, the first step, the rest of
the steps, state() (collective), phase-timed steps, close. --debug writes NCCL_DEBUG=INFO
logs to gpurun_out/rccl_dbg/. Used to find why the 4-rank socket runs took 55-118 s.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, steps, strategy, mode, debug):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", GRAVSIM_RCCL_RANK_HOSTS="1")
    if debug:
        d = os.path.join(ROOT, "gpurun_out", "rccl_dbg")
        os.makedirs(d, exist_ok=True)
        os.environ.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,NET,GRAPH,ENV",
                          NCCL_DEBUG_FILE=os.path.join(d, f"w{world}_r{rank}.log"))
    t = [("start", time.perf_counter())]

    def mark(name):
        t.append((name, time.perf_counter()))

    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.parallel import comm
    from gravsim.runtime.engines import HipEngine

    mark("import")
    dist = comm.init(timeout_s=300)
    mark("gloo_init")
    cfg = SimConfig(n=n, dtype="fp32", device="gpu", chunk=1024, step_timeout_s=300,
                    strategy=strategy, mode=mode)
    eng = HipEngine(cfg, rank, world, device=0, dist=dist)
    mark("engine")
    uid = HipEngine.unique_id() if rank == 0 else None
    uid = comm.broadcast_bytes(dist, uid)
    eng.comm_init(uid)
    mark("rccl_init")
    eng.init_ics("solar+random", 5)
    eng.sync(timeout_s=300)
    mark("ics")
    eng.step(1)
    eng.sync(timeout_s=300)
    mark("first_step")
    eng.step(steps - 1)
    eng.sync(timeout_s=300)
    mark("steps")
    eng.state()
    mark("state")
    eng.set_timing(True)
    eng.step(2)
    eng.phase_stats()
    eng.set_timing(False)
    mark("phase_steps")
    eng.close()
    mark("close")
    comm.barrier(dist)
    mark("barrier")
    comm.shutdown(dist)
    mark("shutdown")
    out = {"world": world, "rank": rank, "n": n, "strategy": strategy, "mode": mode}
    out.update({t[i][0]: round(t[i][1] - t[i - 1][1], 3) for i in range(1, len(t))})
    print(json.dumps(out), flush=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--strategy", default="allgather")
    ap.add_argument("--mode", default="sym")
    ap.add_argument("--debug", action="store_true")
    a = ap.parse_args()
    import torch.multiprocessing as mp

    t0 = time.perf_counter()
    mp.start_processes(_worker, args=(a.world, _port(), a.n, a.steps, a.strategy, a.mode,
                                      a.debug),
                       nprocs=a.world, start_method="spawn", join=True)
    print(json.dumps({"world": a.world, "total_s": round(time.perf_counter() - t0, 3)}),
          flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
