"""Headline benchmark: body-updates/s of the direct O(N^2) N-body step at N = 1,048,576 (fp32).

BASELINE.json metric: "body-updates/sec (whole node) at N=1M direct O(N^2), 1/2/4/8 MI355X"
(config "1,048,576 bodies fp32 on 8xMI355X, RCCL all-gather ring over xGMI each step").
N is fixed as the GPU count grows (strong scaling). The default (mode auto) at this size is
the Newton-3 schedule: every unordered pair is evaluated once and applied to both bodies
(csrc/hip/nbody_sym.hip). Each rank owns N/P bodies (a block of 2048-body chunk rows), joins
an in-place RCCL all-gather of positions, evaluates its rows' cyclic half-shell of chunk
pairs, exchanges its reduction-tree node sums of the far sides with ncclSend/ncclRecv, and
integrates its own bodies (kick-drift). Single-rank steps replay a hipGraph; multi-rank steps
replay a segmented plan: the compute work between two collectives as graph segments, the RCCL
calls issued eagerly between them (--graph-comm captures the collectives too, opt-in).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n BODIES] [--dtype fp32|fp64]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Run without a launcher, `--gpus N > 1` starts N ranks itself: a child torch.distributed.run
on 127.0.0.1 (parallel/launch.py; the reference's `mpirun -np P`, mpi.c:140-144), before
anything touches the GPU. Under a launcher, WORLD_SIZE must equal --gpus.

A step is the full simulation step: all-gather + force + exchange + integrate (no work
skipped). Data: synthetic Sun/Earth/Mars + uniform random bodies generated on device
(seeded). Rank 0 prints ONE JSON line; value is the whole-job body-updates/s =
N * K / max_rank(wall).

Audits of the timed work (outside the timed region; the run exits non-zero if one fails):
  * unit count: the sym force kernels count every unit they run on device; after the loop
    each rank must have run exactly rows x (S + D + (Np - 1) Kr) units per timed step (a split
    segment counts as its Np parts);
  * replay: the same warmup + K steps are re-run from the same ICs on an independent
    schedule (eager launches, one static unit per workgroup, ungated) and must give the
    same bits on every rank.
If the gated local-first launch (--overlap auto picked 3 after its 2-step self-check) fails
them, that is a failure of the multi-rank default: the ungated schedule is timed from the same
ICs (config.overlap_fallback), but work_audit reports the failure and the run exits 1.
Also outside it: the sampled accuracy of the step's own accelerations at step 0 and after
the last timed step, the relative drift of total momentum over the run, the drift of total
energy (kinetic + exact-cutoff potential) and angular momentum (two O(N^2) passes), a few
steps with phase events for the comm split (multi-rank: replayed from the same segmented plan
as the timed loop), and the reference's exact hard-cutoff select timed on its own
(exact_cutoff_ms_per_step). Multi-rank runs record per rank the device it bound, what RCCL formed
(ncclCommCount / UserRank / CuDevice) and the RCCL transports its connections used (parsed from
RCCL's INFO log, sent to a file), and refuse to report a number (error line, exit 70) when two
ranks share a GPU, the communicator is not the job, or a single-node connection runs through a
network transport (parallel/verify.py; recorded but not enforced in the one-GPU rehearsal,
GRAVSIM_RCCL_RANK_HOSTS=1). After the timed run they also check P-independence: rank 0 recomputes
2 steps from the same ICs as a 1-rank engine on its own GPU and every rank's rows must be bitwise
equal (--p-audit).

Clock-normalised cost: every force workgroup of the timed steps records its s_memtime (shader
clock) and s_memrealtime (100 MHz) spans; the line reports engine_clock_ghz and
cycles_per_pair_eval (step wall x clock x CUs / pair evaluations), so a slow box and a slow kernel
no longer look alike (profiles/r6_clock_normalised_boxes.txt).

Bounded and self-reporting (gravsim/parallel/guard.py): every stage (gloo init, device,
engine, RCCL init + warm-up, first step, overlap check, warmup, timed, audits, ...) has a
deadline (--init-timeout for start-up; afterwards derived from the first measured step), and
the native step timeout is max(60 s, 20 x the first step), at most 240 s. A stall or a failure
on any rank ends the job within that budget with ONE error JSON line from rank 0 ("status":
"error", the stage reached, each rank's stage, device, RCCL transports and communicator init
stage, HSA_ENABLE_IPC_MODE_LEGACY) and exit code 70, after aborting the RCCL communicator.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "body-updates/sec (whole node) at N=1M direct O(N^2), 1/2/4/8 MI355X"


def parse(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    # (under torch.distributed.run spell it --num-bodies: torchrun's parser takes --n as an
    # ambiguous prefix of its own --nnodes/--nproc-per-node even after the script name)
    ap.add_argument("--n", "--num-bodies", dest="n", type=int, default=1 << 20)
    ap.add_argument("--dtype", choices=["fp32", "fp64"], default="fp32")
    ap.add_argument("--kernel", default="auto", choices=["auto", "lds", "smem", "mfma"])
    ap.add_argument("--mode", default="auto", choices=["auto", "fused", "split", "sym"])
    ap.add_argument("--ipl", type=int, default=0)
    ap.add_argument("--no-graph", dest="graph", action="store_false")
    ap.add_argument("--graph-comm", dest="graph_comm", action="store_true",
                    help="capture multi-rank steps, RCCL collectives included, in a hipGraph")
    ap.add_argument("--no-graph-comm", dest="graph_comm", action="store_false",
                    help=argparse.SUPPRESS)
    ap.add_argument("--overlap", default="auto", choices=["auto", "0", "3"],
                    help="sym work beside the all-gather. auto (multi-rank sym): the gated "
                         "local-first launch (3) if a 2-step self-check from the same ICs "
                         "gives the same bits as the ungated schedule (0), else 0")
    ap.add_argument("--dt", type=float, default=3600.0)
    ap.add_argument("--cutoff-mode", default="auto", choices=["auto", "exact", "fast"])
    ap.add_argument("--strategy", default="allgather", choices=["allgather", "ring"],
                    help="multi-rank exchange: in-place all-gather or pipelined ring pass")
    ap.add_argument("--check-samples", type=int, default=256,
                    help="bodies whose step-0 accelerations are checked against an fp64 row "
                         "sum on the host (0 = skip)")
    ap.add_argument("--phase-steps", type=int, default=4,
                    help="steps with phase events after the timed loop (the comm split), on "
                         "the timed loop's schedule (multi-rank: the segmented plan)")
    ap.add_argument("--no-replay-audit", dest="replay_audit", action="store_false",
                    help="skip the independent-schedule re-run of the timed steps")
    ap.add_argument("--no-energy", dest="energy", action="store_false",
                    help="skip the conserved-quantity passes (total energy with the exact-cutoff "
                         "potential, momenta) before the warmup and after the timed steps")
    ap.add_argument("--exact-steps", type=int, default=10,
                    help="steps timed with the reference's exact cutoff after the headline, on "
                         "the headline's schedule (graph / segmented-plan replay; 0 = skip)")
    ap.add_argument("--init-timeout", type=float, default=180.0,
                    help="seconds each start-up stage (gloo, device, engine, RCCL init and "
                         "warm-up, the first step) may take before the run is stopped with an "
                         "error JSON line")
    ap.add_argument("--step-timeout", type=float, default=0.0,
                    help="native progress bound: abort RCCL and stop with an error JSON line "
                         "when no step completes for this long (0: max(--step-timeout-min, "
                         "20 x the first measured step), at most 240 s)")
    ap.add_argument("--step-timeout-min", type=float, default=60.0,
                    help="floor of the derived step timeout")
    ap.add_argument("--p-audit", default="auto", choices=["auto", "on", "off"],
                    help="P > 1: after the timed run, rank 0 recomputes 2 steps from the same "
                         "ICs as a 1-rank engine on its own GPU and every rank's rows must have "
                         "the same bits (auto: up to 4M bodies fp32, 1M fp64)")
    return ap.parse_args(argv)


def rccl_log_setup(directory: str, rank: int) -> str | None:
    """Route RCCL's INFO log to a per-rank file in the job's guard directory (before any RCCL
    call; stdout stays rank 0's JSON line), so the transport each connection used can be
    reported, by this rank after init and by rank 0's guard if the run stalls. A level the
    user set (NCCL_DEBUG=WARN...) is raised to INFO for the file; its WARN lines are echoed to
    stderr afterwards. Left alone when the user already chose a log file."""
    if "NCCL_DEBUG_FILE" in os.environ:
        return None
    os.environ["GRAVSIM_USER_NCCL_DEBUG"] = os.environ.get("NCCL_DEBUG", "")
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ["NCCL_DEBUG_SUBSYS"] = "INIT,P2P,NET"
    os.environ["NCCL_DEBUG_FILE"] = os.path.join(directory, f"rccl.{rank}.log")
    return os.environ["NCCL_DEBUG_FILE"]


def rccl_transports(path: str | None) -> dict:
    """Transports of this rank's RCCL connections ("Channel .. via P2P/IPC", "NET/Socket",
    "SHM"...) and the RCCL version, from the INFO log; its WARN lines go to stderr."""
    from gravsim.parallel.guard import parse_rccl_log

    if not path:
        return {"transports": None, "rccl_version": None, "net": None,
                "rccl_log": "NCCL_DEBUG_FILE set by the user: not parsed"}
    if os.path.exists(path):
        with open(path, errors="replace") as f:
            for line in f:
                if " WARN " in line:
                    sys.stderr.write(line)
    return parse_rccl_log(path)


def device_record(dev: int) -> dict:
    import socket

    import torch

    p = torch.cuda.get_device_properties(dev)
    return {"device": dev, "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
            "arch": p.gcnArchName, "cus": p.multi_processor_count, "host": socket.gethostname()}


def p_independence_audit(eng, cfg, dist, comm, dev: int, steps: int = 2) -> str:
    """Untimed: the P-rank engine steps `steps` times from the benchmark ICs; rank 0 runs the
    same steps as a 1-rank engine on its own GPU, and every rank's own rows (positions and
    velocities) must hash equal to the same rows of the 1-rank state. The canonical
    decomposition makes the bits independent of P (the reference's mpi.c is not: SURVEY.md
    §2.7 D6). Collective; returns "bitwise" or the ranks that differ."""
    import hashlib

    from gravsim.runtime.engines import HipEngine

    def sha(x) -> str:
        return hashlib.sha256(x.tobytes()).hexdigest()[:24]

    eng.init_ics("solar+random", cfg.seed)
    eng.step(steps)
    eng.sync()
    pos, vel, _ = own_state(eng)
    rows = eng.layout.real_local
    mine = (rows.start, rows.stop, sha(pos), sha(vel))
    recs = comm.allgather_object(dist, mine)
    verdict = ""
    if dist.rank == 0:
        # (the schedule the P-rank engine resolved, so "auto" cannot pick another one for P = 1)
        import dataclasses

        from gravsim.ops import _native

        one_cfg = dataclasses.replace(cfg, mode=_native.MODE_NAMES[eng.native_layout["mode"]])
        one = HipEngine(one_cfg, 0, 1, device=dev)
        try:
            one.init_ics("solar+random", cfg.seed)
            one.step(steps)
            one.sync()
            b = one.state()
        finally:
            one.close()
        bad = [q for q, (r0, r1, hp, hv) in enumerate(recs)
               if sha(b.pos[r0:r1]) != hp or sha(b.vel[r0:r1]) != hv]
        verdict = "bitwise" if not bad else f"differs from 1 rank on rank(s) {bad}"
    return comm.allgather_object(dist, verdict)[0]


def own_state(eng):
    """(positions, velocities) of this rank's real bodies (collective for P > 1)."""
    b = eng.state()
    own = eng.layout.real_local
    return b.pos[own.start:own.stop].copy(), b.vel[own.start:own.stop].copy(), \
        b.mass[own.start:own.stop].copy()


def momentum(dist, comm, vel, mass):
    """(total momentum vector, sum of m |v|) over all ranks' own bodies."""
    import numpy as np

    p = (mass[:, None] * vel).sum(axis=0)
    scale = float((mass * np.linalg.norm(vel, axis=1)).sum())
    return np.array([comm.allreduce_sum(dist, float(x)) for x in p]), \
        comm.allreduce_sum(dist, scale)


# Rounding bound of the sampled accuracy gate: |a_gpu - a_ref| <= ACC_BOUND_C * eps_dtype *
# sum_j |term_ij| per body and component (the small-N kernel tests use the same form,
# tests/test_gpu_kernels.py assert_close_sum).
ACC_BOUND_C = 128.0


def sampled_error(eng, cfg, samples: int, seed: int = 7) -> tuple[float, float]:
    """(max relative error, max bound ratio) over sampled own bodies: |a_gpu - a_ref| / |a_ref|
    and |a_gpu - a_ref| / (eps * sum_j |term_ij|) per component, where a_gpu is the step's own
    force path (sym kernels, configured cutoff mode) and a_ref, sum |term| a row sum over all N
    bodies by the native CPU engine (fp64 for an fp32 run, long double for an fp64 run; 4
    blocks of samples/4 contiguous rows). The bound ratio must stay <= ACC_BOUND_C, for either
    dtype. Collective."""
    import numpy as np

    from gravsim.ops import _native

    a_gpu = eng.accel(step_path=True)  # (n_local, 4), collective for P > 1
    st = eng.state()  # full positions (collective)
    L = eng.layout
    real = max(0, min(L.n_local, cfg.n - L.local_begin))
    if samples <= 0 or real == 0:
        return 0.0, 0.0
    rng = np.random.default_rng(seed + eng.rank)
    blk = max(1, min(samples // 4, real))
    starts = sorted(set(int(x) for x in rng.integers(0, real - blk + 1, size=4)))
    mu = cfg.G * st.mass
    X = np.zeros((cfg.n, 4))
    X[:, :3] = st.pos  # (the device positions, exactly)
    X[:, 3] = mu.astype(np.float32) if cfg.dtype == "fp32" else mu  # mu as the kernel sees it
    lib = _native.cpu_lib()
    eps = 2.0 ** -24 if cfg.dtype == "fp32" else 2.0 ** -53
    # the reference: an fp64 row sum for fp32 runs, a long-double one for fp64 runs (an fp64
    # sum's own rounding is of the fp64 kernel's order)
    ref_fn = lib.gs_cpu_accel_abs_f64 if cfg.dtype == "fp32" else lib.gs_cpu_accel_abs_ld
    worst, ratio = 0.0, 0.0
    eps2 = cfg.softening ** 2  # the intended physics: hard cutoff, no core
    for s0 in starts:
        g0 = L.local_begin + s0
        out = np.zeros((blk, 8))
        _native.check(lib, ref_fn(_native.dptr(X), cfg.n, g0, g0 + blk, cfg.cutoff ** 2, eps2,
                                  _native.dptr(out)), "cpu accel abs")
        ref, absref = out[:, :3], out[:, 4:7]
        got = a_gpu[s0:s0 + blk, :3]
        err = np.linalg.norm(got - ref, axis=1) / np.maximum(np.linalg.norm(ref, axis=1), 1e-300)
        worst = max(worst, float(err.max()))
        ratio = max(ratio, float((np.abs(got - ref) / (eps * absref + 1e-300)).max()))
    return worst, ratio


def overlap_self_check(eng, cfg, dist, comm, steps: int = 2):
    """The gated local-first launch (overlap 3) against the ungated schedule (0): same bits
    from the benchmark ICs on every rank after `steps` steps, then the faster of the two in an
    alternating race (runtime/selfcheck.py). Untimed. Returns (mode, verdict)."""
    from gravsim.runtime.selfcheck import gated_self_check

    race = 3 if cfg.n <= (4 << 20) else 1
    mode, verdict, _ = gated_self_check(eng, dist, comm,
                                        lambda: eng.init_ics("solar+random", cfg.seed),
                                        steps=steps, race=race)
    return mode, verdict


def clock_summary(ghz_sum: float, ghz_min: float, ghz_max: float, wg_cycles: float,
                  wall: float, cus: float, pair_evals: float, world: int) -> dict:
    """Clock-normalised cost of the timed steps (a slow box and a slow kernel look
    alike in ms): the engine clock the force launches ran at (per workgroup s_memtime span /
    s_memrealtime span, duration-weighted; mean over ranks), the CU-cycles per pair evaluation
    of the whole step at that clock, and the force kernels' own workgroup-cycles per pair (no
    clock in it at all). None where the schedule keeps no clock record (one-sided kernels)."""
    ghz = ghz_sum / world if ghz_sum > 0 else None
    return {"engine_clock_ghz": ghz,
            "engine_clock_ghz_ranks": [ghz_min, ghz_max] if world > 1 and ghz else None,
            "cycles_per_pair_eval": wall * ghz * 1e9 * cus / pair_evals if ghz else None,
            "force_wg_cycles_per_pair_eval": wg_cycles / pair_evals if wg_cycles else None,
            "cus": int(cus),
            "method": "per workgroup: s_memtime span / s_memrealtime span x 100 MHz, "
                      "duration-weighted over the timed steps' force launches; "
                      "cycles_per_pair_eval = step wall x clock x CUs / pair evals"}


def launch_info() -> dict:
    from gravsim.parallel import launch

    return {"probe_devices": int(os.environ[launch.PROBE_ENV])
            if os.environ.get(launch.PROBE_ENV) else None,
            "rehearsal_rank_hosts": os.environ.get("GRAVSIM_RCCL_RANK_HOSTS") == "1",
            "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")}


DATA = "synthetic: seeded Sun/Earth/Mars + uniform random bodies (device RNG)"
MODEL = "direct-sum N-body, KD (symplectic Euler) integrator, cutoff 1e-10 m"


def error_line(a, world: int, reason: str, records: list) -> dict:
    """Rank 0's JSON line when the run is stopped (parallel/guard.py): the metric line with no
    value, "status": "error", the stage reached and every rank's record (stage, seconds in it,
    device, RCCL transports so far, the native communicator's init stage, error)."""
    return {"metric": METRIC, "value": None, "unit": "body-updates/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": None, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": a.dtype, "data": DATA,
            "status": "error", "error": reason,
            "stage": records[0].get("stage") if records else None, "work_audit": "not run",
            "config": {"model": MODEL, "n_bodies": a.n, "global_batch": a.n, "seq_len": 1,
                       "dt": a.dt, "ranks": records, "launch": launch_info()}}



def check_topology(world: int, ranks_info: list, env, note=None) -> dict:
    """What RCCL formed and what it runs over (parallel/verify.py): one GPU per rank, the whole
    job in one communicator, no network transport inside one node. Returns the record for the
    JSON line; raises SystemExit (the guard turns it into the error line, exit 70) when a
    problem is found, except in the one-GPU rehearsal, which shares device 0 over sockets by
    design (recorded, not enforced)."""
    from gravsim.parallel import verify

    problems = verify.topology_problems(world, ranks_info)
    topology = {"enforced": not verify.rehearsal(env), "problems": problems,
                **verify.transport_summary(ranks_info)}
    if note:
        note(topology)
    if problems and topology["enforced"]:
        raise SystemExit("multi-GPU topology check failed: " + "; ".join(problems))
    return topology

def main(argv=None) -> int:
    raw = list(sys.argv[1:] if argv is None else argv)
    a = parse(raw)
    world_env = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if world_env == 0 and a.gpus > 1:
        # No launcher: start the ranks ourselves (child process; nothing touched the GPU).
        from gravsim.parallel import launch

        launch.check_device_count(a.gpus)
        return launch.spawn(a.gpus, [os.path.join(ROOT, "bench.py")], raw, keep_gpus=True)
    if world_env and world_env != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE {world_env}: run one rank per GPU "
                         "(torch.distributed.run --nproc-per-node must equal --gpus)")

    import gravsim  # noqa: F401
    from gravsim.parallel import guard as gd

    world = max(1, world_env)
    # Every stage of the run has a deadline; a stall or a failure on any rank ends the job
    # with rank 0's error JSON line instead of an external kill with no record.
    g = gd.RunGuard(int(os.environ.get("RANK", "0") or 0), world,
                    lambda reason, recs: error_line(a, world, reason, recs))
    try:
        rc = run(a, g)
    except (Exception, SystemExit) as e:  # noqa: BLE001 - every failure becomes a report
        if isinstance(e, SystemExit) and e.code in (0, None):
            raise
        g.fail(f"{type(e).__name__}: {e}")
    g.close()
    return rc


def run(a, g) -> int:
    import numpy as np
    import torch

    from gravsim.config import SimConfig
    from gravsim.ops import _native
    from gravsim.parallel import comm
    from gravsim.parallel import guard as gd
    from gravsim.runtime.engines import HipEngine
    from gravsim.runtime.simulation import conservation_summary, engine_conserved

    init_b = a.init_timeout
    g.stage("gloo_init", init_b)
    dist = comm.init(timeout_s=max(init_b, 120.0))
    world, rank = dist.world, dist.rank
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but the job has {world} rank(s)")
    g.stage("device", init_b)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device (MI355X)")
    ndev = torch.cuda.device_count()
    if world > ndev and os.environ.get("GRAVSIM_RCCL_RANK_HOSTS") != "1":
        raise SystemExit(f"{world} ranks but {ndev} visible GPU(s)")
    dev = dist.local_rank % ndev
    torch.cuda.set_device(dev)
    g.note(**device_record(dev))

    cfg = SimConfig(n=a.n, dt=a.dt, dtype=a.dtype, device="gpu", kernel=a.kernel, mode=a.mode,
                    ipl=a.ipl, graph=a.graph, graph_comm=a.graph_comm,
                    cutoff_mode=a.cutoff_mode, strategy=a.strategy,
                    step_timeout_s=init_b).validate()
    rccl_log = rccl_log_setup(g.dir, rank) if world > 1 else None  # before the first RCCL call
    g.note(rccl_log_path=rccl_log)
    g.stage("engine", init_b)
    eng = HipEngine(cfg, rank, world, device=dev, dist=dist)
    g.on_abort(eng.abort)
    g.probe(lambda: {"comm_stage": eng.comm_stage()})
    ranks_info = topology = None
    if world > 1:
        g.stage("rccl_uid", init_b)
        uid = HipEngine.unique_id() if rank == 0 else None
        uid = comm.broadcast_bytes(dist, uid)
        g.stage("comm_init", init_b)  # ncclCommInitRank + warm-up of every connection
        eng.comm_init(uid)
        g.stage("rank_info", init_b)
        rec = {"rank": rank, **device_record(dev), **eng.comm_info(),
               **rccl_transports(rccl_log)}
        ranks_info = comm.allgather_object(dist, rec)
        topology = check_topology(world, ranks_info, os.environ, note=lambda t: g.note(topology=t))

    # One eager step from the ICs: its time bounds every later stage, and the native step
    # timeout becomes max(60 s, 20 x step), at most 240 s (a 16M / 8-rank step is ~5 s).
    g.stage("first_step", init_b)
    eng.init_ics("solar+random", cfg.seed)
    eng.sync()
    comm.barrier(dist)
    t0 = time.perf_counter()
    eng.step(1)
    eng.sync()
    first_s = comm.allreduce_max(dist, time.perf_counter() - t0)
    step_to = a.step_timeout or gd.step_timeout(first_s, floor_s=a.step_timeout_min)
    eng.set_step_timeout(step_to)
    g.note(first_step_s=round(first_s, 4), step_timeout_s=step_to)

    def budget(steps: float, host_s: float = 60.0) -> float:
        """Deadline of a stage that runs `steps` steps plus host work."""
        return step_to + 4.0 * first_s * steps + host_s

    sym = _native.MODE_NAMES.get(eng.native_layout["mode"]) == "sym"
    overlap, overlap_check = (0, None)
    if a.overlap != "auto":
        overlap = int(a.overlap)
    elif world > 1 and sym:
        g.stage("overlap_check", budget(4 + 4 * 4))
        overlap, overlap_check = overlap_self_check(eng, cfg, dist, comm)
    eng.set_overlap(overlap)
    g.stage("ics", budget(0))
    eng.init_ics("solar+random", cfg.seed)
    eng.sync()

    # Accuracy of the step's own force path at step 0, and the initial momentum (untimed).
    g.stage("accuracy", budget(2, 180))
    err = bound0 = None
    if a.check_samples > 0:
        err, bound0 = (comm.allreduce_max(dist, x) for x in sampled_error(eng, cfg,
                                                                           a.check_samples))
    _, vel0, mass = own_state(eng)
    p0, pscale = momentum(dist, comm, vel0, mass)
    g.stage("energy", budget(4, 180))
    cons0 = engine_conserved(eng, dist) if a.energy else None  # exact-cutoff potential pass

    def measure(overlap: int) -> dict:
        """Warmup + the K timed steps from the ICs already loaded, then the audits of that
        work and the end-of-run physics (all untimed)."""
        g.stage("warmup", budget(a.warmup + 2))
        eng.step(a.warmup)
        # (untimed) up to 2 more steps so the timed ones start on a replayable period: graph
        # replay on one rank, the segmented plan on many
        extra = eng.align_period() if a.graph else 0
        eng.sync()
        eng.audit_reset()
        eng.clock()  # (reset: the engine-clock record covers the timed steps only)
        torch.cuda.synchronize()
        comm.barrier(dist)
        torch.cuda.synchronize()
        g.stage("timed", budget(a.steps))
        t0 = time.perf_counter()
        eng.step(a.steps)
        eng.sync()
        torch.cuda.synchronize()
        comm.barrier(dist)
        t1 = time.perf_counter()
        wall = comm.allreduce_max(dist, t1 - t0)
        g.stage("audits", budget(4, 180))
        clk = eng.clock()  # the timed steps' force launches (sym schedule)
        ginfo = eng.graph_info()
        # HBM the stepper holds (its allocation ledger; RCCL's own buffers excluded), max
        # over ranks
        mem = eng.mem_info() if hasattr(eng, "mem_info") else {}
        hbm_max = comm.allreduce_max(dist, float(sum(mem.values())))

        # ---- audits of the timed work (untimed) ----------------------------------------
        failures = []
        done, per_step = eng.audit()
        if per_step:
            short = comm.allreduce_sum(dist, 0.0 if done == per_step * a.steps else 1.0)
            units = {"units_per_step_rank0": per_step,
                     "units_done_rank0": done, "ranks_short": int(short)}
            if short:
                S, D, Kr, Np = eng.sym_geometry()
                failures.append(f"unit count: {int(short)} rank(s) did not run rows x (S + D + "
                                f"(Np - 1) Kr) units per timed step (S {S}, D {D}, Kr {Kr}, Np "
                                f"{Np}; rank {rank}: "
                                f"{done} of {per_step * a.steps})")
        else:
            units = None  # one-sided schedules: no unit counter, the replay audit still runs
        if overlap == 3 and os.environ.get("GRAVSIM_TEST_FAIL_GATED_AUDIT") == "1":
            failures.append("injected failure (GRAVSIM_TEST_FAIL_GATED_AUDIT, test hook)")
        bad = comm.allreduce_sum(dist, eng.nonfinite())
        pos_t, vel_t, _ = own_state(eng)
        p1, _ = momentum(dist, comm, vel_t, mass)
        drift = float(np.linalg.norm(p1 - p0)) / max(pscale, 1e-300)
        err_end = bound_end = None
        if a.check_samples > 0:
            err_end, bound_end = (comm.allreduce_max(dist, x) for x in sampled_error(
                eng, cfg, a.check_samples))
            worst_bound = max(bound0, bound_end)
            if worst_bound > ACC_BOUND_C:
                failures.append(f"accuracy: a sampled body's error is {worst_bound:.1f} x "
                                f"eps x sum|terms| (bound {ACC_BOUND_C:.0f})")
        conservation = None
        if cons0 is not None:
            conservation = conservation_summary(cons0, engine_conserved(eng, dist))
            conservation.pop("samples")
            conservation["note"] = (
                "KD (first order) at dt = 3600 s on uniform random ICs: a body passing close to "
                "the point-mass Sun or to another body within one step changes the total energy "
                "by orders of magnitude (the reference's configuration); the Newton-3 pairs keep "
                "momentum and angular momentum at rounding level")

        # Comm/compute split (untimed): a few eager steps with per-step phase events.
        phase = None
        if a.phase_steps > 0:
            g.stage("phase", budget(a.phase_steps + 2))
            if a.graph:
                # whole periods (the state reads above gathered the current buffer), so the
                # phase events come from the schedule the timed loop replayed: the step graph
                # (one rank) or the segmented plan
                eng.align_period()
            eng.set_timing(True)
            eng.step(a.phase_steps)
            phase = eng.phase_stats()
            eng.set_timing(False)
            for k in ("step_ms", "comm_ms", "exposed_comm_ms", "gather_ms", "exchange_ms"):
                phase[k] = comm.allreduce_max(dist, phase[k])

        # Replay: warmup + K steps from the same ICs on an independent schedule must give the
        # timed run's bits (eager launches, one static unit per workgroup, no gating).
        replay = None
        if a.replay_audit:
            g.stage("replay", budget(a.warmup + extra + a.steps))
            cap = eng.dyn_cap
            eng.set_schedule(0, 0)
            eng.set_overlap(0)
            eng.init_ics("solar+random", cfg.seed)
            eng.step(a.warmup + extra + a.steps)
            eng.sync()
            pos_r, vel_r, _ = own_state(eng)
            same = np.array_equal(pos_r, pos_t) and np.array_equal(vel_r, vel_t)
            diff = comm.allreduce_sum(dist, 0.0 if same else 1.0)
            replay = "bitwise" if not diff else f"differs on {int(diff)} rank(s)"
            if diff:
                failures.append(f"replay: the independent schedule differs on {int(diff)} rank(s)")
            eng.set_schedule((2 if a.graph_comm else 1) if a.graph else 0, cap)
            eng.set_overlap(overlap)
        return dict(extra=extra, wall=wall, clk=clk, ginfo=ginfo, mem=mem, hbm_max=hbm_max,
                    failures=failures,
                    units=units, bad=bad, drift=drift, err_end=err_end, bound_end=bound_end,
                    conservation=conservation, phase=phase, replay=replay)

    res = measure(overlap)
    fallback = None
    if res["failures"] and overlap == 3 and a.overlap == "auto":
        # The gated local-first launch (the multi-rank default) passed its 2-step self-check
        # but the audit of its timed steps failed. That is a failure of the default schedule:
        # the ungated schedule is timed from the same ICs so the run still has a (labelled)
        # number, but work_audit reports the failure and the run exits non-zero.
        fallback = {"from_overlap": 3, "to_overlap": 0, "failures": res["failures"]}
        overlap = 0
        eng.set_overlap(0)
        g.stage("ics", budget(0))
        eng.init_ics("solar+random", cfg.seed)
        eng.sync()
        res = measure(0)
        res["failures"] = ["gated schedule (the multi-rank default) failed its audit, fell back "
                           "to the ungated one: " + "; ".join(fallback["failures"])] + \
            res["failures"]
    wall, ginfo, mem, hbm_max = res["wall"], res["ginfo"], res["mem"], res["hbm_max"]
    failures, units, bad, drift = res["failures"], res["units"], res["bad"], res["drift"]
    err_end, conservation, phase, replay = (res["err_end"], res["conservation"], res["phase"],
                                            res["replay"])
    bound_end = res["bound_end"]
    # Engine clock over the timed steps, per rank (each GPU holds its own DVFS state): the
    # whole job's workgroup-cycles and the CUs it ran on, for clock-normalised costs
    clk = res["clk"]
    ghz_min = comm.allreduce_max(dist, -clk["ghz"]) * -1.0
    ghz_max = comm.allreduce_max(dist, clk["ghz"])
    ghz_sum = comm.allreduce_sum(dist, clk["ghz"])
    wg_cycles = comm.allreduce_sum(dist, clk["wg_cycles"])
    # CUs of the distinct GPUs the job ran on (the one-GPU rehearsal's ranks share one)
    cus_local = float(torch.cuda.get_device_properties(torch.cuda.current_device())
                      .multi_processor_count)
    cus_total = (float(sum({(r.get("host"), r.get("pci")): r.get("cus") or 0
                            for r in ranks_info}.values())) if ranks_info else cus_local)

    # P-independence (untimed, P > 1): the multi-rank bits against one rank on rank 0's GPU.
    p_audit = None
    small = cfg.n <= ((4 << 20) if a.dtype == "fp32" else (1 << 20))
    if world > 1 and (a.p_audit == "on" or (a.p_audit == "auto" and small)):
        g.stage("p_audit", budget(4 * world + 4, 180))
        p_audit = p_independence_audit(eng, cfg, dist, comm, dev)
        if p_audit != "bitwise":
            failures.append(f"P-independence: {p_audit}")
    elif world > 1:
        p_audit = "skipped (--p-audit off or size)"

    # The reference's exact hard-cutoff select (cuda.cu:39, mpi.c:64), timed on its own.
    lay = eng.native_layout
    fmode = eng.force_mode()
    exact_ms = None
    if a.exact_steps > 0:
        # the same schedule as the headline: the replayed step graph (segmented plan for
        # P > 1) rebuilt for the exact kernels, timed from a period start
        g.stage("exact", budget(4 + 2 * a.exact_steps))
        eng.set_cutoff_mode("exact")
        eng.step(2)
        if a.graph:
            eng.align_period()
        eng.sync()
        comm.barrier(dist)
        t0 = time.perf_counter()
        eng.step(a.exact_steps)
        eng.sync()
        comm.barrier(dist)
        exact_ms = 1e3 * comm.allreduce_max(dist, time.perf_counter() - t0) / a.exact_steps
    g.stage("close", budget(0))
    eng.close()
    if rank == 0:
        value = cfg.n * a.steps / wall
        mode = _native.MODE_NAMES.get(lay["mode"])
        if mode == "sym":
            # Newton-3 schedule: each unordered pair once, both sides (nbody_sym.hip); the
            # tile shape is the compiled one (gs_sym_tile_shape)
            kernel_info = {"kernel": _native.sym_kernel_label(a.dtype == "fp64"),
                           "n_pad": lay["n_pad"]}
            exch = ("ring of P-1 neighbour stages" if a.strategy == "ring" else "all-gather") + \
                " + node-sum send/recv"
            pairs = cfg.n * (cfg.n - 1) / 2  # unordered pairs, each evaluated once
        else:
            kernel_info = {"kernel": _native.KERNEL_NAMES.get(lay["kernel"]), "ipl": lay["ipl"],
                           "chunk": lay["chunk"]}
            exch = "ring send/recv" if a.strategy == "ring" else "all-gather"
            pairs = float(cfg.n) * cfg.n  # one-sided: every ordered pair evaluated
        parallelism = (f"body-decomposition x{world} (RCCL {exch})" if world > 1
                       else "single GPU")
        clock = clock_summary(ghz_sum, ghz_min, ghz_max, wg_cycles, wall, cus_total,
                              pairs * a.steps, world)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "body-updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": 1e3 * wall / a.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,  # the reference publishes no numbers
            "dtype": a.dtype,
            "data": DATA,
            "status": "ok" if not failures else "audit failed",
            "engine_clock_ghz": clock["engine_clock_ghz"],
            "cycles_per_pair_eval": clock["cycles_per_pair_eval"],
            "config": {
                "model": MODEL,
                "n_bodies": cfg.n,
                "global_batch": cfg.n,
                "seq_len": 1,
                "dt": cfg.dt,
                "parallelism": parallelism,
                "mode": mode,
                **kernel_info,
                "cutoff_path": "exact-select" if fmode["exact"] else
                f"fast (r^2 + c^2 with c^2={fmode['eps2']:.3g} m^2 instead of the hard-cutoff "
                "select: bit-identical to the 1e-10 m select for separations above ~1 cm; a "
                "pair closer than the cutoff gets a finite softened force mu r / (r^2 + c^2)^1.5 "
                "instead of 0; exact_cutoff_ms_per_step times the select)",
                # eager | graph (one-rank hipGraphs of graph_steps_per_launch steps, and of two
                # for a remainder) | segmented (multi-rank: compute
                # segments as graphs, RCCL collectives eager between them)
                "graph": ginfo["mode"],
                "graph_segments": ginfo["segments"] or None,
                # one-rank replays: steps per graph launch (every step's kernels are in it)
                "graph_steps_per_launch": ginfo.get("steps_per_launch"),
                "overlap": overlap,
                "overlap_check": overlap_check,
                "overlap_fallback": fallback,
                "step_timeout_s": step_to,
                # untimed steps added after the warmup so the timed ones start on a replayable
                # two-step period (graph / segmented plan)
                "warmup_align_steps": res["extra"],
                "first_step_ms": 1e3 * first_s,
                # N^2 ordered pair terms per step (what a one-sided sum evaluates) ...
                "effective_interactions_per_s": float(cfg.n) * cfg.n * a.steps / wall,
                # ... and the pair evaluations actually performed (sym: N(N-1)/2 per step)
                "pair_evals_per_s": pairs * a.steps / wall,
                "sampled_rel_err": err,
                "sampled_rel_err_final": err_end,
                # max |a - a_ref| / (eps x sum_j |term_ij|) over the sampled bodies and
                # components, at step 0 and after the run (gate: <= ACC_BOUND_C)
                "sampled_bound_ratio": [bound0, bound_end],
                "momentum_rel_drift": drift,
                # total energy (kinetic + exact-cutoff potential), momentum and angular momentum
                # before the warmup and after the timed steps (KD is first order: the energy
                # drift is the integrator's, at dt = 3600 s)
                "conservation": conservation,
                "exact_cutoff_ms_per_step": exact_ms,
                "nonfinite": int(bad),
                "clock": clock,
                "hbm": {"gb_per_rank_max": round(hbm_max / 1e9, 3),
                        "by_buffer_gb_rank0": {k: round(v / 1e9, 4) for k, v in mem.items()}},
            },
            "work_audit": "ok" if not failures else "; ".join(failures),
            "audit": {"units": units, "replay": replay, "p_independence": p_audit},
        }
        if world > 1:
            out["config"]["launch"] = launch_info()
            out["config"]["ranks"] = ranks_info
            out["config"]["topology"] = topology
            out["rccl_nranks"] = ranks_info[0].get("rccl_nranks") if ranks_info else None
        if phase is not None:
            out["comm_ms"] = phase["comm_ms"]
            out["exposed_comm_ms"] = phase["exposed_comm_ms"]
            out["config"]["phase"] = {k: phase[k] for k in (
                "steps", "step_ms", "gather_ms", "exchange_ms", "exposed_gather_ms",
                "exposed_exchange_ms", "deferred_units", "graph")}
        print(json.dumps(out), flush=True)
    g.stage("shutdown", init_b)
    comm.shutdown(dist)
    if failures:
        print("bench.py: work audit FAILED: " + "; ".join(failures), file=sys.stderr, flush=True)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
