"""Command-line entry: `python -m gravsim --n N --dt DT --steps STEPS [...]`.

Replaces the three reference `main`s, none of which parses arguments (cuda.cu:120,
mpi.c:140, pyspark.py:152), and the Spark configuration sweep (pyspark.py:166-200, `--sweep`).
Multi-process runs: `python -m torch.distributed.run --nproc-per-node P --master-addr
127.0.0.1 -m gravsim ...` (one rank per GPU; gloo control plane, RCCL data plane).
"""
from __future__ import annotations

import argparse
import sys
from typing import Optional

from .config import SimConfig


def build_parser() -> argparse.ArgumentParser:
    d = SimConfig()
    p = argparse.ArgumentParser(prog="gravsim", description="MI355X-native direct-sum N-body "
                                "gravity simulator (Sun/Earth/Mars + random bodies by default)")
    p.add_argument("--n", "--num-bodies", dest="n", type=int, default=d.n,
                   help="number of bodies (use --num-bodies under torch.distributed.run, "
                        "whose own options make --n ambiguous)")
    p.add_argument("--dt", type=float, default=d.dt, help="time step [s]")
    p.add_argument("--steps", type=int, default=d.steps, help="number of steps")
    p.add_argument("--dtype", choices=["fp32", "fp64"], default=d.dtype)
    p.add_argument("--device", choices=["auto", "cpu", "gpu"], default=d.device)
    p.add_argument("--init", default=d.init,
                   help="IC family: solar+random | random | plummer | kepler | cold")
    p.add_argument("--seed", type=int, default=d.seed)
    p.add_argument("--G", type=float, default=d.G)
    p.add_argument("--cutoff", type=float, default=d.cutoff)
    p.add_argument("--softening", type=float, default=d.softening)
    p.add_argument("--cutoff-mode", choices=["auto", "exact", "fast"], default=d.cutoff_mode,
                   help="GPU force path: exact hard-cutoff select, or fast (r^2 + a core of "
                        "the cutoff scale, no select; bit-identical for separations above ~1 cm)")
    p.add_argument("--integrator", choices=["kd", "leapfrog"], default=d.integrator,
                   help="kd: the reference's kick-drift update; leapfrog: the same kernel on "
                        "half-step-staggered velocities (second order)")
    p.add_argument("--kernel", choices=["auto", "lds", "smem", "mfma"], default=d.kernel,
                   help="GPU force kernel: lds (LDS-DMA j tiles), smem (SGPR j stream), mfma "
                        "(experimental fp32: r^2 on the matrix cores, re-centred; slower)")
    p.add_argument("--mode", choices=["auto", "fused", "split", "sym"], default=d.mode,
                   help="GPU schedule; sym = Newton-3 pairs (any P <= 8; the default from 16K bodies)")
    p.add_argument("--ipl", type=int, default=d.ipl, choices=[0, 1, 2, 4, 8])
    p.add_argument("--chunk", type=int, default=d.chunk)
    p.add_argument("--no-graph", dest="graph", action="store_false")
    p.add_argument("--graph-comm", dest="graph_comm", action="store_true",
                   help="replay multi-rank steps from a hipGraph that captures them, RCCL "
                        "collectives included (opt-in: over RCCL's socket transport the capture "
                        "is known to crash with a SIGSEGV inside hipStreamEndCapture)")
    p.add_argument("--no-graph-comm", dest="graph_comm", action="store_false",
                   help=argparse.SUPPRESS)
    p.add_argument("--step-timeout", dest="step_timeout_s", type=float, default=d.step_timeout_s,
                   help="multi-rank hang detection: abort the RCCL communicator when no step "
                        "completes for this many seconds (default: max(60, 20 x the measured "
                        "step time), at most 240; 0 = wait forever)")
    p.add_argument("--overlap", type=int, choices=[-1, 0, 3], default=d.overlap,
                   help="multi-rank sym schedule: work beside the all-gather (3: one launch, "
                        "rank-local units first, remote units once the gather is published, "
                        "the built-in default for P > 1; 0: wait for the gather, one launch; "
                        "-1: built-in default)")
    p.add_argument("--strategy", choices=["allgather", "ring"], default=d.strategy,
                   help="multi-rank GPU exchange: one all-gather overlapped with the local "
                        "chunks, or a ring of P-1 neighbour send/recv steps computed on arrival")
    p.add_argument("--threads", type=int, default=0)
    p.add_argument("--log-dir", default=None, help="write the text log under this directory")
    p.add_argument("--log-format", choices=["mpi", "spark", "cuda", "none"], default=d.log_format)
    p.add_argument("--progress-every", type=int, default=d.progress_every)
    p.add_argument("--print-positions", type=int, default=d.print_positions)
    p.add_argument("--dump", dest="dump_path", default=None,
                   help="final state: .txt (mpi.c 'Particle i: (x, y, z)' lines) or .gsck")
    p.add_argument("--dump-every", type=int, default=0,
                   help="also write mpi.c-format positions every k steps "
                        "(<dump stem>_stepNNNNNNNN.txt, or positions_stepNNNNNNNN.txt in "
                        "--log-dir / the working directory)")
    p.add_argument("--checkpoint-dir", default=None)
    p.add_argument("--checkpoint-every", type=int, default=0)
    p.add_argument("--resume", default=None, help="checkpoint file (or directory: latest)")
    p.add_argument("--record-every", type=int, default=0)
    p.add_argument("--record-path", default=None, help="trajectory .npy (frames x n x 3)")
    p.add_argument("--nan-check-every", type=int, default=0)
    p.add_argument("--metrics-json", default=None, help="append the run's JSON metrics line here")
    p.add_argument("--phase-timing", action="store_true",
                   help="GPU: time every step's phases with events and report the comm/compute "
                        "split (comm_ms, exposed_comm_ms) in the metrics (eager steps)")
    p.add_argument("--sweep", default=None,
                   help="comma-separated N values: run each config in turn (pyspark.py sweep)")
    p.add_argument("--nproc", "--gpus", dest="nproc", type=int, default=0,
                   help="launch this many ranks (one per GPU) on this node through "
                        "torch.distributed.run, like `mpirun -np N` (mpi.c); 0 = as launched")
    p.add_argument("--diagnostics", action="store_true",
                   help="conserved quantities (total energy with the exact-cutoff potential, "
                        "linear and angular momentum) at the start and end of the run, and "
                        "their relative drift in the metrics JSON")
    p.add_argument("--diag-every", type=int, default=0,
                   help="also sample them every k steps (implies --diagnostics; each sample is "
                        "an O(N^2) pass, excluded from the timed wall)")
    p.add_argument("--quiet", action="store_true")
    return p


def config_from_args(a: argparse.Namespace) -> SimConfig:
    from .utils import checkpoint as ckpt

    resume = a.resume
    if resume:
        import os

        if os.path.isdir(resume):
            resume = ckpt.latest(resume)
    return SimConfig(n=a.n, dt=a.dt, steps=a.steps, dtype=a.dtype, device=a.device, init=a.init,
                     seed=a.seed, G=a.G, cutoff=a.cutoff, softening=a.softening,
                     cutoff_mode=a.cutoff_mode, integrator=a.integrator, kernel=a.kernel,
                     mode=a.mode, ipl=a.ipl, chunk=a.chunk, graph=a.graph, graph_comm=a.graph_comm,
                     strategy=a.strategy, step_timeout_s=a.step_timeout_s, overlap=a.overlap,
                     threads=a.threads,
                     log_dir=a.log_dir, log_format=a.log_format, progress_every=a.progress_every,
                     print_positions=a.print_positions, dump_path=a.dump_path,
                     dump_every=a.dump_every,
                     checkpoint_dir=a.checkpoint_dir, checkpoint_every=a.checkpoint_every,
                     resume=resume, record_every=a.record_every, record_path=a.record_path,
                     nan_check_every=a.nan_check_every, metrics_json=a.metrics_json,
                     phase_timing=a.phase_timing,
                     diagnostics=a.diagnostics or a.diag_every > 0,
                     diag_every=a.diag_every).validate()


def run_one(cfg: SimConfig, dist, log, quiet: bool = False, final: bool = True,
            guard=None) -> dict:
    from .runtime.simulation import Simulation
    from .utils.logs import format_positions_mpi

    sim = Simulation(cfg, dist, guard=guard)
    try:
        if log and dist.is_root:
            log.header(dist.world, cfg.n, cfg.steps, cfg.dt)
        if guard:
            guard.stage("run", None)  # bounded by the native step timeout (progress)
        m = sim.run(cfg.steps, log if dist.is_root else None)
        if guard:
            guard.stage("output", None)
        state = sim.global_state()  # collective
        if cfg.dump_path and cfg.dump_path.endswith(".gsck"):
            sim.save_checkpoint(cfg.dump_path)  # collective; rank 0 writes
        if dist.is_root:
            if log:
                log.stats(m.wall_s, m.steps)
                log.positions(state.pos, cfg.print_positions)
                if final:
                    log.completed()
            if cfg.dump_path and not cfg.dump_path.endswith(".gsck"):
                with open(cfg.dump_path, "w") as f:
                    f.write(format_positions_mpi(state.pos))
            if cfg.record_path:
                sim.save_trajectory(cfg.record_path)
            line = m.to_json()
            if not quiet:
                print(line, flush=True)
            if cfg.metrics_json:
                with open(cfg.metrics_json, "a") as f:
                    f.write(line + "\n")
        return {"metrics": m, "state": state}
    finally:
        sim.close()


def _launch(nproc: int, argv: list[str]) -> int:
    """Re-run this CLI as `nproc` ranks under torch.distributed.run in a child process (no
    exec, nothing has touched the GPU yet); rendezvous on 127.0.0.1 (parallel/launch.py)."""
    from .parallel import launch

    return launch.spawn(nproc, ["-m", "gravsim"], argv)


def main(argv: Optional[list[str]] = None) -> int:
    import os

    from .parallel import comm
    from .utils.logs import RunLog

    raw = list(sys.argv[1:] if argv is None else argv)
    a = build_parser().parse_args(raw)
    if a.nproc > 1 and "WORLD_SIZE" not in os.environ:
        if a.device != "cpu":
            import torch  # device_count() does not initialise the GPU on this image

            if a.device == "gpu" or torch.cuda.device_count() > 0:
                from .parallel import launch

                launch.check_device_count(a.nproc)  # one rank per GPU
        return _launch(a.nproc, raw)
    if a.nproc > 0 and int(os.environ.get("WORLD_SIZE", "1")) != a.nproc:
        raise SystemExit(f"--gpus/--nproc {a.nproc} but WORLD_SIZE {os.environ.get('WORLD_SIZE')}")
    cfg = config_from_args(a)
    guard = None
    world = int(os.environ.get("WORLD_SIZE", "1") or 1)
    if world > 1:
        # Multi-rank: a stalled or failed rank ends the job with rank 0's error JSON line
        # (stage, every rank's record) and exit code 70 instead of a hang (parallel/guard.py).
        from .parallel.guard import INIT_TIMEOUT_S, RunGuard

        guard = RunGuard(int(os.environ.get("RANK", "0") or 0), world,
                         lambda reason, recs: {"status": "error", "error": reason,
                                               "stage": recs[0].get("stage") if recs else None,
                                               "n": cfg.n, "nranks": world, "ranks": recs})
        guard.stage("gloo_init", INIT_TIMEOUT_S)
    dist = comm.init(timeout_s=180.0 if guard else 600.0)
    from .runtime.simulation import NonFiniteError

    try:
        if a.sweep:
            sizes = [int(x) for x in a.sweep.split(",") if x]
            fmt = cfg.log_format if a.log_format != "mpi" else "spark"
            log = RunLog(fmt, cfg.log_dir if dist.is_root else None, echo=dist.is_root)
            for n in sizes:
                run_one(cfg.replace(n=n, log_format=fmt), dist, log, a.quiet, final=False,
                        guard=guard)
            if dist.is_root:
                log.completed()
        else:
            log = RunLog(cfg.log_format, cfg.log_dir if dist.is_root else None,
                         echo=dist.is_root and not a.quiet)
            run_one(cfg, dist, log, a.quiet, guard=guard)
    except NonFiniteError as e:  # the NaN/Inf guard (--nan-check-every): fail loudly
        print(f"gravsim: error: {e}", file=sys.stderr, flush=True)
        return 3
    except Exception as e:  # noqa: BLE001 - multi-rank: every failure becomes a report
        if guard is None:
            raise
        guard.fail(f"{type(e).__name__}: {e}")
    finally:
        comm.shutdown(dist)
    if guard:
        guard.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
