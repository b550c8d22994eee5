"""Self-launch of P ranks on one node: the `mpirun -np P ./mpi` step of the reference
(mpi.c:140-144) for this framework's entry points.

`python bench.py --gpus 8` / `python -m gravsim --gpus 8 ...` started WITHOUT a launcher
re-run themselves as P ranks under `torch.distributed.run` in a CHILD process (never an
exec: the parent has not touched the GPU, and on this pool exec'ing from a process that has
would take the machine down). Rendezvous is on 127.0.0.1 with a free port. The child's
stdout/stderr are inherited, so rank 0's output (bench.py's single JSON line) is the only
thing printed, and the parent exits with the child's return code.

Everything here is host-side and GPU-free, so `torchrun_cmd` is unit-tested on the CPU.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import Iterable, Optional

# Options that select the rank count; the children get them back as `--gpus P` only when the
# entry point asks for it (bench.py re-checks WORLD_SIZE against it).
_RANK_FLAGS = ("--nproc", "--gpus")


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def strip_rank_flags(argv: Iterable[str]) -> list[str]:
    """Drop `--gpus P` / `--nproc P` (either spelling, `=` form too) and rename `--n` to
    `--num-bodies`: torch.distributed.run's own parser reads `--n` as an ambiguous prefix of
    its `--nnodes`/`--nproc-per-node` even after the script name."""
    rest: list[str] = []
    skip = False
    for x in argv:
        if skip:
            skip = False
            continue
        if x in _RANK_FLAGS:
            skip = True
            continue
        if x.startswith(tuple(f + "=" for f in _RANK_FLAGS)):
            continue
        if x == "--n":
            rest.append("--num-bodies")
        elif x.startswith("--n="):
            rest.append("--num-bodies=" + x[4:])
        else:
            rest.append(x)
    return rest


def torchrun_cmd(nproc: int, target: list[str], argv: Iterable[str], port: int,
                 keep_gpus: bool = False) -> list[str]:
    """The child command: `python -m torch.distributed.run --nnodes 1 --nproc-per-node P
    --master-addr 127.0.0.1 --master-port PORT <target> <argv without rank flags>`.
    `target` is `[script.py]` or `["-m", "module"]`. With keep_gpus the children get
    `--gpus P` back (bench.py checks it against WORLD_SIZE)."""
    if nproc < 1:
        raise ValueError("nproc must be >= 1")
    rest = strip_rank_flags(argv)
    if keep_gpus:
        rest = ["--gpus", str(nproc), *rest]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
            str(nproc), "--master-addr", "127.0.0.1", "--master-port", str(port), *target, *rest]


PROBE_ENV = "GRAVSIM_LAUNCH_PROBE"  # the parent's device count, handed to the ranks


def check_device_count(nproc: int) -> int:
    """Count the visible HIP devices (torch.cuda.device_count() does not initialise the GPU
    on this image) and refuse more ranks than devices: one rank per GPU. The one-GPU RCCL
    rehearsal (GRAVSIM_RCCL_RANK_HOSTS=1: every rank on device 0 over loopback sockets) runs
    the same probe and skips only the refusal, so it executes the production parent sequence
    probe -> torchrun child -> RCCL. Returns the count and exports it to the children
    (GRAVSIM_LAUNCH_PROBE; bench.py reports it)."""
    import torch

    have = torch.cuda.device_count()
    os.environ[PROBE_ENV] = str(have)
    if nproc > have and os.environ.get("GRAVSIM_RCCL_RANK_HOSTS") != "1":
        raise SystemExit(f"--gpus {nproc} but only {have} HIP device(s) are visible "
                         "(set GRAVSIM_RCCL_RANK_HOSTS=1 to rehearse several ranks on one GPU)")
    return have


def spawn(nproc: int, target: list[str], argv: Iterable[str], keep_gpus: bool = False,
          env: Optional[dict] = None) -> int:
    """Run `nproc` ranks of `target` as a child torch.distributed.run; return its exit code."""
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    e = dict(os.environ if env is None else env)
    e["PYTHONPATH"] = root + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this driver
    e.setdefault("OMP_NUM_THREADS", "1")
    cmd = torchrun_cmd(nproc, target, argv, free_port(), keep_gpus=keep_gpus)
    return subprocess.call(cmd, env=e)
