"""Process-group bootstrap and host-side collectives.

One process per GPU (or per CPU shard), launched by `torch.distributed.run` / torchrun
(RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT in the environment). Replaces
mpi.c:142-144 (MPI_Init / Comm_rank / Comm_size) and pyspark.py:49-53 (SparkSession).

* Control plane: a torch.distributed **gloo** group (barrier, max-reduce of timings, the
  broadcast of the 128-byte RCCL unique id, final-state gathers for dumps).
* GPU data plane: the native RCCL communicator inside the Stepper (in-place ncclAllGather
  over xGMI every step) — see csrc/hip/stepper.hip.
* CPU data plane (no GPU): gloo all-gather of the own position slice every step, the
  direct analogue of mpi.c's per-step MPI_Allgatherv (mpi.c:227-231) without its aliasing.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import numpy as np


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    initialized: bool = False  # we own a torch.distributed process group

    @property
    def is_root(self) -> bool:
        return self.rank == 0


def env_info() -> DistInfo:
    return DistInfo(rank=int(os.environ.get("RANK", "0")),
                    world=int(os.environ.get("WORLD_SIZE", "1")),
                    local_rank=int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))))


def rccl_rank_hosts(rank: int) -> None:
    """Rehearsal knob (GRAVSIM_RCCL_RANK_HOSTS=1): give every rank its own NCCL_HOSTID so that
    RCCL accepts several ranks on ONE GPU (it refuses two ranks of one host on one device) and
    connects them through its socket transport over loopback. Lets a 1-GPU box run the real
    multi-rank RCCL schedule (tests/test_rccl_gpu.py, scripts/gpu_torchrun.sh); never set on
    a multi-GPU node, where the ranks must share a host to use xGMI."""
    os.environ["NCCL_HOSTID"] = f"gravsim-rank{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")


def init(timeout_s: float = 600.0) -> DistInfo:
    """Initialise the gloo control group when WORLD_SIZE > 1 (no-op for a single process)."""
    info = env_info()
    if info.world <= 1:
        return info
    if os.environ.get("GRAVSIM_RCCL_RANK_HOSTS") == "1":
        rccl_rank_hosts(info.rank)
    import torch.distributed as dist

    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=info.rank, world_size=info.world,
                                timeout=datetime.timedelta(seconds=timeout_s))
    info.initialized = True
    return info


def shutdown(info: DistInfo) -> None:
    if info.initialized:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()
        info.initialized = False


def barrier(info: DistInfo) -> None:
    if info.world > 1:
        import torch.distributed as dist

        dist.barrier()


def broadcast_bytes(info: DistInfo, payload: bytes | None, src: int = 0) -> bytes:
    if info.world <= 1:
        assert payload is not None
        return payload
    import torch
    import torch.distributed as dist

    n = torch.tensor([len(payload) if info.rank == src else 0], dtype=torch.int64)
    dist.broadcast(n, src)
    buf = torch.zeros(int(n.item()), dtype=torch.uint8)
    if info.rank == src:
        buf.copy_(torch.frombuffer(bytearray(payload), dtype=torch.uint8))
    dist.broadcast(buf, src)
    return bytes(buf.numpy().tobytes())


def allgather_object(info: DistInfo, obj) -> list:
    """Every rank's picklable `obj`, in rank order (control plane only: small records)."""
    if info.world <= 1:
        return [obj]
    import torch.distributed as dist

    out = [None] * info.world
    dist.all_gather_object(out, obj)
    return out


def allreduce_max(info: DistInfo, value: float) -> float:
    if info.world <= 1:
        return float(value)
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(info: DistInfo, value: float) -> float:
    if info.world <= 1:
        return float(value)
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def allgather_rows(info: DistInfo, full: np.ndarray, local_begin: int, n_local: int) -> None:
    """In-place all-gather of equal row slices of `full` (rows [r*n_local, (r+1)*n_local))."""
    if info.world <= 1:
        return
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(full)  # shares memory
    mine = t[local_begin:local_begin + n_local].clone()
    dist.all_gather_into_tensor(t, mine)


def gather_rows_to_root(info: DistInfo, full: np.ndarray, rows: slice) -> None:
    """Make `full` complete on every rank from each rank's own `rows` (sum of disjoint slices)."""
    if info.world <= 1:
        return
    import torch
    import torch.distributed as dist

    mask = np.zeros(full.shape[0], dtype=bool)
    mask[rows] = True
    part = np.where(mask.reshape((-1,) + (1,) * (full.ndim - 1)), full, 0.0)
    t = torch.from_numpy(np.ascontiguousarray(part))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    full[...] = t.numpy()
