"""What a multi-rank run actually ran on: the communicator RCCL formed, the GPU each rank bound
and the transport each connection used, checked before a number is reported.

The reference's MPI job trusts `mpirun` (mpi.c:142-144) and its exchange is whatever transport
MPI picked (mpi.c:227-236). A multi-GPU MI355X run can go wrong in ways that still produce a
plausible ms/step: two ranks bound to one device (a bad LOCAL_RANK or HIP_VISIBLE_DEVICES),
RCCL falling back to its socket transport instead of xGMI peer-to-peer, or a communicator with
fewer ranks than the job. `topology_problems` turns the per-rank records bench.py gathers
(device, PCI id, host, ncclCommCount / UserRank / CuDevice, the transports parsed from RCCL's
INFO log) into a list of such problems; bench.py refuses to report a number when it is not
empty, except in the one-GPU rehearsal (GRAVSIM_RCCL_RANK_HOSTS=1), where every rank shares
device 0 over loopback sockets by design.
"""
from __future__ import annotations

from collections import defaultdict

# RCCL transports that carry data off the GPU fabric: on one node every peer should be
# reachable through P2P (xGMI, IPC) instead.
_NETWORK_PREFIXES = ("NET/",)


def rehearsal(env: dict) -> bool:
    """The one-GPU multi-rank rehearsal (every rank on device 0, sockets over loopback)."""
    return env.get("GRAVSIM_RCCL_RANK_HOSTS") == "1"


def topology_problems(world: int, ranks: list[dict]) -> list[str]:
    """Problems with a multi-rank run's topology; [] when it is what a one-GPU-per-rank node
    run must be. `ranks`: one record per rank with keys rank, host, device, pci, rccl_nranks,
    rccl_rank, rccl_device and transports (a list, or None when the RCCL log was not parsed).

    * the communicator: ncclCommCount must equal the job's world size, ncclCommUserRank the
      rank, ncclCommCuDevice the device the rank bound;
    * one GPU per rank: no PCI id twice on one host;
    * one node: no connection through a network transport (NET/Socket, NET/IB) when every
      rank is on the same host.
    """
    out: list[str] = []
    if len(ranks) != world:
        out.append(f"{len(ranks)} rank record(s) for a world of {world}")
    for r in sorted(ranks, key=lambda x: x.get("rank", -1)):
        q = r.get("rank")
        if r.get("rccl_nranks") is None:  # (a library that cannot report it: nothing to check)
            continue
        if r.get("rccl_nranks") != world:
            out.append(f"rank {q}: RCCL communicator has {r.get('rccl_nranks')} rank(s), the job "
                       f"{world}")
        if r.get("rccl_rank") != q:
            out.append(f"rank {q}: RCCL placed it at rank {r.get('rccl_rank')}")
        if r.get("rccl_device") != r.get("device"):
            out.append(f"rank {q}: RCCL runs on device {r.get('rccl_device')}, the rank bound "
                       f"device {r.get('device')}")
    by_gpu: dict = defaultdict(list)
    for r in ranks:
        by_gpu[(r.get("host"), r.get("pci"))].append(r.get("rank"))
    for (host, pci), rs in sorted(by_gpu.items(), key=lambda kv: str(kv[0])):
        if len(rs) > 1:
            out.append(f"ranks {sorted(rs)} share GPU {pci} on host {host}")
    hosts = {r.get("host") for r in ranks}
    if len(hosts) == 1:
        for r in sorted(ranks, key=lambda x: x.get("rank", -1)):
            net = [t for t in (r.get("transports") or []) if t.startswith(_NETWORK_PREFIXES)]
            if net:
                out.append(f"rank {r.get('rank')}: connections through {net} on a single node "
                           "(expected P2P over xGMI)")
    return out


def transport_summary(ranks: list[dict]) -> dict:
    """Transports in use across the job and whether every rank's log was parsed."""
    seen = sorted({t for r in ranks for t in (r.get("transports") or [])})
    return {"transports": seen,
            "parsed_ranks": sum(1 for r in ranks if r.get("transports") is not None),
            "p2p": any(t.startswith("P2P") for t in seen),
            "network": [t for t in seen if t.startswith(_NETWORK_PREFIXES)]}
