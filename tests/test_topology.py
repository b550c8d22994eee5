"""bench.py's multi-GPU topology enforcement (parallel/verify.py) on canned RCCL INFO logs: a
run is refused when the communicator RCCL formed is not the job, when two ranks bind one GPU,
or when a single-node connection goes through a network transport; the one-GPU rehearsal
(GRAVSIM_RCCL_RANK_HOSTS=1) is recorded but not enforced."""
from __future__ import annotations

from gravsim.parallel import guard, verify

# Lines in the shape RCCL prints with NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,P2P,NET (the
# socket lines are the ones the one-GPU rehearsal logs, profiles/r5_torchrun_rehearsal.txt).
P2P_LOG = """\
node0:1234:1240 [0] NCCL INFO RCCL version 2.26.6-HEAD:1b0bd2b
node0:1234:1240 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC
node0:1234:1240 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC
node0:1234:1240 [0] NCCL INFO Channel 00/1 : 0[0] -> 1[1] via P2P/IPC/read
"""
SOCKET_LOG = """\
node0:1234:1240 [0] NCCL INFO RCCL version 2.26.6-HEAD:1b0bd2b
node0:1234:1240 [0] NCCL INFO Using network Socket
node0:1234:1240 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[0] [send] via NET/Socket/0
node0:1234:1240 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[0] [send] via NET/Socket/0/Shared
"""


def _ranks(tmp_path, world, logs, pcis=None, devices=None, host="node0", over=None):
    out = []
    for r in range(world):
        p = tmp_path / f"rccl.{r}.log"
        p.write_text(logs[r] if isinstance(logs, list) else logs)
        rec = {"rank": r, "host": host, "device": (devices or list(range(world)))[r],
               "pci": (pcis or [f"0000:{0x11 + r:02x}:00" for r in range(world)])[r],
               "rccl_nranks": world, "rccl_rank": r,
               "rccl_device": (devices or list(range(world)))[r],
               **guard.parse_rccl_log(str(p))}
        rec.update((over or {}).get(r, {}))
        out.append(rec)
    return out


def test_clean_eight_gpu_node_passes(tmp_path):
    ranks = _ranks(tmp_path, 8, P2P_LOG)
    assert verify.topology_problems(8, ranks) == []
    summ = verify.transport_summary(ranks)
    assert summ["p2p"] and summ["network"] == [] and summ["parsed_ranks"] == 8
    assert "P2P/IPC" in summ["transports"]


def test_socket_transport_on_one_node_is_refused(tmp_path):
    ranks = _ranks(tmp_path, 2, [P2P_LOG, SOCKET_LOG])
    probs = verify.topology_problems(2, ranks)
    assert len(probs) == 1 and "rank 1" in probs[0] and "NET/Socket" in probs[0], probs


def test_two_ranks_on_one_gpu_are_refused(tmp_path):
    ranks = _ranks(tmp_path, 4, P2P_LOG,
                   pcis=["0000:11:00", "0000:12:00", "0000:12:00", "0000:14:00"])
    probs = verify.topology_problems(4, ranks)
    assert probs == ["ranks [1, 2] share GPU 0000:12:00 on host node0"], probs


def test_short_communicator_and_wrong_device_are_refused(tmp_path):
    ranks = _ranks(tmp_path, 2, P2P_LOG, over={1: {"rccl_nranks": 1, "rccl_device": 0}})
    probs = verify.topology_problems(2, ranks)
    assert any("communicator has 1 rank(s), the job 2" in p for p in probs), probs
    assert any("runs on device 0, the rank bound device 1" in p for p in probs), probs
    assert verify.topology_problems(3, ranks)[0] == "2 rank record(s) for a world of 3"


def test_network_transport_across_nodes_is_allowed(tmp_path):
    """Two hosts: the inter-node connections are network ones by necessity."""
    ranks = _ranks(tmp_path, 2, SOCKET_LOG, over={1: {"host": "node1"}})
    assert verify.topology_problems(2, ranks) == []


def test_same_pci_on_two_hosts_is_not_a_shared_gpu(tmp_path):
    ranks = _ranks(tmp_path, 2, P2P_LOG, pcis=["0000:11:00", "0000:11:00"],
                   over={1: {"host": "node1"}})
    assert verify.topology_problems(2, ranks) == []


def test_rehearsal_flag_and_its_records(tmp_path):
    """The one-GPU rehearsal: every rank on device 0 over sockets: the problems are listed
    (so the JSON line shows them) but bench.py does not enforce them there."""
    ranks = _ranks(tmp_path, 2, SOCKET_LOG, pcis=["0000:11:00"] * 2, devices=[0, 0])
    probs = verify.topology_problems(2, ranks)
    assert any("share GPU" in p for p in probs) and any("NET/Socket" in p for p in probs)
    assert verify.rehearsal({"GRAVSIM_RCCL_RANK_HOSTS": "1"})
    assert not verify.rehearsal({})


def test_unparsed_logs_are_reported_not_guessed(tmp_path):
    ranks = _ranks(tmp_path, 2, P2P_LOG,
                   over={0: {"transports": None}, 1: {"transports": None}})
    assert verify.topology_problems(2, ranks) == []
    assert verify.transport_summary(ranks)["parsed_ranks"] == 0


def test_unknown_communicator_fields_are_not_guessed(tmp_path):
    """A library that cannot report what RCCL formed (None) is not a failure by itself."""
    ranks = _ranks(tmp_path, 2, P2P_LOG, over={0: {"rccl_nranks": None, "rccl_rank": None,
                                                   "rccl_device": None}})
    assert verify.topology_problems(2, ranks) == []


def test_bench_enforces_the_topology(tmp_path):
    """bench.py's check_topology: a clean node passes and is recorded; a socket connection on
    one node stops the run (SystemExit, which the guard reports as the error line); the
    one-GPU rehearsal records the same problems without stopping."""
    import pytest

    import bench

    seen = []
    ok = bench.check_topology(2, _ranks(tmp_path, 2, P2P_LOG), {}, note=seen.append)
    assert ok["enforced"] and ok["problems"] == [] and ok["p2p"] and seen == [ok]
    bad = _ranks(tmp_path, 2, [P2P_LOG, SOCKET_LOG])
    with pytest.raises(SystemExit, match="multi-GPU topology check failed: rank 1"):
        bench.check_topology(2, bad, {})
    rehearsal = bench.check_topology(2, bad, {"GRAVSIM_RCCL_RANK_HOSTS": "1"})
    assert not rehearsal["enforced"] and len(rehearsal["problems"]) == 1
