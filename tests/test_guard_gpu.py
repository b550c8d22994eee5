"""A stalled multi-rank bench run ends inside its budget with a parseable error line
(VERDICT r3 "next round" #1). Two RCCL ranks share the one GPU of the box (every rank its own
NCCL_HOSTID: RCCL's socket transport, gravsim/parallel/comm.py); GRAVSIM_TEST_STALL makes
rank 1 sleep when it enters a stage (gravsim/parallel/guard.py):

* comm_init: rank 0 blocks inside ncclCommInitRank waiting for rank 1's bootstrap; its guard
  stops the job after --init-timeout with the stage and the native init stage;
* timed: rank 0's timed steps wait on an all-gather rank 1 never joins; the native progress
  bound (--step-timeout) aborts the communicator and rank 0 reports the failed stage.
"""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(tmp_path, stall, *args, timeout=300):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           "2", "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--num-bodies", "65536", "--steps",
           "4", "--warmup", "1", "--exact-steps", "0", *args]
    env = dict(os.environ, PYTHONPATH=ROOT, GRAVSIM_RCCL_RANK_HOSTS="1",
               GRAVSIM_GUARD_DIR=str(tmp_path), GRAVSIM_TEST_STALL=stall, OMP_NUM_THREADS="1",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    t0 = time.time()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    return r, lines, time.time() - t0


def test_stall_in_comm_init_reports_within_budget(hip, tmp_path):
    r, lines, took = _bench(tmp_path, "comm_init@1:120", "--init-timeout", "25")
    assert r.returncode != 0, r.stdout[-2000:]
    assert len(lines) == 1, (r.stdout[-3000:], r.stderr[-3000:])
    e = lines[0]
    assert e["status"] == "error" and e["value"] is None and e["stage"] == "comm_init", e
    ranks = e["config"]["ranks"]
    assert ranks[0]["comm_stage"] == "in ncclCommInitRank", ranks[0]
    assert ranks[1]["stage"] == "comm_init"
    assert ranks[0].get("pci") and e["config"]["launch"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert took < 120, took  # start-up + 25 s budget, far inside the driver's 600 s


def test_stall_in_a_step_aborts_rccl_and_reports(hip, tmp_path):
    r, lines, took = _bench(tmp_path, "timed@1:200", "--step-timeout", "15")
    assert r.returncode != 0, r.stdout[-2000:]
    assert len(lines) == 1, (r.stdout[-3000:], r.stderr[-3000:])
    e = lines[0]
    assert e["status"] == "error" and e["stage"] == "timed", e
    assert "communicator aborted" in e["error"] or "timeout" in e["error"], e["error"]
    assert [x["stage"] for x in e["config"]["ranks"]] == ["timed", "timed"]
    assert took < 180, took
