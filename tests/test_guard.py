"""The run guard (gravsim/parallel/guard.py): stage deadlines, failures on any rank, rank 0's
error JSON line and exit code, and bench.py's error path end to end on the CPU (no GPU here:
bench.py stops at its device stage and must say so in one parseable line)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import textwrap
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gravity-simulator-using-mpi-spark-and-cuda_amd")


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(**kw):
    e = dict(os.environ, PYTHONPATH=ROOT, **{k: str(v) for k, v in kw.items()})
    e.pop("GRAVSIM_TEST_STALL", None)
    e.update({k: str(v) for k, v in kw.items()})
    return e


SCRIPT = textwrap.dedent("""
    import os, sys, time
    import gravsim
    from gravsim.parallel.guard import RunGuard
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    g = RunGuard(rank, world, lambda reason, recs: {"status": "error", "error": reason,
                 "stages": [r.get("stage") for r in recs],
                 "errors": [r.get("error") for r in recs]})
    mode = os.environ["MODE"]
    if mode == "deadline":
        g.stage("slow", 0.5)
        time.sleep(20)
    elif mode == "ok":
        g.stage("quick", 5)
        g.close()
        print("done", flush=True)
    elif mode == "peer_fails":
        if rank == 1:
            g.stage("compute", 30)
            try:
                raise RuntimeError("boom on rank 1")
            except RuntimeError as e:
                g.fail(str(e))
        g.stage("wait_for_peer", 60)
        time.sleep(30)
    elif mode == "both_fail":
        # every rank meets the same failure, rank 1 a little later (it started slower)
        g.stage("device", 30)
        time.sleep(0.8 * rank)
        g.fail(f"no device on rank {rank}")
    elif mode == "stall_hook":
        g.stage("setup", 0.8)  # GRAVSIM_TEST_STALL sleeps past this budget
        g.close()
        print("not stopped", flush=True)
""")


def _run(mode, world=1, timeout=40, **env):
    d = env.pop("guard_dir")
    procs = []
    t0 = time.time()
    for r in range(world):
        e = _env(MODE=mode, RANK=r, WORLD_SIZE=world, GRAVSIM_GUARD_DIR=d, **env)
        procs.append(subprocess.Popen([sys.executable, "-c", SCRIPT], env=e,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=timeout) for p in procs]
    return [p.returncode for p in procs], outs, time.time() - t0


def test_stage_deadline_reports_and_exits(tmp_path):
    from gravsim.parallel.guard import EXIT_CODE

    rcs, outs, took = _run("deadline", guard_dir=tmp_path)
    assert rcs == [EXIT_CODE], outs
    line = json.loads(outs[0][0].strip().splitlines()[-1])
    assert line["status"] == "error" and "slow" in line["error"] and line["stages"] == ["slow"]
    assert took < 15, took


def test_clean_run_is_not_stopped(tmp_path):
    rcs, outs, _ = _run("ok", guard_dir=tmp_path)
    assert rcs == [0] and outs[0][0].strip() == "done", outs
    assert not os.path.exists(tmp_path / "rank0.json")


def test_failure_on_another_rank_is_reported_by_rank0(tmp_path):
    from gravsim.parallel.guard import EXIT_CODE

    rcs, outs, took = _run("peer_fails", world=2, guard_dir=tmp_path)
    assert rcs == [EXIT_CODE, EXIT_CODE], outs
    line = json.loads(outs[0][0].strip().splitlines()[-1])
    assert "rank 1" in line["error"] and "boom on rank 1" in line["error"]
    assert line["stages"] == ["wait_for_peer", "compute"]
    assert "boom on rank 1" in line["errors"][1]
    assert took < 20, took  # rank 0 did not sit out its 60 s stage


def test_report_waits_briefly_for_peers_to_end(tmp_path):
    """Rank 0 fails first; rank 1 meets the same failure 0.8 s later. The report shows both
    ranks' own errors (PEER_GRACE_S), not rank 1 still entering its stage."""
    from gravsim.parallel.guard import EXIT_CODE

    rcs, outs, took = _run("both_fail", world=2, guard_dir=tmp_path)
    assert rcs == [EXIT_CODE, EXIT_CODE], outs
    line = json.loads(outs[0][0].strip().splitlines()[-1])
    assert line["stages"] == ["device", "device"], line
    assert line["errors"] == ["no device on rank 0", "no device on rank 1"], line
    assert took < 20, took


def test_stall_hook(tmp_path):
    from gravsim.parallel.guard import EXIT_CODE

    rcs, outs, _ = _run("stall_hook", guard_dir=tmp_path, GRAVSIM_TEST_STALL="setup@0:5")
    assert rcs == [EXIT_CODE], outs
    assert "setup" in json.loads(outs[0][0].strip().splitlines()[-1])["error"]


def test_step_timeout_bounds():
    from gravsim.parallel.guard import step_timeout

    assert step_timeout(0.16) == 60.0  # 1M on one GPU
    assert step_timeout(5.2) == 104.0  # 16M / 8 ranks
    assert step_timeout(100.0) == 240.0  # capped well under the driver's 600 s
    assert step_timeout(0.01, floor_s=10) == 10.0


def _json_lines(text):
    out = []
    for ln in text.splitlines():
        if ln.startswith("{"):
            out.append(json.loads(ln))
    return out


def test_bench_without_gpu_prints_error_json(tmp_path):
    """bench.py on a box without a HIP device: one parseable error line, exit 70."""
    from gravsim.parallel.guard import EXIT_CODE

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--n", "4096",
                        "--init-timeout", "30"], env=_env(GRAVSIM_GUARD_DIR=tmp_path,
                                                          HIP_VISIBLE_DEVICES=""),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == EXIT_CODE, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    e = lines[0]
    assert e["status"] == "error" and e["value"] is None and e["stage"] == "device"
    assert e["metric"].startswith("body-updates/sec") and e["n_gpus"] == 1
    assert "HIP device" in e["error"]


def test_bench_two_ranks_stalled_init_reports_within_budget(tmp_path):
    """Two gloo ranks under torch.distributed.run; rank 1 stalls before joining the control
    plane. Rank 0's gloo init stage must end the job within --init-timeout with an error line
    naming the stage and both ranks' records."""
    from gravsim.parallel.guard import EXIT_CODE

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           "2", "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--num-bodies", "4096",
           "--init-timeout", "8"]
    t0 = time.time()
    r = subprocess.run(cmd, env=_env(GRAVSIM_GUARD_DIR=tmp_path,
                                     GRAVSIM_TEST_STALL="gloo_init@1:60", OMP_NUM_THREADS=1),
                       capture_output=True, text=True, timeout=240)
    took = time.time() - t0
    assert r.returncode != 0
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, (r.stdout[-3000:], r.stderr[-3000:])
    e = lines[0]
    assert e["status"] == "error" and e["stage"] == "gloo_init", e
    ranks = e["config"]["ranks"]
    assert [x["rank"] for x in ranks] == [0, 1]
    assert ranks[1]["stage"] == "gloo_init"
    assert "HSA_ENABLE_IPC_MODE_LEGACY" in e["config"]["launch"]
    assert took < 60, took
    del EXIT_CODE


def test_stale_peer_record_of_an_earlier_job_is_ignored(tmp_path):
    """A reused guard directory still holds a 'failed' record of rank 1 from an earlier job
    (its process gone): rank 0 of the new job must not fire on it, and a record of
    a live peer of this job still counts."""
    import io

    from gravsim.parallel import guard as gd

    stale = {"rank": 1, "pid": 2 ** 22 + 12345, "stage": "timed", "status": "failed",
             "error": "old job", "t_stage": time.time() - 3600, "t_start": time.time() - 3600}
    (tmp_path / "rank1.json").write_text(json.dumps(stale))
    g = gd.RunGuard(0, 2, lambda reason, recs: {"error": reason}, directory=str(tmp_path),
                    poll_s=0.05, out=io.StringIO())
    try:
        assert g._peer_records() == []
        time.sleep(0.3)
        assert not g._fired
        with g._lock:
            g._closed = True  # (stop the watchdog before a live 'failed' record appears)
        time.sleep(0.15)
        live = dict(stale, pid=os.getpid(), t_start=time.time(), error="this job")
        (tmp_path / "rank1.json").write_text(json.dumps(live))
        assert [r["error"] for r in g._peer_records()] == ["this job"]
    finally:
        g._closed = True


def test_failed_record_of_an_exited_peer_of_this_job_is_reported(tmp_path, monkeypatch):
    """A peer of THIS job that recorded "failed" and exited (its pid gone) is still reported,
    and so is one whose pid lives on another node (a shared GRAVSIM_GUARD_DIR); a record with
    another job id is not (the filter is the job and its start time, not pid
    liveness)."""
    import io

    from gravsim.parallel import guard as gd

    monkeypatch.setenv("GRAVSIM_JOB_ID", "job-a")
    g = gd.RunGuard(0, 3, lambda reason, recs: {"error": reason}, directory=str(tmp_path),
                    poll_s=60.0, out=io.StringIO())
    try:
        now = time.time()
        dead = {"rank": 1, "pid": 2 ** 22 + 4321, "stage": "timed", "status": "failed",
                "error": "exited peer", "t_stage": now, "t_start": now, "job": "job-a"}
        other = dict(dead, rank=2, error="other job", job="job-b")
        (tmp_path / "rank1.json").write_text(json.dumps(dead))
        (tmp_path / "rank2.json").write_text(json.dumps(other))
        assert [r["error"] for r in g._peer_records()] == ["exited peer"]
    finally:
        g._closed = True
