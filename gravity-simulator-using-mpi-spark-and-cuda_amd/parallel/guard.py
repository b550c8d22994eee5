"""Bounded, self-reporting runs: a per-rank watchdog thread with stage deadlines.

The reference has no failure handling at all: MPI's default MPI_ERRORS_ARE_FATAL and a
blocking MPI_Allgatherv + MPI_Barrier every step (mpi.c:142-144, 227-236), unchecked CUDA
calls (cuda.cu:145-160). A rank that stalls there hangs the whole job until something outside
kills it, and nothing records where it stopped. Here every rank of bench.py / the CLI runs a
RunGuard:

* The run is cut into named stages (gloo_init, engine, comm_init, warmup, timed, audits...),
  each with a deadline. A daemon thread checks it every 0.25 s; the blocking native calls
  (ctypes releases the GIL) and gloo waits do not stop it.
* Each rank keeps a small JSON record (stage, status, device, error) in a per-job directory
  shared by the ranks of the node (GRAVSIM_GUARD_DIR, else /tmp/gravsim_job_<launcher pid>_
  <MASTER_PORT>), and routes RCCL's INFO log there, so rank 0 can report every rank's stage
  and RCCL transports without any collective (a stalled job cannot run one).
* On a missed deadline, or a failure a rank records (an exception, the native step timeout's
  RCCL abort), rank 0 prints ONE error JSON line (the caller's `report` builds it: for
  bench.py the metric line with "status": "error", the stage and the per-rank records),
  aborts its RCCL communicator and exits with EXIT_CODE; the other ranks record their state,
  wait briefly for rank 0's report, abort and exit too. Nothing is re-exec'ed.
* Test hook: GRAVSIM_TEST_STALL="<stage>@<rank>:<seconds>" makes that rank sleep when it
  enters that stage (tests/test_guard_gpu.py injects stalls into comm init and into a step).
"""
from __future__ import annotations

import json
import os
import re
import sys
import tempfile
import threading
import time
from typing import Callable, Optional

EXIT_CODE = 70  # EX_SOFTWARE: the run was stopped by its own guard
INIT_TIMEOUT_S = 180.0  # default budget of each start-up stage (gloo, engine, RCCL init)


def job_dir(rank: int = 0, world: int = 1) -> str:
    """Directory shared by the ranks of one job on this node."""
    d = os.environ.get("GRAVSIM_GUARD_DIR")
    if not d:
        # torchrun's ranks share their parent (the elastic agent) and MASTER_PORT; a single
        # process keys on its own pid
        # (plus torchrun's rendezvous run id when it names the job: a directory reused by an
        # earlier job of the same parent pid and port cannot leak its records into this one)
        run_id = os.environ.get("TORCHELASTIC_RUN_ID", "none")
        tag = (f"{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}" if world > 1
               else f"{os.getpid()}_single")
        if world > 1 and run_id not in ("", "none"):
            tag += "_" + re.sub(r"[^\w.-]", "_", run_id)[:40]
        d = os.path.join(tempfile.gettempdir(), f"gravsim_job_{tag}")
    os.makedirs(d, exist_ok=True)
    return d


def parse_rccl_log(path: Optional[str]) -> dict:
    """Transports of a rank's RCCL connections ("P2P/IPC", "NET/Socket", "SHM"...), the RCCL
    version and the network plugin, from its INFO log (NCCL_DEBUG_SUBSYS=INIT,P2P,NET)."""
    out = {"transports": None, "rccl_version": None, "net": None}
    if not path or not os.path.exists(path):
        out["rccl_log"] = f"no RCCL log at {path}" if path else "not routed"
        return out
    seen, net, lines = set(), set(), 0
    with open(path, errors="replace") as f:
        for line in f:
            lines += 1
            m = re.search(r" via (\S+)", line)
            if m and "Channel" in line:
                seen.add(re.sub(r"/\d+$", "", m.group(1)))
            m = re.search(r"(?:RCCL|NCCL) version[ :]+(\S+)", line)
            if m and out["rccl_version"] is None:
                out["rccl_version"] = m.group(1)
            m = re.search(r"Using network (\S+)", line)
            if m:
                net.add(m.group(1))
    out["transports"] = sorted(seen)
    out["net"] = sorted(net) or None
    out["rccl_log"] = f"{lines} lines"
    return out


class RunGuard:
    """Per-rank stage watchdog (see the module docstring). `report(reason, records)` returns
    the dict rank 0 prints as its JSON line when the run is stopped."""

    def __init__(self, rank: int, world: int, report: Callable[[str, list], dict],
                 directory: Optional[str] = None, poll_s: float = 0.25, ack_wait_s: float = 10.0,
                 out=None):
        self.rank, self.world = rank, world
        self.dir = directory or job_dir(rank, world)
        self.report = report
        self.poll_s, self.ack_wait_s = poll_s, ack_wait_s
        self.out = out  # stream of rank 0's JSON line (default: file descriptor 1)
        self.t_start = time.time()
        self.job = job_id()
        self.rec: dict = {"rank": rank, "pid": os.getpid(), "stage": "start", "status": "running",
                          "t_stage": self.t_start, "t_start": self.t_start, "job": self.job}
        self._deadline: Optional[float] = None
        self._aborts: list[Callable[[], None]] = []
        self._probes: list[Callable[[], dict]] = []
        self._lock = threading.Lock()
        self._fired = False
        self._closed = False
        self._ack = os.path.join(self.dir, "reported")
        if rank == 0 and os.path.exists(self._ack):
            os.remove(self._ack)  # (a directory reused by an earlier job of the same tag)
        self._write()
        self._thread = threading.Thread(target=self._loop, name="gravsim-guard", daemon=True)
        self._thread.start()

    # -- stages -----------------------------------------------------------------------------
    def stage(self, name: str, budget_s: Optional[float], **info) -> None:
        """Enter stage `name`, which must end within budget_s seconds (None: unbounded)."""
        with self._lock:
            self.rec.update(info)
            self.rec.update(stage=name, budget_s=budget_s, t_stage=time.time())
            self._deadline = time.monotonic() + budget_s if budget_s else None
        self._write()
        self._maybe_stall(name)

    def note(self, **info) -> None:
        """Add facts to this rank's record (device, transports...) without a new deadline."""
        with self._lock:
            self.rec.update(info)
        self._write()

    def on_abort(self, fn: Callable[[], None]) -> None:
        """Called (best effort) before the process exits on a stop: e.g. ncclCommAbort."""
        self._aborts.append(fn)

    def probe(self, fn: Callable[[], dict]) -> None:
        """Called when the guard fires; its dict is merged into this rank's record (e.g. the
        native communicator's init stage)."""
        self._probes.append(fn)

    def fail(self, error: str) -> None:
        """A failure on this rank (an exception): record it, stop the job, exit. Never returns."""
        with self._lock:
            self.rec.update(status="failed", error=error[:2000])
        self._write()
        self._fire(f"rank {self.rank} failed in stage {self.rec['stage']}: {error[:500]}")
        time.sleep(30.0)  # (reached only while the guard thread is already stopping the run)
        os._exit(EXIT_CODE)

    def close(self) -> None:
        """Normal end: disarm and drop this rank's record."""
        with self._lock:
            self._closed = True
            self._deadline = None
        for p in (self._path(self.rank), self.rec.get("rccl_log_path")):
            try:
                if p:
                    os.remove(p)  # (RCCL may still hold its log open: unlinking is fine)
            except OSError:
                pass
        if self.rank == 0:
            try:
                os.rmdir(self.dir)  # only when every rank has removed its record
            except OSError:
                pass

    # -- internals --------------------------------------------------------------------------
    def _path(self, r: int) -> str:
        return os.path.join(self.dir, f"rank{r}.json")

    def _write(self) -> None:
        p = self._path(self.rank)
        tmp = f"{p}.{os.getpid()}.tmp"
        try:
            with open(tmp, "w") as f:
                json.dump(self.rec, f, default=str)
            os.replace(tmp, p)
        except OSError:
            pass

    def records(self) -> list[dict]:
        out = []
        for r in range(self.world):
            try:
                with open(self._path(r)) as f:
                    rec = json.load(f)
            except (OSError, ValueError):
                rec = {"rank": r, "stage": None, "status": "no record"}
            if rec.get("t_stage"):
                rec["in_stage_s"] = round(time.time() - float(rec["t_stage"]), 1)
            rec.update(parse_rccl_log(rec.pop("rccl_log_path", None)))
            out.append(rec)
        return out

    def _maybe_stall(self, name: str) -> None:
        spec = os.environ.get("GRAVSIM_TEST_STALL", "")
        m = re.fullmatch(r"([\w.-]+)@(\d+):([\d.]+)", spec)
        if m and m.group(1) == name and int(m.group(2)) == self.rank:
            time.sleep(float(m.group(3)))

    def _loop(self) -> None:
        while True:
            time.sleep(self.poll_s)
            with self._lock:
                if self._closed:
                    return
                late = self._deadline is not None and time.monotonic() > self._deadline
                stage, budget = self.rec["stage"], self.rec.get("budget_s")
            if late:
                with self._lock:
                    self.rec.update(status="timeout",
                                    error=f"stage {stage} exceeded its {budget} s budget")
                self._write()
                self._fire(f"rank {self.rank}: stage {stage} exceeded its {budget} s budget")
            if self.rank == 0 and self.world > 1:
                for rec in self._peer_records():
                    if rec.get("status") in ("failed", "timeout"):
                        self._fire(f"rank {rec['rank']} {rec['status']} in stage "
                                   f"{rec.get('stage')}: {rec.get('error', '')[:500]}")

    def _peer_records(self) -> list[dict]:
        """Peer records of THIS job: a record left in a reused directory by an earlier job (a
        different job id, or started long before this guard) is ignored until the peer of this
        job overwrites it, so it cannot fire a false error. Whether the peer's
        process is still alive does not matter: a peer of this job that recorded "failed" or
        "timeout" and exited is still reported, and with a GRAVSIM_GUARD_DIR shared across
        nodes a remote pid says nothing at all."""
        out = []
        for r in range(1, self.world):
            try:
                with open(self._path(r)) as f:
                    rec = json.load(f)
            except (OSError, ValueError):
                continue
            same_job = not (self.job and rec.get("job")) or rec.get("job") == self.job
            if same_job and float(rec.get("t_start") or 0.0) >= self.t_start - STALE_RECORD_S:
                out.append(rec)
        return out

    def _await_peers(self) -> None:
        """Before rank 0 reports: give peers that have not ended in failed / timeout up to
        PEER_GRACE_S to get there, so a failure every rank meets (no GPU, a bad device) shows
        every rank's own error rather than whichever stage the slower ranks were entering."""
        t_end = time.monotonic() + PEER_GRACE_S
        while time.monotonic() < t_end:
            done = {r["rank"] for r in self._peer_records()
                    if r.get("status") in ("failed", "timeout") and "rank" in r}
            if len(done) >= self.world - 1:
                return
            time.sleep(0.1)

    def _fire(self, reason: str) -> None:
        with self._lock:
            if self._fired or self._closed:
                return
            self._fired = True
        for fn in self._probes:
            try:
                with self._lock:
                    self.rec.update(fn())
            except Exception as e:  # noqa: BLE001 - best effort while stopping
                self.rec["probe_error"] = repr(e)
        self._write()
        if self.rank == 0:
            self._await_peers()
            try:
                line = json.dumps(self.report(reason, self.records()), default=str)
            except Exception as e:  # noqa: BLE001
                line = json.dumps({"status": "error", "error": reason, "report_error": repr(e)})
            try:
                sys.stdout.flush()
            except Exception:  # noqa: BLE001
                pass
            if self.out is not None:
                self.out.write(line + "\n")
                self.out.flush()
            else:
                os.write(1, (line + "\n").encode())
            try:
                open(self._ack, "w").close()
            except OSError:
                pass
        else:
            sys.stderr.write(f"gravsim guard: {reason}\n")
            sys.stderr.flush()
            t_end = time.monotonic() + self.ack_wait_s  # let rank 0 read this record first
            while time.monotonic() < t_end and not os.path.exists(self._ack):
                time.sleep(0.1)
        for fn in self._aborts:
            try:
                fn()
            except Exception:  # noqa: BLE001
                pass
        os._exit(EXIT_CODE)


# A peer record whose guard started this long before rank 0's belongs to an earlier job (the
# ranks of one job start their guards within seconds of each other).
STALE_RECORD_S = 120.0
# How long rank 0 waits, once the run is being stopped, for the other ranks' records to show
# how they ended (a stalled peer never does: the report then goes out after this).
PEER_GRACE_S = 2.0


def job_id() -> str:
    """Identity of the job every rank of it shares: torchrun's rendezvous run id when it names
    one, else the rendezvous endpoint (MASTER_ADDR:MASTER_PORT); GRAVSIM_JOB_ID overrides.
    "" when none is known (a single process): records are then filtered by start time only."""
    if os.environ.get("GRAVSIM_JOB_ID"):
        return os.environ["GRAVSIM_JOB_ID"]
    run_id = os.environ.get("TORCHELASTIC_RUN_ID", "")
    if run_id not in ("", "none"):
        return run_id
    if os.environ.get("MASTER_PORT"):
        return f"{os.environ.get('MASTER_ADDR', '')}:{os.environ['MASTER_PORT']}"
    return ""


STEP_TIMEOUT_FLOOR_S = 60.0
STEP_TIMEOUT_CAP_S = 240.0  # well under the driver's 600 s bench limit


def step_timeout(step_s: float, floor_s: float = STEP_TIMEOUT_FLOOR_S,
                 cap_s: float = STEP_TIMEOUT_CAP_S) -> float:
    """Native progress bound for a run whose steps take step_s seconds: max(floor, 20 x step),
    capped (a stalled first 8-GPU run must end, and report, inside the driver's
    own limit)."""
    return min(cap_s, max(floor_s, 20.0 * float(step_s)))
