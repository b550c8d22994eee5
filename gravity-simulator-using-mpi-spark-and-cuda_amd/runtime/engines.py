"""Execution engines behind the Simulation driver.

Both engines expose the same small interface (load / init_ics / step / sync / state / accel /
nonfinite / close) and the same canonical layout, so the driver, the tests and the CLI do not
care where the bodies live.

* HipEngine — the native GPU Stepper (csrc/hip/stepper.hip): device-resident state, gfx950
  force kernels with the KD integrate fused in, hipGraph replay, RCCL all-gather for P > 1.
  Replaces cuda.cu:145-167 (per-step kernel + sync + D2H + host update).
* CpuEngine — the native C++/OpenMP engine (csrc/cpu/cpu_engine.cpp) with a gloo all-gather
  for P > 1. Replaces mpi.c:189-237's step loop (with Jacobi semantics) and pyspark.py's
  driver-side reduce/update (pyspark.py:59-102).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from ..config import SimConfig
from ..models.initial_conditions import DEVICE_IC_IDS, BodySet, make, solar_random, random_cube
from ..ops import _native
from ..parallel import comm
from ..parallel.partition import Layout, layout as make_layout


def _gs_config(cfg: SimConfig, rank: int, nranks: int, device: int) -> _native.GsConfig:
    return _native.GsConfig(
        n=cfg.n, dtype=_native.GS_FP64 if cfg.dtype == "fp64" else _native.GS_FP32,
        kernel=_native.KERNEL_IDS[cfg.kernel], mode=_native.MODE_IDS[cfg.mode], ipl=cfg.ipl,
        chunk=cfg.chunk, rank=rank, nranks=nranks, device=device,
        use_graph=(2 if cfg.graph_comm else 1) if cfg.graph else 0,
        split_groups=cfg.split_groups, cutoff_mode=_native.CUTOFF_IDS[cfg.cutoff_mode],
        strategy=_native.STRATEGY_IDS[cfg.strategy], dt=cfg.dt,
        G=cfg.G, cutoff=cfg.cutoff, softening=cfg.softening)


def gpu_available() -> bool:
    try:
        import torch

        if not torch.cuda.is_available():
            return False
        return _native.hip_lib().gs_hip_device_count() > 0
    except Exception:
        return False


class HipEngine:
    """GPU engine: one native gs_stepper per process (or per virtual rank)."""

    kind = "gpu"

    def __init__(self, cfg: SimConfig, rank: int = 0, nranks: int = 1, device: int = 0,
                 dist: Optional[comm.DistInfo] = None):
        self.cfg = cfg
        self.rank, self.nranks, self.device = rank, nranks, device
        self.dist = dist
        self.lib = _native.hip_lib()
        c = _gs_config(cfg, rank, nranks, device)
        self._s = ctypes.c_void_p()
        _native.check(self.lib, self.lib.gs_stepper_create(ctypes.byref(c), ctypes.byref(self._s)),
                      "gs_stepper_create")
        L = _native.GsLayout()
        _native.check(self.lib, self.lib.gs_stepper_layout(self._s, ctypes.byref(L)), "layout")
        self.native_layout = L.as_dict()
        # P > 1: a progress bound from the start (the RCCL warm-up included); a derived
        # timeout (cfg None) starts at the start-up budget until a step has been measured
        if nranks > 1:
            from ..parallel.guard import INIT_TIMEOUT_S

            self.step_timeout_s = (INIT_TIMEOUT_S if cfg.step_timeout_s is None
                                   else float(cfg.step_timeout_s))
        else:
            self.step_timeout_s = 0.0
        if self.step_timeout_s:
            self.lib.gs_stepper_set_timeout(self._s, self.step_timeout_s)
        if cfg.overlap >= 0:
            self.set_overlap(cfg.overlap)
        self.layout: Layout = make_layout(cfg.n, rank, nranks, L.chunk,
                                          sym=L.mode == _native.MODE_IDS["sym"])
        assert self.layout.n_pad == L.n_pad, "Python layout mirror disagrees with native"
        self.mass: Optional[np.ndarray] = None

    # -- communicator ---------------------------------------------------------------------
    def comm_init(self, uid: bytes) -> None:
        buf = ctypes.create_string_buffer(uid, 128)
        _native.check(self.lib, self.lib.gs_stepper_comm_init(self._s, buf, self.rank,
                                                              self.nranks), "comm_init")

    @staticmethod
    def unique_id() -> bytes:
        lib = _native.hip_lib()
        buf = ctypes.create_string_buffer(128)
        _native.check(lib, lib.gs_rccl_unique_id(buf), "rccl unique id")
        return buf.raw

    def comm_info(self) -> dict:
        """What RCCL formed for this rank (ncclCommCount / UserRank / CuDevice, checked
        natively at comm_init): rccl_nranks 0 when no communicator is kept (one rank)."""
        if not hasattr(self.lib, "gs_stepper_comm_info"):  # (round-5 builds for A/B runs)
            return {"rccl_nranks": None, "rccl_rank": None, "rccl_device": None}
        c, r, d = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _native.check(self.lib, self.lib.gs_stepper_comm_info(
            self._s, ctypes.byref(c), ctypes.byref(r), ctypes.byref(d)), "comm info")
        return {"rccl_nranks": c.value, "rccl_rank": r.value, "rccl_device": d.value}

    def comm_check(self) -> None:
        _native.check(self.lib, self.lib.gs_stepper_comm_check(self._s), "rccl health")

    COMM_STAGES = {0: "not started", 1: "in ncclCommInitRank", 2: "warm-up all-gather",
                   3: "warm-up ring send/recv", 4: "warm-up peer send/recv",
                   5: "waiting for the warm-up", 6: "done", -1: "aborted"}

    def comm_stage(self) -> str:
        """How far comm_init got (safe from a watchdog thread while comm_init blocks)."""
        if not self._s:
            return "no stepper"
        return self.COMM_STAGES.get(int(self.lib.gs_stepper_comm_stage(self._s)), "?")

    def abort(self) -> bool:
        """ncclCommAbort the live communicator once (from a watchdog thread: unblocks
        collectives that will never complete). True if one was aborted."""
        return bool(self._s) and bool(self.lib.gs_stepper_abort(self._s))

    def set_step_timeout(self, seconds: float) -> None:
        """Native progress bound of sync() and of the host running ahead: abort RCCL when no
        enqueued step completes for this long (0: unbounded)."""
        self.step_timeout_s = float(seconds)
        self.lib.gs_stepper_set_timeout(self._s, float(seconds))

    # -- state ----------------------------------------------------------------------------
    def init_ics(self, family: str, seed: int) -> None:
        if family in DEVICE_IC_IDS:
            _native.check(self.lib, self.lib.gs_stepper_init_ics(self._s, DEVICE_IC_IDS[family],
                                                                 seed), "init_ics")
            self.mass = None
        else:
            self.load(make(family, self.cfg.n, seed, self.cfg.G))

    def load(self, b: BodySet) -> None:
        pos = np.ascontiguousarray(b.pos, dtype=np.float64)
        vel = np.ascontiguousarray(b.vel, dtype=np.float64)
        mass = np.ascontiguousarray(b.mass, dtype=np.float64)
        _native.check(self.lib, self.lib.gs_stepper_set_state(
            self._s, _native.dptr(pos), _native.dptr(vel), _native.dptr(mass)), "set_state")
        self.mass = mass

    def step(self, n: int) -> None:
        if n > 0:
            _native.check(self.lib, self.lib.gs_stepper_step(self._s, int(n)), "step")

    def sync(self, timeout_s: float = 0.0) -> None:
        """Wait for the enqueued steps. With a timeout (or the engine's step timeout: P > 1
        cfg.step_timeout_s, or set_step_timeout) the wait polls RCCL async errors and aborts the
        communicator when no step completes for that long (it bounds progress, not the length
        of the run). One rank without a timeout passed here waits with a blocking stream sync:
        there is no collective to hang on, and the poll's 200 us sleep would land inside a
        timed region (up to 2.7 % of a 10-step 65K run); the run guard's stage
        deadline still bounds it."""
        if timeout_s <= 0:
            timeout_s = self.step_timeout_s if self.nranks > 1 else 0.0
        if timeout_s > 0:
            _native.check(self.lib, self.lib.gs_stepper_wait(self._s, timeout_s), "wait")
        else:
            _native.check(self.lib, self.lib.gs_stepper_sync(self._s), "sync")

    # -- phase timing / schedule knobs ------------------------------------------------------
    def set_timing(self, on: bool) -> None:
        """Eager steps record per-step phase events while on (graph replay pauses)."""
        _native.check(self.lib, self.lib.gs_stepper_set_timing(self._s, int(bool(on))), "timing")

    def phase_stats(self) -> dict:
        """Per-step averages over the timed steps since set_timing(True) / the last call.
        comm_ms: the step's collectives on the comm stream (all-gather + node-sum exchange);
        exposed_comm_ms: how long the compute stream stalled on them; deferred_units: the
        most force units a step had to run after the gather (overlap 3)."""
        out = (ctypes.c_double * 8)()
        _native.check(self.lib, self.lib.gs_stepper_phase_stats(self._s, out), "phase stats")
        v = list(out)
        steps, planned = int(v[0]), int(v[7])
        # how the timed steps ran: replayed (one rank: the step graph; several: the segmented
        # plan), eagerly, or both (a step count that is not a whole number of two-step periods)
        rep = "segmented" if self.nranks > 1 else "graph"
        graph = (rep if planned == steps else "eager" if planned == 0 else
                 f"{rep} ({planned} of {steps} steps)") if steps else None
        return {"steps": steps, "step_ms": v[1], "gather_ms": v[2], "exchange_ms": v[3],
                "exposed_gather_ms": v[4], "exposed_exchange_ms": v[5],
                "deferred_units": int(v[6]), "comm_ms": v[2] + v[3],
                "exposed_comm_ms": v[4] + v[5], "graph": graph}

    def sym_geometry(self) -> tuple[int, int, int, int]:
        """(S shell segments, D diagonal parts, Kr split segments, Np parts per split segment)
        per chunk row of the sym schedule: a step runs rows x (S + D + (Np - 1) Kr) units on a
        rank (the work audit)."""
        n_pad = int(self.native_layout["n_pad"])
        v = [ctypes.c_int32() for _ in range(5)]
        self.lib.gs_sym_geometry(n_pad, *[ctypes.byref(x) for x in v])
        parts = (int(self.lib.gs_sym_split_parts(n_pad))
                 if hasattr(self.lib, "gs_sym_split_parts") else 2)  # (pre-round-4 builds: 2)
        return (int(v[3].value), int(v[4].value), int(self.lib.gs_sym_split_segments(n_pad)),
                parts)

    def unit_trace(self) -> np.ndarray:
        """(entries, 4) uint64 timeline of the last sym force launch (GRAVSIM_UNIT_TRACE set
        at creation): start, end (100 MHz ticks), HW_ID | XCC_ID << 32, row << 32 | segment.
        Empty when tracing is off."""
        cap = int(self.lib.gs_stepper_unit_trace(self._s, None, 0))
        out = np.zeros((max(cap, 0), 4), dtype=np.uint64)
        if cap > 0:
            got = int(self.lib.gs_stepper_unit_trace(self._s, out.ctypes.data, cap))
            if got < 0:
                _native.check(self.lib, -1, "unit_trace")
            out = out[:got]
        return out

    def set_overlap(self, mode: int) -> None:
        """Sym-schedule work beside the all-gather (0 wait, 3 gated local-first launch, the
        native default for P > 1; see gravsim.h)."""
        _native.check(self.lib, self.lib.gs_stepper_set_overlap(self._s, int(mode)), "overlap")

    @property
    def overlap(self) -> int:
        """The sym schedule's overlap mode in force (3 by default for P > 1)."""
        return int(self.lib.gs_stepper_get_overlap(self._s))

    @property
    def dyn_cap(self) -> int:
        """Units a dynamic-fetch workgroup may take after the first wave (<= 1: static)."""
        return int(self.lib.gs_stepper_get_dyn_cap(self._s))

    def set_schedule(self, graph: int, dyn_cap: int = -1) -> None:
        """graph: 0 eager, 1 single-rank hipGraph replay, 2 multi-rank capture too;
        dyn_cap: <= 1 static force units (one per workgroup), > 1 dynamic unit fetch,
        < 0 unchanged. Same bits in every combination (an independent schedule for audits)."""
        _native.check(self.lib, self.lib.gs_stepper_set_schedule(self._s, int(graph),
                                                                 int(dyn_cap)), "schedule")

    def set_tuning(self, first_wave: int = 0, fused_tail: int = -1, persist: int = -1) -> None:
        """Test / A-B tuning of the sym schedule, same bits either way: first_wave > 0 sets
        how many workgroups of a dynamic launch take one unit each (default: the resident
        slots); fused_tail 1 / 0 forces the one-rank fused reduction tail / the three-kernel
        tail (default -1: fused up to 256K bodies); persist 1 / 0: one-rank launches with
        persistent workgroups (the default) / workgroups that exit after their cap."""
        _native.check(self.lib, self.lib.gs_stepper_set_tuning(self._s, int(first_wave),
                                                               int(fused_tail)), "tuning")
        if persist >= 0:
            if not hasattr(self.lib, "gs_stepper_set_persist"):
                raise RuntimeError("set_tuning(persist=...): this native build has no persist mode")
            _native.check(self.lib, self.lib.gs_stepper_set_persist(self._s, int(persist)),
                          "persist")

    def set_cutoff_mode(self, mode: str) -> None:
        """Re-resolve the force path: auto | exact (reference hard-cutoff select) | fast."""
        _native.check(self.lib, self.lib.gs_stepper_set_cutoff_mode(
            self._s, _native.CUTOFF_IDS[mode]), "cutoff mode")

    def audit(self) -> tuple[int, int]:
        """(force units completed since the last audit_reset, units per step on this rank);
        (0, 0) for the one-sided schedules, which have no unit audit. Waits for the GPU."""
        done, per = ctypes.c_uint64(), ctypes.c_uint64()
        _native.check(self.lib, self.lib.gs_stepper_audit(self._s, ctypes.byref(done),
                                                          ctypes.byref(per)), "audit")
        return int(done.value), int(per.value)

    def graph_info(self) -> dict:
        """How replayed steps run: eager, one graph per two steps, or a segmented plan
        (multi-rank: compute segments as graphs, collectives eagerly between them)."""
        m, n = ctypes.c_int32(), ctypes.c_int32()
        self.lib.gs_stepper_graph_info(self._s, ctypes.byref(m), ctypes.byref(n))
        out = {"mode": ("eager", "graph", "segmented")[m.value], "segments": n.value}
        if hasattr(self.lib, "gs_stepper_graph_steps"):  # (older builds for A/B runs: absent)
            out["steps_per_launch"] = int(self.lib.gs_stepper_graph_steps(self._s))
        return out

    def mem_info(self) -> dict:
        """HBM this rank's stepper holds, by buffer (bytes), from its allocation ledger (RCCL's
        own buffers are not included)."""
        tag, nb = ctypes.c_char_p(), ctypes.c_uint64()
        n = self.lib.gs_stepper_mem_entry(self._s, -1, None, None)
        out: dict = {}
        for i in range(max(n, 0)):
            self.lib.gs_stepper_mem_entry(self._s, i, ctypes.byref(tag), ctypes.byref(nb))
            out[tag.value.decode()] = out.get(tag.value.decode(), 0) + int(nb.value)
        return out

    def clock(self) -> dict:
        """Engine clock of the sym force launches since the last call (then reset): each
        workgroup's s_memtime span against its s_memrealtime span. ghz: the duration-weighted
        shader clock; wg_cycles: workgroup shader-cycles (a cost independent of the DVFS
        state); wg_seconds, workgroups. Zeros for the one-sided schedules. Waits for the GPU."""
        out = (ctypes.c_double * 4)()
        if hasattr(self.lib, "gs_stepper_clock"):  # (round-5 builds for A/B runs: zeros)
            _native.check(self.lib, self.lib.gs_stepper_clock(self._s, out), "clock")
        return {"ghz": out[0], "wg_cycles": out[1], "wg_seconds": out[2],
                "workgroups": int(out[3])}

    def audit_reset(self) -> None:
        _native.check(self.lib, self.lib.gs_stepper_audit_reset(self._s), "audit reset")

    def state(self) -> BodySet:
        """Full positions (collective for P > 1), own velocity rows, masses."""
        n = self.cfg.n
        pos = np.zeros((n, 3))
        vel = np.zeros((n, 3))
        mass = np.zeros(n)
        _native.check(self.lib, self.lib.gs_stepper_get_state(
            self._s, _native.dptr(pos), _native.dptr(vel), _native.dptr(mass)), "get_state")
        return BodySet(pos, vel, mass)

    def accel(self, step_path: bool = False) -> np.ndarray:
        """(n_local, 4) = (ax, ay, az, phi) of this rank's rows (ghost rows included).
        step_path=True evaluates the integrator's own force path (configured kernel and
        cutoff mode; phi column 0) instead of the exact-cutoff diagnostic path."""
        out = np.zeros((self.layout.n_local, 4))
        fn = self.lib.gs_stepper_accel_step_path if step_path else self.lib.gs_stepper_accel
        _native.check(self.lib, fn(self._s, _native.dptr(out)), "accel")
        return out

    def nonfinite(self) -> int:
        r = int(self.lib.gs_stepper_count_nonfinite(self._s))
        if r < 0:
            raise RuntimeError("nonfinite check failed: " + self.lib.gs_last_error().decode())
        return r

    @property
    def steps_done(self) -> int:
        return int(self.lib.gs_stepper_steps_done(self._s))

    def align_period(self) -> int:
        """Step (0, 1 or 2 steps) until the next step starts a replayable two-step period, so
        that the following steps run from the step graph / segmented plan, not eagerly (a
        state read gathers the current buffer; an odd step count ends mid-period). Returns
        the steps taken."""
        n = 0
        while not self.lib.gs_stepper_period_start(self._s) and n < 2:
            self.step(1)
            n += 1
        return n

    def force_mode(self) -> dict:
        """Resolved force path: exact hard-cutoff select, or the fast core-softened path."""
        ex, e2 = ctypes.c_int32(), ctypes.c_double()
        self.lib.gs_stepper_force_mode(self._s, ctypes.byref(ex), ctypes.byref(e2))
        return {"exact": bool(ex.value), "eps2": e2.value}

    def close(self) -> None:
        if self._s:
            self.lib.gs_stepper_destroy(self._s)
            self._s = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class CpuEngine:
    """Native CPU engine; P > 1 exchanges position slices with a gloo all-gather."""

    kind = "cpu"

    def __init__(self, cfg: SimConfig, rank: int = 0, nranks: int = 1,
                 dist: Optional[comm.DistInfo] = None):
        self.cfg = cfg
        self.rank, self.nranks = rank, nranks
        self.dist = dist or comm.DistInfo(rank=rank, world=nranks)
        self.lib = _native.cpu_lib()
        self.layout: Layout = make_layout(cfg.n, rank, nranks, cfg.chunk)
        self.np_dtype = np.float64 if cfg.dtype == "fp64" else np.float32
        L = self.layout
        self.X = [np.zeros((L.n_pad, 4), self.np_dtype), np.zeros((L.n_pad, 4), self.np_dtype)]
        self.V = np.zeros((L.n_local, 4), self.np_dtype)
        self.k = 0
        self.mass = np.zeros(cfg.n)
        suf = "f64" if cfg.dtype == "fp64" else "f32"
        self._step = getattr(self.lib, f"gs_cpu_step_{suf}")
        self._accel = getattr(self.lib, f"gs_cpu_accel_{suf}")
        self._ptr = _native.dptr if cfg.dtype == "fp64" else _native.fptr
        if cfg.threads:
            self.lib.gs_cpu_set_threads(int(cfg.threads))

    def init_ics(self, family: str, seed: int) -> None:
        n, L = self.cfg.n, self.layout
        if family == "solar+random":
            b = solar_random(n, seed)
        elif family == "random":
            b = random_cube(n, seed)
        else:
            b = make(family, n, seed, self.cfg.G)
        self.load(b)

    def load(self, b: BodySet) -> None:
        L, n = self.layout, self.cfg.n
        X = self.X[0]
        X[:] = 0
        X[:n, :3] = b.pos
        X[:n, 3] = self.cfg.G * b.mass
        self.V[:] = 0
        rows = L.real_local
        if len(rows):
            self.V[: len(rows), :3] = b.vel[rows.start:rows.stop]
        self.mass = np.array(b.mass, dtype=np.float64)
        self.k = 0

    def step(self, n: int) -> None:
        L = self.layout
        T = self.np_dtype
        cut2 = T(self.cfg.cutoff ** 2)
        eps2 = T(self.cfg.softening ** 2)
        for _ in range(int(n)):
            cur, nxt = self.X[self.k & 1], self.X[(self.k + 1) & 1]
            rc = self._step(self._ptr(cur), self._ptr(nxt), self._ptr(self.V), L.n,
                            L.local_begin, L.local_end, L.chunk, T(self.cfg.dt), cut2, eps2)
            _native.check(self.lib, rc, "cpu step")
            comm.allgather_rows(self.dist, nxt, L.local_begin, L.n_local)
            self.k += 1

    def sync(self) -> None:
        pass

    def state(self) -> BodySet:
        n, L = self.cfg.n, self.layout
        X = self.X[self.k & 1]
        pos = X[:n, :3].astype(np.float64)
        vel = np.zeros((n, 3))
        rows = L.real_local
        if len(rows):
            vel[rows.start:rows.stop] = self.V[: len(rows), :3]
        return BodySet(pos, vel, self.mass.copy())

    def accel(self) -> np.ndarray:
        L = self.layout
        T = self.np_dtype
        out = np.zeros((L.n_local, 4), T)
        rc = self._accel(self._ptr(self.X[self.k & 1]), L.n, L.local_begin, L.local_end, L.chunk,
                         T(self.cfg.cutoff ** 2), T(self.cfg.softening ** 2), self._ptr(out))
        _native.check(self.lib, rc, "cpu accel")
        return out.astype(np.float64)

    def nonfinite(self) -> int:
        L = self.layout
        X = self.X[self.k & 1][L.local_begin:L.local_end, :3]
        return int((~np.isfinite(X)).sum() + (~np.isfinite(self.V[:, :3])).sum())

    @property
    def steps_done(self) -> int:
        return self.k

    def close(self) -> None:
        pass


class VirtualGroup:
    """P virtual ranks (one HipEngine each, rank r of P) on one device, stepped in lockstep by
    the native gs_group_step: the RCCL schedule with the all-gather done by device copies."""

    def __init__(self, cfg: SimConfig, nranks: int, device: int = 0):
        self.cfg = cfg
        self.shards = [HipEngine(cfg, r, nranks, device) for r in range(nranks)]
        self.lib = self.shards[0].lib

    def init_ics(self, family: str, seed: int) -> None:
        for s in self.shards:
            s.init_ics(family, seed)

    def load(self, b: BodySet) -> None:
        for s in self.shards:
            s.load(b)

    def step(self, n: int) -> None:
        arr = (ctypes.c_void_p * len(self.shards))(*[s._s.value for s in self.shards])
        _native.check(self.lib, self.lib.gs_group_step(arr, len(self.shards), int(n)),
                      "group_step")

    def sync(self) -> None:
        for s in self.shards:
            s.sync()

    def state(self) -> BodySet:
        """Assemble the global state from each shard's own rows."""
        n = self.cfg.n
        pos = np.zeros((n, 3))
        vel = np.zeros((n, 3))
        mass = None
        for s in self.shards:
            b = s.state()
            rows = s.layout.real_local
            if len(rows):
                pos[rows.start:rows.stop] = b.pos[rows.start:rows.stop]
                vel[rows.start:rows.stop] = b.vel[rows.start:rows.stop]
            mass = b.mass
        return BodySet(pos, vel, mass)

    def close(self) -> None:
        for s in self.shards:
            s.close()
