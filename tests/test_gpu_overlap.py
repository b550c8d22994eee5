"""Comm/compute split and overlap of the multi-rank sym step, measured on one GPU.

Per-rank emulation (GRAVSIM_EMULATE_RANK) runs rank r's exact launch shapes of a P-rank run;
with GRAVSIM_EMU_COMM ("GB/s,latency us") the all-gather and the node-sum exchange become modeled
collectives (comm_model.hip) of their exact byte counts on the comm stream, so the phase
events see what an xGMI collective would cost. The reference times its whole loop, the
MPI_Allgatherv included (mpi.c:189,227-247). Overlap modes (gravsim.h, set_overlap):
0 wait for the gather then one launch, 3 one local-first launch with the remote units gated
in-kernel.
"""
import numpy as np
import pytest

from gravsim.config import SimConfig

pytestmark = pytest.mark.gpu


def _emu(monkeypatch, n, P, rank, gbps, overlap, strategy="allgather", graph=True):
    from gravsim.runtime.engines import HipEngine

    monkeypatch.setenv("GRAVSIM_EMULATE_RANK", "1")
    monkeypatch.setenv("GRAVSIM_EMU_COMM", f"{gbps},15")
    e = HipEngine(SimConfig(n=n, dtype="fp32", device="gpu", mode="sym", strategy=strategy,
                            graph=graph), rank, P)
    e.set_overlap(overlap)
    return e


@pytest.mark.parametrize("strategy,overlap,sync", [("allgather", 3, "flags"),
                                                   ("allgather", 0, "flags"),
                                                   ("allgather", 3, "events"),
                                                   ("ring", 3, "events")])
def test_segmented_plan_matches_eager(hip, monkeypatch, strategy, overlap, sync):
    """Multi-rank steps replay a plan by default: the collectives (here the emulation's modeled
    ones, on a real node RCCL) run eagerly on the comm stream, the compute work is replayed
    from graphs. With flag sync (the all-gather default) the streams order each other through
    device counters and a period is ONE compute graph; with events (GRAVSIM_SYNC=events, and
    the ring) every cross-stream point cuts the period into segments. Same bits as eager steps
    either way, every unit run once per step, and the plan is what ran."""
    if sync == "events":
        monkeypatch.setenv("GRAVSIM_SYNC", "events")
    res = {}
    for graph in (True, False):
        e = _emu(monkeypatch, 262144, 8, 6, 64, overlap, strategy=strategy, graph=graph)
        e.init_ics("solar+random", 2)
        e.audit_reset()
        e.step(6)
        e.sync()
        done, per = e.audit()
        assert done == 6 * per and per > 0
        gi = e.graph_info()
        assert gi["mode"] == ("segmented" if graph else "eager"), gi
        if graph:
            if sync == "flags":
                assert gi["segments"] == 1, gi  # one compute graph per period
            else:
                assert gi["segments"] >= 4, gi
        b = e.state()
        own = e.layout.real_local
        res[graph] = (b.pos[own.start:own.stop].copy(), b.vel[own.start:own.stop].copy())
        e.close()
    assert np.array_equal(res[True][0], res[False][0])
    assert np.array_equal(res[True][1], res[False][1])


def test_counter_collection_selects_event_ordering(hip, monkeypatch):
    """rocprofv3 --pmc serializes dispatches (it exports ROCPROF_COUNTER_COLLECTION): a
    flag-sync wait kernel would wait for a signal queued behind it until the step timeout, so
    the stepper orders its streams with events then (a segmented plan), unless
    GRAVSIM_SYNC=flags says otherwise. Same bits either way."""
    res = {}
    for env in ("", "1"):
        if env:
            monkeypatch.setenv("ROCPROF_COUNTER_COLLECTION", env)
        else:
            monkeypatch.delenv("ROCPROF_COUNTER_COLLECTION", raising=False)
        e = _emu(monkeypatch, 262144, 8, 3, 64, 3)
        e.init_ics("solar+random", 6)
        e.step(4)
        e.sync()
        gi = e.graph_info()
        assert gi["mode"] == "segmented", gi
        assert (gi["segments"] > 1) == bool(env), gi
        b = e.state()
        own = e.layout.real_local
        res[env] = b.pos[own.start:own.stop].copy()
        e.close()
    monkeypatch.delenv("ROCPROF_COUNTER_COLLECTION", raising=False)
    assert np.array_equal(res[""], res["1"])


@pytest.mark.parametrize("P,rank", [(3, 0), (3, 2), (5, 4), (6, 5), (7, 0), (7, 6)])
def test_uneven_rank_emulation_runs(hip, monkeypatch, P, rank):
    """Per-rank emulation of P not dividing the 256 row blocks (1M bodies): rank 0 holds the
    most blocks, the last ranks the fewest and receive the most tree nodes; the modeled
    collectives (gather, node exchange) stay inside their buffers and every unit runs."""
    e = _emu(monkeypatch, 1 << 20, P, rank, 64, 3)
    try:
        e.init_ics("solar+random", 2)
        e.audit_reset()
        e.step(2)
        e.sync()
        done, per = e.audit()
        assert done == 2 * per and per > 0
        assert e.nonfinite() == 0
    finally:
        e.close()


def test_overlap_modes_same_bits(hip, monkeypatch):
    """Every overlap mode computes every unit exactly once into the same slots: the emulated
    rank's state after 4 steps is bitwise identical for modes 0 and 3 (a unit missed by the
    local-first order of mode 3 would leave uninitialised partials behind)."""
    res = []
    for ov in (0, 3):
        e = _emu(monkeypatch, 262144, 8, 5, 64, ov)
        e.init_ics("solar+random", 2)
        e.step(4)
        e.sync()
        b = e.state()
        own = e.layout.real_local
        res.append((b.pos[own.start:own.stop].copy(), b.vel[own.start:own.stop].copy()))
        e.close()
    for pos, vel in res[1:]:
        assert np.array_equal(pos, res[0][0])
        assert np.array_equal(vel, res[0][1])


def test_ring_stages_same_bits_and_defer(hip, monkeypatch):
    """Ring strategy (P-1 modeled neighbour stages, each publishing its own gate): the gated
    launch equals the ungated one bitwise, and with a slow ring (0.05 GB/s per stage) remote
    units wait on their own stage's gate or are deferred, with the same bits."""
    res, deferred = [], []
    for gbps, ov in ((64, 0), (64, 3), (0.05, 3)):
        e = _emu(monkeypatch, 262144, 8, 5, gbps, ov, strategy="ring")
        e.init_ics("solar+random", 2)
        e.step(2)
        e.sync()
        e.set_timing(True)
        e.step(2)
        deferred.append(e.phase_stats()["deferred_units"])
        e.set_timing(False)
        b = e.state()
        own = e.layout.real_local
        res.append((b.pos[own.start:own.stop].copy(), b.vel[own.start:own.stop].copy()))
        e.close()
    for pos, vel in res[1:]:
        assert np.array_equal(pos, res[0][0])
        assert np.array_equal(vel, res[0][1])
    assert deferred[0] == 0 and deferred[2] > 0


def test_phase_split_reports_modeled_comm(hip, monkeypatch):
    """Phase events: the modeled gather (7/8 of 262144 x 16 B = 3.67 MB at 8 GB/s + 15 us =
    474 us) and exchange (the 4 of 7 peers whose node sums can be nonzero, gs_sym_pair_live:
    1.57 MB in two stages, 197 + 2 x 15 = 227 us) show up as comm time; with overlap 0 the compute
    stream stalls for the whole gather. With overlap 3 the local units run beside it, the
    remote units that find it unfinished are deferred to the launch behind the gather event,
    and the step is no slower."""
    out = {}
    for ov in (0, 3):
        e = _emu(monkeypatch, 262144, 8, 7, 8, ov)
        e.init_ics("solar+random", 2)
        e.step(2)
        e.sync()
        e.set_timing(True)
        e.step(4)
        out[ov] = e.phase_stats()
        e.set_timing(False)
        e.close()
    p0, p3 = out[0], out[3]
    for p in (p0, p3):
        assert p["steps"] == 4
        assert p["gather_ms"] > 0.9 * 0.474, p
        assert p["exchange_ms"] > 0.9 * 0.227, p
    assert p0["exposed_gather_ms"] > 0.8 * p0["gather_ms"], p0
    assert p0["deferred_units"] == 0, p0
    assert p3["exposed_gather_ms"] < p0["exposed_gather_ms"], (p0, p3)
    assert p3["step_ms"] < 1.03 * p0["step_ms"], (p0, p3)


def test_slow_gather_defers_remote_units(hip, monkeypatch):
    """A gather far slower than the local work (modeled at 0.01 GB/s: ~92 ms) leaves every
    remote unit deferred; nothing waits on the GPU and the bits equal overlap 0."""
    res, deferred = [], []
    for ov in (0, 3):
        e = _emu(monkeypatch, 65536, 8, 3, 0.01, ov)
        e.init_ics("solar+random", 2)
        e.step(2)
        e.sync()
        e.set_timing(True)
        e.step(2)
        deferred.append(e.phase_stats()["deferred_units"])
        e.set_timing(False)
        b = e.state()
        own = e.layout.real_local
        res.append(b.pos[own.start:own.stop].copy())
        e.close()
    assert np.array_equal(res[0], res[1])
    assert deferred[0] == 0
    assert deferred[1] > 0


def test_long_healthy_run_does_not_trip_step_timeout(hip):
    """The bounded wait bounds progress, not the run: 1500 steps of 65,536 bodies (~1.1 s of
    queued GPU work, far past a 0.3 s budget) complete without a timeout, because one more
    step finishes every ~0.8 ms (a 600 s budget over a whole queued run used to
    abort long healthy multi-rank runs)."""
    from gravsim.runtime.engines import HipEngine

    e = HipEngine(SimConfig(n=65536, dtype="fp32", device="gpu", mode="sym", graph=False))
    try:
        e.lib.gs_stepper_set_timeout(e._s, 0.3)
        e.init_ics("solar+random", 1)
        e.step(1500)
        e.sync(timeout_s=0.3)
        assert e.steps_done == 1500 and e.nonfinite() == 0
    finally:
        e.close()


def test_stalled_step_trips_step_timeout(hip, monkeypatch):
    """A step that cannot finish for ~1.8 s (a modeled gather at 0.0005 GB/s) against a
    0.3 s progress budget: the wait reports a step timeout instead of blocking."""
    e = _emu(monkeypatch, 65536, 8, 3, 0.0005, 0)
    try:
        e.init_ics("solar+random", 2)
        e.step(2)
        with pytest.raises(RuntimeError, match="step timeout: no step completed"):
            e.sync(timeout_s=0.3)
    finally:
        e.close()


def test_device_wait_give_up_fails_sync(hip, monkeypatch):
    """A flag-sync wait kernel that gives up (here its device bound forced to 0.2 s against a
    ~1.8 s modeled gather, the host's own progress bound 30 s) must not let the step finish
    silently on an unfinished gather: it sets the sticky failure word, later waits fall
    through, and sync() raises. Without the bound override the device waits
    outlast the host's timeout (2 x timeout + 10 s), so the host abort wins a stall."""
    monkeypatch.setenv("GRAVSIM_SYNC_LIMIT_S", "0.2")
    e = _emu(monkeypatch, 65536, 8, 3, 0.0005, 0)
    try:
        e.set_step_timeout(30.0)
        e.init_ics("solar+random", 2)
        e.step(2)
        with pytest.raises(RuntimeError, match="flag sync: a cross-stream wait gave up"):
            e.sync()
        with pytest.raises(RuntimeError, match="flag sync"):
            e.state()  # a state the wait gave up on is never returned
    finally:
        e.close()


def test_host_step_timeout_beats_device_wait_bound(hip, monkeypatch):
    """With the default device bound (2 x the step timeout + 10 s) a stalled gather trips the
    host's 0.3 s progress bound first; the host then releases the spinning wait kernels
    (failure word), so close() does not sit out the device bound, and the stepper stays
    failed."""
    import time

    e = _emu(monkeypatch, 65536, 8, 3, 0.0005, 0)
    try:
        e.set_step_timeout(0.3)
        e.init_ics("solar+random", 2)
        e.step(2)
        with pytest.raises(RuntimeError, match="step timeout: no step completed"):
            e.sync()
        with pytest.raises(RuntimeError, match="flag sync"):
            e.sync()
    finally:
        t0 = time.perf_counter()
        e.close()
        assert time.perf_counter() - t0 < 5.0  # the 1.8 s modeled gather, not a 10.6 s wait


def test_per_link_exchange_price(hip, monkeypatch):
    """GRAVSIM_EMU_LINKS=1 prices each exchange stage at its largest single peer's bytes (the
    peers' xGMI links in parallel) instead of all of them through one pipe: at P = 7 (several
    peers per stage) the modeled exchange is shorter; the all-gather's price does not change."""
    out = {}
    for links in ("0", "1"):
        monkeypatch.setenv("GRAVSIM_EMU_LINKS", links)
        e = _emu(monkeypatch, 262144, 7, 3, 8, 3)
        e.init_ics("solar+random", 2)
        e.step(2)
        e.sync()
        e.set_timing(True)
        e.step(4)
        out[links] = e.phase_stats()
        e.set_timing(False)
        e.close()
    monkeypatch.delenv("GRAVSIM_EMU_LINKS", raising=False)
    one, per = out["0"], out["1"]
    assert per["exchange_ms"] < 0.8 * one["exchange_ms"], (one, per)
    assert abs(per["gather_ms"] - one["gather_ms"]) < 0.1 * one["gather_ms"], (one, per)
