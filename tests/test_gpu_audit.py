"""Work audit of the sym force launches and pinned cutoff semantics (GPU).

bench.py must not be able to print a fast headline for steps that skipped work (round 2:
graph replays after the first ran no units until commit 8fdec84). The force kernels count
every unit they run (nbody_sym.hip audit_unit); a step must run rows x (S + D + (Np - 1) Kr)
units per rank (Kr split segments of Np parts per row) whatever the launch split, band count,
fetch order or graph replay. A skipped-unit fault
(GRAVSIM_FAULT_SKIP_UNITS: the dynamic counter starts past 0, the failure class of a stale
re-armed counter) must be caught by bench.py's unit count and by its independent replay.

The reference times its whole loop with the work in it (cuda.cu:154-171, mpi.c:189-247).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

from gravsim.config import SimConfig
from gravsim.models import initial_conditions as ic

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n,dtype,P,band_mb,graph", [
    (65536, "fp32", 1, None, True),     # fused tail re-arms the counter, graph replay
    (65536, "fp32", 1, None, False),    # eager
    (40000, "fp32", 1, "1", True),      # one 2048-body row per band, static launches
    (40000, "fp64", 2, None, False),    # virtual ranks: each shard counts its own rows
])
def test_unit_audit_counts_every_unit(hip, monkeypatch, n, dtype, P, band_mb, graph):
    from gravsim.runtime.engines import VirtualGroup

    if band_mb:
        monkeypatch.setenv("GRAVSIM_SYM_BAND_MB", band_mb)
    g = VirtualGroup(SimConfig(n=n, dtype=dtype, device="gpu", mode="sym", graph=graph), P)
    try:
        g.init_ics("solar+random", 5)
        for s in g.shards:
            s.audit_reset()
        steps = 5
        g.step(steps)
        g.sync()
        per = []
        for s in g.shards:
            done, per_step = s.audit()
            S, D, Kr, Np = s.sym_geometry()
            assert per_step == s.layout.n_local // 2048 * (S + D + (Np - 1) * Kr)
            assert done == per_step * steps, (done, per_step)
            per.append(per_step)
        # every rank's rows together: all NC rows x (S + D + (Np - 1) Kr)
        NC = g.shards[0].layout.n_pad // 2048
        assert sum(per) == NC * (S + D + (Np - 1) * Kr)
        # the step-path acceleration query runs every unit once more
        if P == 1:
            s = g.shards[0]
            s.audit_reset()
            s.accel(step_path=True)
            assert s.audit() == (per[0], per[0])
    finally:
        g.close()


def _bench(args, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


def test_bench_audit_ok_and_reports_physics(hip):
    r, out = _bench(["--n", "65536", "--steps", "6", "--warmup", "2", "--exact-steps", "2"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert out["work_audit"] == "ok"
    assert out["audit"]["replay"] == "bitwise"
    u = out["audit"]["units"]
    assert u["units_done_rank0"] == 6 * u["units_per_step_rank0"] and u["ranks_short"] == 0
    c = out["config"]
    assert c["sampled_rel_err"] < 1e-4 and c["sampled_rel_err_final"] < 1e-4
    assert c["momentum_rel_drift"] < 1e-5
    assert c["exact_cutoff_ms_per_step"] > 0
    assert c["hbm"]["gb_per_rank_max"] > 0 and "sym_Pj" in c["hbm"]["by_buffer_gb_rank0"]
    k = c["conservation"]  # energy with the exact-cutoff potential, before warmup / after
    assert k["energy_start"] < 0 and k["energy_end"] < 0  # bound system (solar + random)
    assert 0 <= k["energy_rel_drift"] < 1e-2 and k["momentum_rel_drift"] < 1e-5
    assert k["angular_momentum_rel_drift"] < 1e-5


def test_bench_audit_catches_skipped_units(hip):
    """The dynamic counter starts at 64 in every force launch: 64 units per step never run.
    The step is slightly faster and wrong; bench.py must say so and exit non-zero."""
    r, out = _bench(["--n", "65536", "--steps", "4", "--warmup", "1", "--exact-steps", "0",
                     "--phase-steps", "0"], {"GRAVSIM_FAULT_SKIP_UNITS": "64"})
    assert r.returncode == 1, (r.returncode, r.stderr[-3000:])
    assert "work audit FAILED" in r.stderr
    assert out is not None and out["work_audit"] != "ok"
    assert "unit count" in out["work_audit"] and "replay" in out["work_audit"]
    u = out["audit"]["units"]
    assert u["units_done_rank0"] == 4 * (u["units_per_step_rank0"] - 64)


@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
def test_cutoff_paths_below_the_cutoff_pinned(hip, dtype):
    """A pair closer than the reference's 1e-10 m cutoff: the exact path (the reference's
    select, cuda.cu:39, mpi.c:64) gives it zero force; the fast path (the default) adds the
    core c^2 instead, so the pair gets mu r / (r^2 + c^2)^1.5: finite, huge, never NaN.
    Every other pair is the same in both paths (bit-identical above ~1 cm)."""
    from gravsim.runtime.engines import HipEngine

    n = 4096
    b = ic.solar_random(n, seed=21)
    b.pos[101] = b.pos[100] + np.array([5e-11, 0.0, 0.0])  # 0.5 cutoff apart
    out = {}
    for mode in ("exact", "fast"):
        e = HipEngine(SimConfig(n=n, dtype=dtype, device="gpu", mode="sym", cutoff_mode=mode))
        try:
            e.load(b)
            out[mode] = (e.accel(step_path=True)[:n, :3], e.force_mode())
        finally:
            e.close()
    a_ex, fm_ex = out["exact"]
    a_fa, fm_fa = out["fast"]
    assert fm_ex["exact"] and not fm_fa["exact"]
    c2 = fm_fa["eps2"]
    mu = 6.67430e-11 * b.mass
    d = b.pos[101] - b.pos[100]
    r2 = float(d @ d)
    want_100 = mu[101] * d / (r2 + c2) ** 1.5  # the pair's term on body 100 (fast path)
    got_100 = a_fa[100] - a_ex[100]
    assert np.all(np.isfinite(a_fa)) and np.all(np.isfinite(a_ex))
    np.testing.assert_allclose(got_100, want_100, rtol=1e-4 if dtype == "fp32" else 1e-9,
                               atol=1e-6 * np.abs(want_100).max())
    # far bodies see both paths alike
    far = np.setdiff1d(np.arange(n), [100, 101])
    rel = np.abs(a_fa[far] - a_ex[far]).max() / np.abs(a_ex[far]).max()
    assert rel < (1e-5 if dtype == "fp32" else 1e-12), rel


@pytest.mark.parametrize("n,band_mb,steps", [(65536, "1", 20), (1 << 20, "1540", 2)])
def test_dynamic_counter_rearm_many_launches(hip, monkeypatch, n, band_mb, steps):
    """Many dynamic launches back to back on one stream, band after band, replayed from a
    hipGraph (65,536 bodies: one row per band, 32 launches per step, a 16-workgroup first wave
    so every band launch fetches dynamically; 1M: 4 bands): the stream-ordered memset re-arms
    the unit counter before each launch, so every unit runs exactly once per step (device
    count) and the bits equal one static unit per workgroup. (Round 2's in-kernel
    last-workgroup re-arm failed exactly this pattern and was retired, docs/DESIGN.md §8.)"""
    from gravsim.runtime.engines import HipEngine

    monkeypatch.setenv("GRAVSIM_SYM_BAND_MB", band_mb)
    out = {}
    for cap in (2, 0):
        e = HipEngine(SimConfig(n=n, dtype="fp32", device="gpu", mode="sym"))
        try:
            e.set_schedule(1, cap)
            e.set_tuning(first_wave=16)
            e.init_ics("solar+random", 13)
            e.audit_reset()
            e.step(steps)
            e.sync()
            done, per = e.audit()
            assert done == per * steps, (cap, done, per)
            assert e.graph_info()["mode"] == "graph"
            b = e.state()
            out[cap] = (b.pos, b.vel)
        finally:
            e.close()
    assert np.array_equal(out[2][0], out[0][0])
    assert np.array_equal(out[2][1], out[0][1])


def test_device_memory_ledger(hip):
    """The stepper's HBM ledger (gs_stepper_mem_entry) lists every buffer with the size the
    layout implies: ping-pong rows, the one band of partial slots, the node sums."""
    from gravsim.parallel import partition
    from gravsim.runtime.engines import HipEngine

    n = 65536
    e = HipEngine(SimConfig(n=n, dtype="fp32", device="gpu", mode="sym"))
    try:
        m = e.mem_info()
        n_pad = e.layout.n_pad
        g = partition.sym_geometry(n_pad)
        assert m["X0"] == m["X1"] == n_pad * 16
        assert m["vel"] == n_pad * 16
        slots = n_pad * 3 * 4
        assert m["sym_Pi"] == slots * g["S"] and m["sym_Pj"] == slots * g["H"]
        assert m["sym_Pd"] == slots * g["D"]
        kr, np_ = partition.sym_split(n_pad)  # split segments: parts 1 .. Np-1 in Px
        assert m.get("sym_Px", 0) == slots * kr * (np_ - 1)
        assert m["sym_S"] == len(partition.sym_nodes(n_pad, 1)[0]) * 3 * n_pad * 4
        assert "sym_R" not in m and "partial" not in m  # one rank: R is S; no split slots
        assert all(v > 0 for v in m.values())
    finally:
        e.close()


def test_bench_two_ranks_gated_audit_failure_is_reported(hip):
    """Two RCCL ranks on one GPU (sockets, GRAVSIM_RCCL_RANK_HOSTS=1) through the production
    launch sequence. A failed audit of the gated launch's timed steps (injected by bench.py's
    test hook) is a failure of the multi-rank default: the ungated schedule is timed from the
    same ICs (config.overlap_fallback, so the line still carries a labelled number), but
    work_audit reports the gated failure and bench.py exits 1."""
    r, out = _bench(["--gpus", "2", "--n", "65536", "--steps", "3", "--warmup", "1",
                     "--exact-steps", "0", "--phase-steps", "0", "--check-samples", "0",
                     "--no-energy"],
                    {"GRAVSIM_RCCL_RANK_HOSTS": "1", "GRAVSIM_TEST_FAIL_GATED_AUDIT": "1"})
    assert out.get("status") != "error", (out.get("error"), out.get("stage"))
    c = out["config"]
    if c["overlap_check"] and "overlap 0" in c["overlap_check"] and c["overlap_fallback"] is None:
        assert r.returncode == 0, r.stderr[-3000:]
        pytest.skip("the race picked the ungated schedule: no gated run to fall back from")
    assert r.returncode == 1, r.stderr[-3000:]
    fb = c["overlap_fallback"]
    assert fb and fb["from_overlap"] == 3 and fb["to_overlap"] == 0
    assert "injected" in fb["failures"][0]
    assert c["overlap"] == 0 and out["status"] == "audit failed"
    assert out["work_audit"].startswith("gated schedule (the multi-rank default) failed")
    assert out["audit"]["replay"] == "bitwise" and out["n_gpus"] == 2
