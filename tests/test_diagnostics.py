"""Conserved-quantity diagnostics of the Simulation driver (--diagnostics / --diag-every).

The reference has no conservation check (it only prints positions, mpi.c:249-257); these tests
pin the new one: the engine-side sums equal the fp64 NumPy diagnostics of the same state, the
integrators conserve what they should (leapfrog energy to rounding level on a Kepler orbit,
KD to first order; momentum and angular momentum to rounding for both, Newton-3 pairs), the
values do not depend on the rank count, and the CLI reports the drifts in its metrics JSON.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _sim(**kw):
    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.runtime.simulation import Simulation

    base = dict(n=300, steps=0, dtype="fp64", device="cpu", chunk=1024)
    base.update(kw)
    return Simulation(SimConfig(**base))


@pytest.mark.parametrize("integrator", ["kd", "leapfrog"])
def test_conserved_matches_numpy_diagnostics(integrator):
    from gravsim.models import diagnostics as dg

    sim = _sim(integrator=integrator, dt=600.0)
    try:
        sim.run(5)
        c = sim.conserved()
        b = sim.global_state()  # synchronized velocities (leapfrog: v_k, not v_{k-1/2})
        e = dg.energy(b.pos, b.vel, b.mass, sim.cfg.G, sim.cfg.cutoff, sim.cfg.softening)
        assert c["energy"] == pytest.approx(e, rel=1e-12)
        np.testing.assert_allclose(c["momentum"], dg.momentum(b.vel, b.mass),
                                   rtol=1e-10, atol=1e-10 * c["momentum_scale"])
        lm = (b.mass[:, None] * np.cross(b.pos, b.vel)).sum(0)
        np.testing.assert_allclose(c["angular_momentum"], lm, rtol=1e-10,
                                   atol=1e-12 * c["angular_momentum_scale"])
        assert c["step"] == 5
    finally:
        sim.close()


def test_kepler_energy_drift_leapfrog_vs_kd():
    drift = {}
    for integ in ("kd", "leapfrog"):
        sim = _sim(n=2, init="kepler", dt=3600.0, integrator=integ, diagnostics=True)
        try:
            m = sim.run(2000)  # 83 days of a 1-year orbit
        finally:
            sim.close()
        c = m.extra["conservation"]
        drift[integ] = c["energy_rel_drift"]
        assert c["angular_momentum_rel_drift"] < 1e-12
        assert c["momentum_rel_drift"] < 1e-12
    assert drift["leapfrog"] < 1e-11          # second order, symplectic: rounding level here
    assert 1e-9 < drift["kd"] < 1e-5           # first order: a visible, bounded drift
    assert drift["leapfrog"] < 1e-3 * drift["kd"]


def test_diag_samples_and_wall_excludes_them():
    sim = _sim(n=500, diagnostics=True, diag_every=3)
    try:
        m = sim.run(9)
    finally:
        sim.close()
    c = m.extra["conservation"]
    assert [s["step"] for s in c["samples"]] == [3, 6]  # the end state is energy_end
    assert c["momentum_rel_drift"] < 1e-12
    assert np.isfinite(c["energy_rel_drift"]) and m.wall_s > 0


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.parallel import comm
    from gravsim.runtime.simulation import Simulation

    dist = comm.init(timeout_s=120)
    try:
        cfg = SimConfig(n=1500, steps=4, dtype="fp64", device="cpu", chunk=1024,
                        integrator="leapfrog", diagnostics=True)
        sim = Simulation(cfg, dist)
        m = sim.run()
        if rank == 0:
            with open(os.path.join(out_dir, f"w{world}.json"), "w") as f:
                json.dump(m.extra["conservation"], f)
        sim.close()
    finally:
        comm.shutdown(dist)


def test_conservation_independent_of_rank_count(tmp_path):
    import torch.multiprocessing as mp

    for world in (1, 2):
        mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                           start_method="spawn", join=True)
    one = json.load(open(tmp_path / "w1.json"))
    two = json.load(open(tmp_path / "w2.json"))
    for k in ("energy_start", "energy_end"):
        assert two[k] == pytest.approx(one[k], rel=1e-12)  # only the all-reduce order differs
    assert two["energy_rel_drift"] == pytest.approx(one["energy_rel_drift"], rel=1e-6, abs=1e-15)


def test_cli_diag_every_reports_conservation(tmp_path):
    out = tmp_path / "m.json"
    env = dict(os.environ, PYTHONPATH=ROOT)
    subprocess.run([sys.executable, "-m", "gravsim", "--n", "200", "--steps", "20", "--device",
                    "cpu", "--dtype", "fp64", "--diag-every", "5", "--log-format", "none",
                    "--quiet", "--metrics-json", str(out)], cwd=ROOT, env=env, check=True,
                   timeout=300)
    d = json.loads(out.read_text().splitlines()[-1])
    c = d["extra"]["conservation"]
    assert [s["step"] for s in c["samples"]] == [5, 10, 15]
    assert c["momentum_rel_drift"] < 1e-12 and c["angular_momentum_rel_drift"] < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,rel", [("fp64", 1e-10), ("fp32", 2e-5)])
def test_gpu_conserved_matches_cpu_engine(dtype, rel):
    """The GPU engine's diagnostic pass (exact-cutoff potential, one-sided kernels) gives the
    CPU engine's energy and momenta on the same state."""
    import torch

    assert torch.cuda.is_available()
    vals = {}
    for dev in ("cpu", "gpu"):
        sim = _sim(n=20000, dtype=dtype, device=dev, chunk=0, integrator="leapfrog")
        try:
            vals[dev] = sim.conserved()
        finally:
            sim.close()
    g, c = vals["gpu"], vals["cpu"]
    assert g["energy"] == pytest.approx(c["energy"], rel=rel)
    assert g["kinetic"] == pytest.approx(c["kinetic"], rel=rel)
    assert np.linalg.norm(np.subtract(g["momentum"], c["momentum"])) <= rel * c["momentum_scale"]
