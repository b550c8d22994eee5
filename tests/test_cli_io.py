"""CLI, reference log formats, dumps, checkpoints, trajectories (CPU engine).

Golden formats from SURVEY.md §2.6: mpi.c:110-138,242-262 (canonical), pyspark.py:153-200
(sweep log), cuda.cu:99-117,140-175 (stdout positions with 14 decimals).
"""
import glob
import io
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from gravsim.cli import main
from gravsim.config import SimConfig
from gravsim.runtime.simulation import NonFiniteError, Simulation
from gravsim.utils import checkpoint as ck
from gravsim.utils.logs import RunLog

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cli_config1_mpi_log_golden(tmp_path, capsys):
    """BASELINE config #1: 1,024 bodies, 100 steps, CPU, mpi.c log layout."""
    rc = main(["--n", "1024", "--steps", "100", "--device", "cpu", "--log-dir", str(tmp_path)])
    assert rc == 0
    out = capsys.readouterr().out
    assert "Step 0/100" in out
    metrics = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert metrics["n"] == 1024 and metrics["steps"] == 100 and metrics["body_updates_per_s"] > 0
    files = glob.glob(str(tmp_path / "gravity_logs_mpi" / "mpi_c_simulation_*.txt"))
    assert len(files) == 1
    assert re.search(r"mpi_c_simulation_\d{8}_\d{6}\.txt$", files[0])
    text = open(files[0]).read()
    pat = (r"^Starting MPI C gravity simulation at \d{8}_\d{6}\n"
           r"Number of processes: 1\nNumber of particles: 1024\nSteps: 100\n"
           r"Timestep: 3600\.000000 seconds\n\n\nPerformance Statistics:\n"
           r"Total execution time: \d+\.\d{2} seconds\nAverage time per step: \d+\.\d{4} seconds\n"
           r"\nFinal positions:\n(Particle \d+: \(-?\d\.\d{6}e[+-]\d\d, -?\d\.\d{6}e[+-]\d\d, "
           r"-?\d\.\d{6}e[+-]\d\d\)\n){1024}\nSimulation completed successfully\n$")
    assert re.match(pat, text), text[:400]
    assert oct(os.stat(os.path.dirname(files[0])).st_mode & 0o777) == "0o700"


def test_cli_spark_sweep_format(tmp_path, capsys):
    main(["--sweep", "10,100", "--steps", "5", "--device", "cpu", "--log-dir", str(tmp_path),
          "--quiet"])
    out = capsys.readouterr().out
    files = glob.glob(str(tmp_path / "gravity_logs_spark" / "simulation_log_*.txt"))
    assert len(files) == 1
    text = open(files[0]).read()
    for n in (10, 100):
        assert f"Starting gravity simulation with 1 cores and {n} particles" in text
    assert text.count("Performance Statistics:") == 2
    assert re.search(r"Particle 99: \(-?[\d.e+-]+, -?[\d.e+-]+, -?[\d.e+-]+\)", text)
    assert text.rstrip().endswith("Simulation completed successfully")
    assert text.count("Simulation completed successfully") == 1
    assert "Simulation took" in out


def test_cuda_format_stdout_positions(tmp_path):
    buf = io.StringIO()
    log = RunLog("cuda", str(tmp_path), stdout=buf)
    log.header(1, 12, 500, 3600.0)
    pos = np.arange(36, dtype=float).reshape(12, 3) * 1.5
    log.positions(pos)
    s = buf.getvalue()
    assert "Final positions of first 10 out of 12 particles:" in s
    assert "Particle 9: (40.50000000000000, 42.00000000000000, 43.50000000000000)" in s
    assert "Particle 10" not in s
    assert open(log.path).read().startswith("Starting gravity simulation")


def test_dump_text_and_binary(tmp_path):
    txt, bin_ = tmp_path / "final.txt", tmp_path / "final.gsck"
    main(["--n", "50", "--steps", "3", "--device", "cpu", "--dump", str(txt), "--quiet",
          "--log-format", "none"])
    main(["--n", "50", "--steps", "3", "--device", "cpu", "--dump", str(bin_), "--quiet",
          "--log-format", "none"])
    lines = open(txt).read().splitlines()
    assert len(lines) == 50 and lines[0].startswith("Particle 0: (")
    c = ck.load(str(bin_))
    assert c.step == 3 and c.bodies.n == 50
    x0 = float(lines[7].split("(")[1].split(",")[0])
    assert x0 == pytest.approx(c.bodies.pos[7, 0], rel=1e-6)


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_resume_is_bit_exact(tmp_path, dtype):
    cfg = SimConfig(n=700, steps=10, dtype=dtype, device="cpu", checkpoint_dir=str(tmp_path),
                    checkpoint_every=4)
    sim = Simulation(cfg)
    sim.run()
    full = sim.global_state()
    sim.close()
    path = ck.path_for(str(tmp_path), 8)
    assert os.path.exists(path)
    sim2 = Simulation(cfg.replace(resume=path, checkpoint_every=0))
    assert sim2.step == 8
    sim2.run(2)
    got = sim2.global_state()
    assert np.array_equal(got.pos, full.pos) and np.array_equal(got.vel, full.vel)


def test_trajectory_recorder(tmp_path):
    cfg = SimConfig(n=40, steps=10, device="cpu", record_every=2)
    sim = Simulation(cfg)
    sim.run()
    assert len(sim.trajectory) == 5
    p = tmp_path / "traj.npy"
    sim.save_trajectory(str(p))
    assert np.load(p).shape == (5, 40, 3)


def test_nan_guard_raises():
    cfg = SimConfig(n=30, steps=4, device="cpu", nan_check_every=2)
    sim = Simulation(cfg)
    b = sim.engine.state()
    b.pos[3, 1] = np.inf
    sim.engine.load(b)
    with pytest.raises(NonFiniteError):
        sim.run()


def test_checkpoint_rejects_garbage(tmp_path):
    p = tmp_path / "bad.gsck"
    p.write_bytes(b"NOTACKPT" + b"\0" * 20)
    with pytest.raises(ValueError):
        ck.load(str(p))


def test_module_entrypoint_subprocess(tmp_path):
    r = subprocess.run([sys.executable, "-m", "gravsim", "--n", "20", "--steps", "2", "--device",
                        "cpu", "--quiet", "--log-format", "none", "--metrics-json",
                        str(tmp_path / "m.jsonl")], cwd=ROOT, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    m = json.loads(open(tmp_path / "m.jsonl").read().splitlines()[0])
    assert m["n"] == 20 and m["device"] == "cpu"


def test_config_validation():
    with pytest.raises(ValueError):
        SimConfig(n=0).validate()
    with pytest.raises(ValueError):
        SimConfig(dtype="bf16").validate()
    with pytest.raises(ValueError):
        SimConfig(chunk=1000).validate()
    # the Newton-3 schedule: both precisions and both cutoff paths; not with the MFMA kernel
    for kw in (dict(dtype="fp32"), dict(dtype="fp64"), dict(cutoff_mode="exact")):
        SimConfig(mode="sym", **kw).validate()
    with pytest.raises(ValueError):
        SimConfig(mode="sym", kernel="mfma").validate()


def test_cli_accepts_sym_mode(capsys):
    """--mode sym parses (the CPU engine ignores the GPU schedule)."""
    assert main(["--n", "64", "--steps", "2", "--device", "cpu", "--mode", "sym",
                 "--log-format", "none"]) == 0


@pytest.mark.parametrize("fam", ["plummer", "cold", "random"])
def test_cli_model_families(fam, capsys):
    assert main(["--n", "64", "--steps", "3", "--device", "cpu", "--init", fam, "--log-format",
                 "none"]) == 0


def test_dump_every_writes_periodic_mpi_dumps(tmp_path, capsys):
    from gravsim.utils.logs import format_positions_mpi

    final = tmp_path / "pos.txt"
    assert main(["--n", "50", "--steps", "6", "--device", "cpu", "--dump", str(final),
                 "--dump-every", "3", "--quiet"]) == 0
    d3, d6 = tmp_path / "pos_step00000003.txt", tmp_path / "pos_step00000006.txt"
    assert d3.exists() and d6.exists()
    assert d6.read_text() == final.read_text() and d3.read_text() != d6.read_text()
    assert d3.read_text().count("Particle ") == 50


def _poisoned_checkpoint(tmp_path, n=64):
    from gravsim.models import initial_conditions as ic

    b = ic.solar_random(n, seed=3)
    b.pos[5, 2] = np.nan
    p = tmp_path / "poison.gsck"
    ck.save(str(p), b, 0, dict(dt=3600.0, dtype="fp64", velocity="synchronized"))
    return p


@pytest.mark.parametrize("device", ["cpu", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_cli_nan_guard_exits_nonzero(tmp_path, device):
    """--nan-check-every 1 on a poisoned state: the run stops at the first check with the
    guard's message and a non-zero exit (the reference printed inf/NaN silently, D1-D3)."""
    p = _poisoned_checkpoint(tmp_path)
    r = subprocess.run([sys.executable, "-m", "gravsim", "--n", "64", "--steps", "5", "--device",
                        device, "--resume", str(p), "--nan-check-every", "1", "--log-format",
                        "none", "--quiet"], cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 3, (r.returncode, r.stderr[-800:])
    assert "non-finite position/velocity components at step 1" in r.stderr


def test_resume_leapfrog_with_new_dt_resynchronises(tmp_path):
    """A leapfrog checkpoint holds v_{k-1/2} for ITS dt. Resuming with another dt first
    synchronises with the stored dt, then re-staggers with the new one: the same as resuming
    the synchronized state of that checkpoint under the new dt."""
    cfg = SimConfig(n=200, steps=4, dtype="fp64", device="cpu", integrator="leapfrog",
                    checkpoint_dir=str(tmp_path), checkpoint_every=4)
    sim = Simulation(cfg)
    sim.run()
    sync = sim.global_state()  # synchronized velocities at step 4
    sim.close()
    path = ck.path_for(str(tmp_path), 4)
    assert ck.load(path).meta["velocity"] == "half-step"
    a = Simulation(cfg.replace(resume=path, checkpoint_every=0, dt=1800.0))
    a.run(3)
    got = a.global_state()
    a.close()
    sp = tmp_path / "sync.gsck"
    ck.save(str(sp), sync, 4, dict(dt=3600.0, velocity="synchronized"))
    b = Simulation(cfg.replace(resume=str(sp), checkpoint_every=0, dt=1800.0))
    b.run(3)
    ref = b.global_state()
    b.close()
    assert np.allclose(got.pos, ref.pos, rtol=1e-13, atol=0)
    assert np.allclose(got.vel, ref.vel, rtol=1e-10, atol=1e-12)


def test_metrics_pair_counts():
    from gravsim.utils.metrics import RunMetrics

    m = RunMetrics(n=1000, steps=10, dt=1.0, dtype="fp32", device="gpu", nranks=1, wall_s=2.0,
                   mode="sym")
    assert m.effective_interactions_per_s == pytest.approx(1000 * 1000 * 10 / 2.0)
    assert m.pair_evals_per_s == pytest.approx(1000 * 999 / 2 * 10 / 2.0)
    d = json.loads(m.to_json())
    assert "interactions_per_s" not in d and d["pair_evals_per_s"] == m.pair_evals_per_s
    m.mode = "split"
    assert m.pair_evals_per_s == m.effective_interactions_per_s


def test_cli_multi_rank_flags_parse():
    from gravsim.cli import build_parser, config_from_args

    a = build_parser().parse_args(["--n", "64", "--step-timeout", "30", "--graph-comm",
                                   "--phase-timing", "--gpus", "2"])
    cfg = config_from_args(a)
    assert cfg.step_timeout_s == 30 and cfg.graph_comm and cfg.phase_timing and a.nproc == 2
    assert not config_from_args(build_parser().parse_args(["--n", "64"])).graph_comm
    with pytest.raises(ValueError):
        SimConfig(step_timeout_s=-1).validate()
