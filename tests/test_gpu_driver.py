"""End-to-end GPU driver paths: CLI, checkpoint/resume bit-exactness, trajectories, NaN guard,
device ICs surviving engine creation, sweep-format logs — all on the HIP Stepper."""
import glob
import json
import os

import numpy as np
import pytest

from gravsim.cli import main
from gravsim.config import SimConfig
from gravsim.models import initial_conditions as ic
from gravsim.runtime.simulation import NonFiniteError, Simulation
from gravsim.utils import checkpoint as ck

pytestmark = pytest.mark.gpu


def test_cli_gpu_fp32_mpi_log(hip, tmp_path, capsys):
    assert main(["--n", "4096", "--steps", "20", "--dtype", "fp32", "--device", "gpu",
                 "--log-dir", str(tmp_path), "--progress-every", "10"]) == 0
    out = capsys.readouterr().out
    m = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert m["device"] == "gpu" and m["n"] == 4096 and m["steps"] == 20
    text = open(glob.glob(str(tmp_path / "gravity_logs_mpi" / "*.txt"))[0]).read()
    assert text.count("Particle ") == 4096 and "Simulation completed successfully" in text


@pytest.mark.parametrize("dtype,mode,integrator", [("fp32", "auto", "kd"), ("fp64", "auto", "kd"),
                                                   ("fp32", "sym", "kd"), ("fp64", "sym", "kd"),
                                                   ("fp32", "sym", "leapfrog")])
def test_gpu_resume_bit_exact(hip, tmp_path, dtype, mode, integrator):
    cfg = SimConfig(n=3000, steps=9, dtype=dtype, device="gpu", checkpoint_dir=str(tmp_path),
                    checkpoint_every=5, mode=mode, integrator=integrator)
    sim = Simulation(cfg)
    sim.run()
    full = sim.global_state()
    sim.close()
    sim2 = Simulation(cfg.replace(resume=ck.path_for(str(tmp_path), 5), checkpoint_every=0))
    sim2.run(4)
    got = sim2.global_state()
    sim2.close()
    assert np.array_equal(got.pos, full.pos) and np.array_equal(got.vel, full.vel)


@pytest.mark.parametrize("mode", ["auto", "sym"])
def test_gpu_matches_cpu_engine_steps_fp64(hip, mode):
    """The GPU Stepper (one-sided or Newton-3 schedule) and the native CPU engine integrate
    the same fp64 trajectory."""
    out = {}
    for dev in ("cpu", "gpu"):
        sim = Simulation(SimConfig(n=1500, steps=10, dtype="fp64", device=dev,
                                   mode=mode if dev == "gpu" else "auto"))
        sim.run()
        out[dev] = sim.global_state()
        sim.close()
    rel = np.abs(out["gpu"].pos - out["cpu"].pos).max() / np.abs(out["cpu"].pos).max()
    assert rel < 1e-12


def test_gpu_trajectory_and_nan_guard(hip):
    sim = Simulation(SimConfig(n=512, steps=6, device="gpu", dtype="fp32", record_every=3))
    sim.run()
    assert len(sim.trajectory) == 2 and sim.trajectory[0].shape == (512, 3)
    b = sim.engine.state()
    b.pos[7, 2] = np.nan
    sim.engine.load(b)
    sim.cfg = sim.cfg.replace(nan_check_every=1)
    with pytest.raises(NonFiniteError):
        sim.run(2)
    sim.close()


def test_device_ics_survive_engine_creation(hip):
    """Regression: buffer zeroing must be ordered before the IC kernel (non-blocking stream)."""
    from gravsim.runtime.engines import HipEngine

    ref = ic.solar_random(20000, 3)
    for _ in range(4):
        e = HipEngine(SimConfig(n=20000, dtype="fp32", device="gpu"))
        e.init_ics("solar+random", 3)
        b = e.state()
        e.close()
        assert np.array_equal(b.vel, ref.vel.astype(np.float32).astype(np.float64))


def test_plummer_model_on_gpu_energy(hip):
    from gravsim.models.diagnostics import energy

    sim = Simulation(SimConfig(n=2048, steps=50, device="gpu", dtype="fp64", init="plummer",
                               dt=3600.0))
    b0 = sim.global_state()
    e0 = energy(b0.pos, b0.vel, b0.mass)
    sim.run()
    b1 = sim.global_state()
    sim.close()
    assert abs(energy(b1.pos, b1.vel, b1.mass) - e0) / abs(e0) < 1e-3


@pytest.mark.parametrize("mode", ["auto", "sym"])
def test_gpu_leapfrog_matches_oracle_kdk(hip, mode):
    from gravsim.ops import oracle

    cfg = SimConfig(n=800, steps=10, dtype="fp64", device="gpu", integrator="leapfrog",
                    mode=mode)
    sim = Simulation(cfg)
    b0 = ic.solar_random(800, cfg.seed)
    sim.run()
    got = sim.global_state()
    sim.close()
    x, v, _ = oracle.simulate(b0.pos, b0.vel, b0.mass, cfg.dt, 10, integrator="leapfrog")
    assert np.abs(got.pos - x).max() / np.abs(x).max() < 1e-12
    assert np.abs(got.vel - v).max() / np.abs(v).max() < 1e-10


def test_native_driver_matches_python_cli_dump(hip, tmp_path, capsys):
    """gravsim_bench (the C++ driver, no Python) runs the same Stepper: its final-position
    dump equals the Python CLI's for the same N / steps / seed, its metrics line reports the
    engine clock of the sym force launches, and no body goes non-finite."""
    import subprocess

    from gravsim.ops import _native

    exe = _native.NATIVE_DIR / "gravsim_bench"
    assert exe.exists(), "gravsim_bench not built (csrc/build.py)"
    seed = 20250307  # (gravsim_bench's default seed)
    r = subprocess.run([str(exe), "--n", "20000", "--steps", "4", "--dump",
                        str(tmp_path / "native.txt"), "--progress-every", "0"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    m = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert m["nonfinite"] == 0 and m["n"] == 20000 and m["steps"] == 4
    assert 0.5 < m["engine_clock_ghz"] < 3.5, m
    assert main(["--n", "20000", "--steps", "4", "--device", "gpu", "--dtype", "fp32",
                 "--seed", str(seed), "--dump", str(tmp_path / "py.txt"), "--log-format", "none",
                 "--metrics-json", str(tmp_path / "m.json"), "--quiet"]) == 0
    # (gravsim_bench's defaults: fp32, dt 3600 s, cutoff 1e-10 m)
    capsys.readouterr()
    assert (tmp_path / "native.txt").read_text() == (tmp_path / "py.txt").read_text()
    pm = json.loads((tmp_path / "m.json").read_text().splitlines()[-1])
    assert pm["mode"] == "sym" and 0.5 < pm["extra"]["engine_clock_ghz"] < 3.5, pm


def test_bench_json_contract(hip, tmp_path):
    """bench.py's one JSON line (the driver's contract) on a short run: metric / config of
    BASELINE.json, the audits, the kernel label from the compiled tile and the clock-normalised
    cost (engine clock within MI355X's range, CU-cycles per pair in the 0.1-0.4 band of the
    sym tile)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "bench.py", "--n", "65536", "--steps", "20", "--warmup",
                        "4", "--exact-steps", "2", "--phase-steps", "2"], cwd=root,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 20 and d["warmup"] == 4 and d["dtype"] == "fp32"
    assert d["status"] == "ok" and d["work_audit"] == "ok", d.get("work_audit")
    assert d["audit"]["replay"] == "bitwise"
    assert "8 i x 2 j per lane" in d["config"]["kernel"]
    # one-rank graph replays: 32 steps per launch at this size (and 2 for the remainder)
    assert d["config"]["graph"] == "graph" and d["config"]["graph_steps_per_launch"] == 32
    assert 0.5 < d["engine_clock_ghz"] < 3.5 and 0.1 < d["cycles_per_pair_eval"] < 0.4, d
    assert abs(d["value"] - 65536 * 1e3 / d["ms_per_step"]) < 1e-6 * d["value"]
