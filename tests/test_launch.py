"""Self-launch of P ranks (parallel/launch.py) for bench.py and the CLI: the `mpirun -np P`
step of the reference (mpi.c:140-144). CPU only: argv rewriting, the world-size guards, and a
real torch.distributed.run child that brings up 2 ranks (which then stop at the GPU check)."""
import os
import subprocess
import sys

import pytest

from gravsim.parallel import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_strip_rank_flags_all_spellings():
    argv = ["--gpus", "8", "--n", "1048576", "--nproc=2", "--gpus=4", "--n=7", "--steps", "3",
            "--dtype", "fp64"]
    assert launch.strip_rank_flags(argv) == ["--num-bodies", "1048576", "--num-bodies=7",
                                             "--steps", "3", "--dtype", "fp64"]


def test_torchrun_cmd_shape():
    cmd = launch.torchrun_cmd(8, ["bench.py"], ["--gpus", "8", "--steps", "5"], 29500,
                              keep_gpus=True)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29500"
    tail = cmd[cmd.index("bench.py"):]
    assert tail == ["bench.py", "--gpus", "8", "--steps", "5"]  # --gpus exactly once
    m = launch.torchrun_cmd(2, ["-m", "gravsim"], ["--gpus", "2", "--n", "64"], 1)
    assert m[-4:] == ["-m", "gravsim", "--num-bodies", "64"]
    with pytest.raises(ValueError):
        launch.torchrun_cmd(0, ["x.py"], [], 1)


def test_device_count_guard(monkeypatch):
    monkeypatch.delenv("GRAVSIM_RCCL_RANK_HOSTS", raising=False)
    import torch

    have = torch.cuda.device_count()
    monkeypatch.delenv(launch.PROBE_ENV, raising=False)
    with pytest.raises(SystemExit, match="HIP device"):
        launch.check_device_count(have + 1)
    monkeypatch.setenv("GRAVSIM_RCCL_RANK_HOSTS", "1")
    monkeypatch.delenv(launch.PROBE_ENV, raising=False)
    # rehearsal: every rank on one GPU; the probe still runs and is handed to the ranks
    assert launch.check_device_count(have + 8) == have
    assert os.environ[launch.PROBE_ENV] == str(have)


def _bench(args, env_extra):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=240, cwd=ROOT)


def test_bench_world_size_mismatch_refused():
    r = _bench(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0
    assert "--gpus 4 but WORLD_SIZE 2" in r.stderr


def test_bench_gpus_without_devices_refused():
    r = _bench(["--gpus", "2", "--steps", "1"], {"GRAVSIM_RCCL_RANK_HOSTS": "0"})
    assert r.returncode != 0
    assert "HIP device(s) are visible" in r.stderr


@pytest.mark.slow
def test_bench_self_launches_two_ranks():
    """No launcher + --gpus 2: bench.py starts 2 ranks under torch.distributed.run. Both come
    up with WORLD_SIZE=2 (the gloo control group forms) and stop at the GPU check here."""
    import json

    r = _bench(["--gpus", "2", "--n", "4096", "--steps", "1"], {"GRAVSIM_RCCL_RANK_HOSTS": "1"})
    assert r.returncode != 0
    # rank 0's guard reports the job in one error line (parallel/guard.py), with both ranks'
    # records: both reached the device stage and failed there
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, (r.stdout[-2000:], r.stderr[-2000:])
    e = lines[0]
    assert e["status"] == "error" and e["stage"] == "device" and e["n_gpus"] == 2, e
    assert [x["stage"] for x in e["config"]["ranks"]] == ["device", "device"]
    assert "bench.py needs a HIP device" in e["error"]
    assert "--gpus 2 but" not in r.stderr  # the children saw WORLD_SIZE == --gpus


def test_bench_clock_summary_normalises_boxes():
    """bench.py's clock-normalised cost: two boxes 6 % apart in ms/step (round 6, 1M on one
    GPU: 170.26 ms at 2.0934 GHz, 160.26 ms at 2.2256 GHz) give the same CU-cycles per pair;
    a schedule without a clock record reports None rather than 0."""
    import bench

    pairs = 1048576 * 1048575 / 2 * 10
    a = bench.clock_summary(2.0934, 2.0934, 2.0934, 0.0, 1.7026, 256, pairs, 1)
    b = bench.clock_summary(2.2256, 2.2256, 2.2256, 0.0, 1.6026, 256, pairs, 1)
    assert abs(a["cycles_per_pair_eval"] - 0.1660) < 5e-4
    assert abs(a["cycles_per_pair_eval"] / b["cycles_per_pair_eval"] - 1) < 2e-3
    assert a["engine_clock_ghz_ranks"] is None and a["force_wg_cycles_per_pair_eval"] is None
    m = bench.clock_summary(2 * 2.1, 2.0, 2.2, 3.3e11, 1.0, 512, pairs, 2)
    assert m["engine_clock_ghz"] == 2.1 and m["engine_clock_ghz_ranks"] == [2.0, 2.2]
    assert m["force_wg_cycles_per_pair_eval"] == 3.3e11 / pairs
    none = bench.clock_summary(0.0, 0.0, 0.0, 0.0, 1.0, 256, pairs, 1)
    assert none["engine_clock_ghz"] is None and none["cycles_per_pair_eval"] is None
