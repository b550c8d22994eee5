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
