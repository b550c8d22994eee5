"""Multi-process body decomposition on CPU: gloo process group, world_size 2 and 3.

The mpi.c analogue (MPI_Allgatherv per step, mpi.c:227-231) with Jacobi semantics: a P-rank
run must equal the 1-rank run bit for bit (the reference's does not: D6).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, steps, dtype, out_dir, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.parallel import comm
    from gravsim.runtime.simulation import Simulation

    dist = comm.init(timeout_s=120)
    try:
        cfg = SimConfig(n=n, steps=steps, dtype=dtype, device="cpu", chunk=1024)
        if mode == "ckpt":
            cfg = cfg.replace(checkpoint_dir=out_dir, checkpoint_every=steps)
        sim = Simulation(cfg, dist)
        sim.run()
        b = sim.global_state()
        if rank == 0:
            np.savez(os.path.join(out_dir, f"w{world}.npz"), pos=b.pos, vel=b.vel)
        sim.close()
    finally:
        comm.shutdown(dist)


def _run(world, n, steps, dtype, out_dir, mode="plain"):
    mp.start_processes(_worker, args=(world, _free_port(), n, steps, dtype, out_dir, mode),
                       nprocs=world, start_method="spawn", join=True)
    return np.load(os.path.join(out_dir, f"w{world}.npz"))


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_gloo_world2_bitwise_equals_single(tmp_path, dtype):
    n, steps = 1500, 8
    from gravsim.config import SimConfig
    from gravsim.runtime.engines import CpuEngine

    eng = CpuEngine(SimConfig(n=n, dtype=dtype, device="cpu", chunk=1024))
    eng.init_ics("solar+random", SimConfig().seed)
    eng.step(steps)
    ref = eng.state()
    got = _run(2, n, steps, dtype, str(tmp_path))
    assert np.array_equal(got["pos"], ref.pos)
    assert np.array_equal(got["vel"], ref.vel)


def test_gloo_world3_uneven_and_checkpoint(tmp_path):
    """N not divisible by P (ghost padding) + a rank-agnostic checkpoint written by rank 0."""
    n, steps = 2051, 4
    got = _run(3, n, steps, "fp64", str(tmp_path), mode="ckpt")
    from gravsim.utils import checkpoint as ck

    c = ck.load(ck.latest(str(tmp_path)))
    assert c.step == steps
    assert np.array_equal(c.bodies.pos, got["pos"]) and np.array_equal(c.bodies.vel, got["vel"])


def test_torchrun_cli_world2_matches_single(tmp_path):
    """`torch.distributed.run -m gravsim` (the `mpirun -np P ./mpi` equivalent) writes the same
    mpi.c-format dump as a single-process run."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=root)
    args = ["-m", "gravsim", "--num-bodies", "700", "--steps", "5", "--device", "cpu", "--quiet"]
    one = tmp_path / "one.txt"
    two = tmp_path / "two.txt"
    subprocess.run([sys.executable, *args, "--dump", str(one)], cwd=root, env=env, check=True,
                   timeout=300)
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
                    "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                    str(_free_port()), *args, "--dump", str(two)], cwd=root, env=env,
                   check=True, timeout=300)
    assert one.read_text() == two.read_text() and one.read_text().count("Particle ") == 700
    # `--nproc 3` launches the ranks itself (the `mpirun -np 3` form)
    three = tmp_path / "three.txt"
    subprocess.run([sys.executable, *args, "--nproc", "3", "--dump", str(three)], cwd=root,
                   env=env, check=True, timeout=300)
    assert three.read_text() == one.read_text()
