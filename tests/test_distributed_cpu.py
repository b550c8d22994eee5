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
