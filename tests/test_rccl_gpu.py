"""Real RCCL path (in-place all-gather + overlapped local chunks, ring pass, the sym
schedule's node-sum send/recv) with 2 to 8 processes (P = 3, 5, 6: uneven slices).

Two families:
* one device for every rank (always run): the GPU box usually exposes one MI355X, and RCCL
  refuses two ranks of one host on one device ("Duplicate GPU detected"), so each rank gets its
  own NCCL_HOSTID: RCCL then treats the ranks as separate hosts and moves data through its
  socket transport over loopback instead of xGMI. The collectives, peer calls, stream/event
  ordering and buffer offsets of the multi-rank schedule are the production ones; only the
  transport differs.
* one distinct device per rank (run when the box shows at least that many GPUs, skipped
  otherwise): no NCCL_HOSTID, LOCAL_RANK = rank, so RCCL connects the ranks peer-to-peer over
  xGMI. These check what the one-device family cannot: what RCCL formed (ncclCommCount /
  UserRank / CuDevice), the P2P transport, the gated launch's system-scope gate with remote
  writes, the collectives captured into the step graph, and a dead peer on another GPU.
"""
import json
import os
import socket
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, n, steps, strategy="allgather", mode="auto",
            dtype="fp32", env=None, devices=False):
    if devices:
        # one GPU per rank, one host: RCCL's intra-node transports (P2P over xGMI); the INFO
        # log names the transport of every connection
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank), NCCL_DEBUG="INFO",
                          NCCL_DEBUG_SUBSYS="INIT,P2P,NET",
                          NCCL_DEBUG_FILE=os.path.join(out_dir, f"rccl.{rank}.log"))
        os.environ.pop("GRAVSIM_RCCL_RANK_HOSTS", None)
    else:
        # one "host" per rank (see the module docstring): gravsim.parallel.comm.rccl_rank_hosts
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK="0", GRAVSIM_RCCL_RANK_HOSTS="1")
    os.environ.update(env or {})
    if os.environ.get("GRAVSIM_TEST_NCCL_DEBUG"):  # diagnostics: RCCL INFO log per rank
        os.makedirs(os.environ["GRAVSIM_TEST_NCCL_DEBUG"], exist_ok=True)
        os.environ.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,BOOTSTRAP,NET,GRAPH,ENV",
                          NCCL_DEBUG_TIMESTAMP_FORMAT="%H:%M:%S.%f ",
                          NCCL_DEBUG_FILE=os.path.join(os.environ["GRAVSIM_TEST_NCCL_DEBUG"],
                                                       f"w{world}_n{n}_r{rank}.log"))
    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.parallel import comm
    from gravsim.runtime.engines import HipEngine

    t_mark = [("start", time.perf_counter())]
    dist = comm.init(timeout_s=120)
    t_mark.append(("gloo_init", time.perf_counter()))
    status = "ok"
    try:
        # "<mode>-graph": the multi-rank step, collectives included, captured in a hipGraph;
        # "<mode>-eager": no graphs at all (the default replays a segmented plan: compute
        # segments as graphs, collectives eager between them)
        graph_comm = mode.endswith("-graph")
        eager = mode.endswith("-eager")
        cfg = SimConfig(n=n, dtype=dtype, device="gpu", chunk=1024, step_timeout_s=120,
                        strategy=strategy, mode=mode.removesuffix("-graph").removesuffix("-eager"),
                        graph_comm=graph_comm, graph=not eager)
        eng = HipEngine(cfg, rank, world, device=rank if devices else 0, dist=dist)
        uid = HipEngine.unique_id() if rank == 0 else None
        uid = comm.broadcast_bytes(dist, uid)
        t_mark.append(("engine", time.perf_counter()))
        try:
            eng.comm_init(uid)
        except RuntimeError as e:
            status = "comm_init failed: " + str(e)
        t_mark.append(("rccl_init", time.perf_counter()))
        ok = comm.allreduce_sum(dist, 0.0 if status == "ok" else 1.0)
        if ok == 0:
            import torch

            from gravsim.parallel.guard import parse_rccl_log

            p = torch.cuda.get_device_properties(eng.device)
            with open(os.path.join(out_dir, f"topo{rank}.json"), "w") as f:
                json.dump({"rank": rank, "device": eng.device, "host": "this",
                           "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
                           **eng.comm_info(),
                           **parse_rccl_log(os.environ.get("NCCL_DEBUG_FILE"))}, f)
            eng.init_ics("solar+random", 5)
            eng.audit_reset()
            eng.step(steps)
            eng.sync(timeout_s=120)
            t_mark.append(("steps", time.perf_counter()))
            done, per = eng.audit()
            gi = eng.graph_info()
            with open(os.path.join(out_dir, f"audit{rank}.txt"), "w") as f:
                f.write(f"{done} {per} {gi['mode']} {gi['segments']}")
            b = eng.state()
            own = eng.layout.real_local  # velocities are rank-local (positions are gathered)
            np.save(os.path.join(out_dir, f"vel{rank}.npy"), b.vel[own.start:own.stop])
            if rank == 0:
                np.save(os.path.join(out_dir, "pos.npy"), b.pos)
                with open(os.path.join(out_dir, "mode.txt"), "w") as f:
                    f.write(str(eng.native_layout["mode"]))
            # two more steps with phase events (after the saved state; state() gathered the
            # current buffer, so the second step is the one that runs the collectives)
            eng.set_timing(True)
            eng.step(2)
            ps = eng.phase_stats()
            eng.set_timing(False)
            if rank == 0:
                with open(os.path.join(out_dir, "comm_ms.txt"), "w") as f:
                    f.write(repr(ps["comm_ms"]))
            t_mark.append(("state_phase", time.perf_counter()))
        eng.close()
        t_mark.append(("close", time.perf_counter()))
    finally:
        # GRAVSIM_TEST_TIMES=<file>: per-rank phase seconds, appended as one JSON line
        if os.environ.get("GRAVSIM_TEST_TIMES"):
            with open(os.environ["GRAVSIM_TEST_TIMES"], "a") as f:
                f.write(json.dumps({"world": world, "rank": rank, "n": n, "mode": mode,
                                    "strategy": strategy, **{
                                        t_mark[i][0]: round(t_mark[i][1] - t_mark[i - 1][1], 3)
                                        for i in range(1, len(t_mark))}}) + "\n")
        if rank == 0:
            with open(os.path.join(out_dir, "status.txt"), "w") as f:
                f.write(status)
        comm.shutdown(dist)


OV3 = {"GRAVSIM_SYM_OVERLAP": "3"}  # one local-first launch, remote units gated (the default)
OV0 = {"GRAVSIM_SYM_OVERLAP": "0"}  # wait for the gather, then one launch
_GRAPH_COMM_XFAIL = pytest.mark.xfail(
    reason="capturing RCCL collectives over the socket transport crashes inside "
           "hipStreamEndCapture (profiles/r2_graph_comm_root_cause.txt); the default "
           "segmented plan keeps RCCL out of the capture", strict=False)


@pytest.mark.parametrize("world,strategy,mode,dtype,n,env", [
    (2, "allgather", "auto", "fp32", 5000, None),
    (2, "ring", "auto", "fp32", 5000, None),
    (2, "allgather", "sym", "fp32", 20000, None),
    (4, "allgather", "sym", "fp32", 20000, None),
    (8, "allgather", "sym", "fp32", 20000, None),  # the 8-GPU shape: one group per destination
    (2, "allgather", "sym", "fp64", 20000, None),
    (4, "ring", "split", "fp32", 9000, None),
    (8, "allgather", "sym", "fp32", 40000, OV3),
    # ring strategy of the sym schedule: P-1 neighbour stages, each gating its own units
    (2, "ring", "sym", "fp32", 20000, None),
    (4, "ring", "sym", "fp32", 40000, None),
    (8, "ring", "sym", "fp32", 40000, None),
    # P not dividing the row blocks (40,000 bodies: 8 blocks): uneven slices, the all-gather
    # as one group of in-place broadcasts, mpi.c's remainder rule
    (3, "allgather", "sym", "fp32", 40000, None),
    (6, "allgather", "sym", "fp32", 40000, None),
    (3, "ring", "sym", "fp32", 40000, None),
    (5, "allgather", "sym-eager", "fp64", 40000, OV0),
    # the round-2 default (ungated, eager) and ungated under the segmented plan
    (2, "allgather", "sym-eager", "fp32", 40000, OV0),
    (8, "allgather", "sym", "fp32", 40000, OV0),
    (2, "allgather", "sym-eager", "fp64", 20000, None),
    # "sym-graph": capturing the multi-rank step, collectives included, over RCCL's socket
    # transport segfaulted inside a rank (round 1: profiles/r1_rccl_multi_rank_tests.log;
    # round 2: profiles/r2_graph_comm_root_cause.txt). It stays opt-in (--graph-comm) and is
    # kept here as an expected failure so its status shows in every run; the remaining
    # capture cases run on request (GRAVSIM_TEST_GRAPH_COMM=1).
    pytest.param(2, "allgather", "sym-graph", "fp32", 20000, None, marks=_GRAPH_COMM_XFAIL),
    *([(2, "allgather", "auto-graph", "fp32", 5000, None),  # split: all-gather only
       (4, "allgather", "sym-graph", "fp32", 20000, None),
       (4, "allgather", "sym-graph", "fp32", 40000, OV3)]
      if os.environ.get("GRAVSIM_TEST_GRAPH_COMM") == "1" else []),
])
def test_rccl_multi_rank_match_single_rank(hip, tmp_path, world, strategy, mode, dtype, n, env):
    """P real RCCL ranks (one process each) give the same bits as one rank without a
    communicator (the canonical decomposition makes the result P-independent)."""
    _run_and_check(tmp_path, world, strategy, mode, dtype, n, env, devices=False)


def _run_and_check(tmp_path, world, strategy, mode, dtype, n, env, devices, steps=5):
    tmp_path.mkdir(parents=True, exist_ok=True)
    mp.start_processes(_worker, args=(world, _port(), str(tmp_path), n, steps, strategy, mode,
                                      dtype, env, devices),
                       nprocs=world, start_method="spawn", join=True)
    status = open(tmp_path / "status.txt").read()
    assert status == "ok", f"RCCL with {world} ranks: {status[:300]}"
    from gravsim.config import SimConfig
    from gravsim.runtime.engines import HipEngine

    variant = mode
    mode = mode.removesuffix("-graph").removesuffix("-eager")
    for r in range(world):  # every rank ran exactly its units, from the expected schedule
        done, per, gmode, segs = open(tmp_path / f"audit{r}.txt").read().split()
        if mode == "sym":
            assert int(done) == int(per) * steps and int(per) > 0, (r, done, per)
            want = {"-eager": "eager", "-graph": "graph"}.get(variant[len(mode):], "segmented")
            assert gmode == want, (r, gmode, want)
            if want == "segmented":
                # flag sync (all-gather): one compute graph per period; the ring's event
                # points cut it into segments
                assert (int(segs) >= 4) if strategy == "ring" else (int(segs) == 1), segs
    # what RCCL formed: the whole job, this rank, the device the rank bound
    topo = [json.loads(open(tmp_path / f"topo{r}.json").read()) for r in range(world)]
    for t in topo:
        assert (t["rccl_nranks"], t["rccl_rank"], t["rccl_device"]) == \
            (world, t["rank"], t["device"]), t
    eng = HipEngine(SimConfig(n=n, dtype=dtype, device="gpu", chunk=1024, mode=mode))
    eng.init_ics("solar+random", 5)
    eng.step(steps)
    ref = eng.state()
    ref_mode = eng.native_layout["mode"]
    eng.close()
    if mode == "sym":  # (the one-sided multi-rank schedule is split; one rank may fuse)
        assert open(tmp_path / "mode.txt").read() == str(ref_mode)
    assert np.array_equal(np.load(tmp_path / "pos.npy"), ref.pos)
    vel = np.concatenate([np.load(tmp_path / f"vel{r}.npy") for r in range(world)])
    assert np.array_equal(vel, ref.vel)
    # every multi-rank schedule times its collectives (all-gather or ring stages + exchange)
    assert float(open(tmp_path / "comm_ms.txt").read()) > 0.0
    return topo


def _need_devices(hip, world):
    n = int(hip.gs_hip_device_count())
    if n < world:
        pytest.skip(f"needs {world} distinct GPUs, the box shows {n}")


@pytest.mark.parametrize("world,strategy,mode,dtype,n,env", [
    (2, "allgather", "sym", "fp32", 20000, OV3),
    (2, "allgather", "sym", "fp64", 20000, None),
    (3, "allgather", "sym", "fp32", 40000, None),  # uneven blocks: broadcast group
    (4, "allgather", "sym", "fp32", 40000, OV3),
    (4, "ring", "sym", "fp32", 40000, None),
    (8, "allgather", "sym", "fp32", 40000, OV3),   # the headline shape: gated + node exchange
    (8, "allgather", "sym", "fp32", 40000, OV0),
    (8, "allgather", "sym-eager", "fp32", 40000, OV3),
    (8, "ring", "sym", "fp32", 40000, None),
    (8, "allgather", "auto", "fp32", 9000, None),   # one-sided split schedule
])
def test_rccl_distinct_devices_match_single_rank(hip, tmp_path, world, strategy, mode, dtype, n,
                                                 env):
    """One process per distinct GPU (no NCCL_HOSTID): RCCL's peer-to-peer transport over
    xGMI, the gated launch reading rows that peers wrote through the system-scope gate, and
    the node-sum exchange between devices; bitwise equal to one rank, and every connection
    P2P, none through a network transport."""
    _need_devices(hip, world)
    topo = _run_and_check(tmp_path, world, strategy, mode, dtype, n, env, devices=True)
    assert len({t["pci"] for t in topo}) == world, topo  # one GPU per rank
    from gravsim.parallel import verify

    for t in topo:
        assert t["transports"], f"rank {t['rank']}: no transport parsed from the RCCL log"
    assert verify.topology_problems(world, topo) == [], topo
    assert verify.transport_summary(topo)["p2p"], topo


@pytest.mark.parametrize("world,mode,n,env", [
    (2, "sym-graph", 20000, None),
    (2, "auto-graph", 5000, None),      # one-sided split: the all-gather captured
    (4, "sym-graph", 40000, OV3),       # gated launch + gate kernels + exchange captured
    (8, "sym-graph", 40000, OV3),
])
def test_rccl_graph_comm_distinct_devices(hip, tmp_path, world, mode, n, env):
    """--graph-comm on real devices: the whole multi-rank step, RCCL collectives included,
    captured in one hipGraph and replayed, bitwise equal to eager steps and to one rank. Over
    the one-device socket transport this capture crashes (the xfail above); on distinct GPUs
    it runs automatically."""
    _need_devices(hip, world)
    _run_and_check(tmp_path / "graph", world, "allgather", mode, "fp32", n, env, devices=True)
    eager = mode.replace("-graph", "-eager")
    _run_and_check(tmp_path / "eager", world, "allgather", eager, "fp32", n, env, devices=True)
    assert np.array_equal(np.load(tmp_path / "graph" / "pos.npy"),
                          np.load(tmp_path / "eager" / "pos.npy"))


@pytest.mark.parametrize("graph,strategy", [(1, "allgather"), (2, "allgather"), (1, "ring"),
                                            (2, "ring"), (1, "sym"), (2, "sym"), (1, "sym3"),
                                            (2, "sym3")])
def test_rccl_one_rank_full_schedule_bitwise(hip, monkeypatch, graph, strategy):
    """A live 1-rank RCCL communicator drives the whole multi-rank step (in-place
    ncclAllGather, concurrent local/remote split, ordered reduce) — eagerly (one-sided
    schedule, graph 1), as a segmented plan (sym, graph 1: compute segments captured, the
    collectives eager between them) and captured whole (use_graph=2 captures the collective
    too) — and must match the plain path."""
    from gravsim.config import SimConfig
    from gravsim.runtime.engines import HipEngine

    monkeypatch.setenv("GRAVSIM_FORCE_COMM", "1")
    # "sym": the Newton-3 schedule (all-gather, then the node-sum exchange through RCCL);
    # "sym3": the same with the gated local-first launch (graph 2 captures the gate kernels).
    sym = strategy.startswith("sym")
    if strategy == "sym3":
        monkeypatch.setenv("GRAVSIM_SYM_OVERLAP", "3")
    mode = "sym" if sym else "auto"
    cfg = SimConfig(n=6000, dtype="fp32", device="gpu", chunk=1024, mode=mode,
                    strategy="allgather" if sym else strategy)
    eng = HipEngine(cfg)
    eng.lib.gs_stepper_destroy(eng._s)  # rebuild with the requested graph mode
    import ctypes

    from gravsim.ops import _native
    from gravsim.runtime.engines import _gs_config

    c = _gs_config(cfg, 0, 1, 0)
    c.use_graph = graph
    eng._s = ctypes.c_void_p()
    _native.check(eng.lib, eng.lib.gs_stepper_create(ctypes.byref(c), ctypes.byref(eng._s)),
                  "create")
    eng.comm_init(HipEngine.unique_id())
    eng.init_ics("solar+random", 4)
    eng.step(7)
    eng.sync(timeout_s=60)
    gi = eng.graph_info()
    if sym and graph == 1:  # a live communicator: the plan, RCCL outside the graph (flag
        # sync: one compute graph per period)
        assert gi["mode"] == "segmented" and gi["segments"] >= 1, gi
    got = eng.state().pos
    eng.close()
    monkeypatch.delenv("GRAVSIM_FORCE_COMM")
    monkeypatch.delenv("GRAVSIM_SYM_OVERLAP", raising=False)
    ref_eng = HipEngine(cfg)
    ref_eng.init_ics("solar+random", 4)
    ref_eng.step(7)
    ref = ref_eng.state().pos
    ref_eng.close()
    assert np.array_equal(got, ref)


def _dead_peer_worker(rank, world, port, out_dir, devices=False):
    """Rank 1 dies after the communicator is up, before any step's collective; rank 0 steps
    and must get an error from its bounded wait instead of hanging in the exchange."""
    import time

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank) if devices else "0")
    if not devices:
        os.environ["GRAVSIM_RCCL_RANK_HOSTS"] = "1"
    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.parallel import comm
    from gravsim.runtime.engines import HipEngine

    dist = comm.init(timeout_s=60)
    cfg = SimConfig(n=20000, dtype="fp32", device="gpu", chunk=1024, mode="sym",
                    step_timeout_s=10)
    eng = HipEngine(cfg, rank, world, device=rank if devices else 0, dist=dist)
    uid = HipEngine.unique_id() if rank == 0 else None
    eng.comm_init(comm.broadcast_bytes(dist, uid))
    eng.init_ics("solar+random", 5)
    eng.sync()
    comm.barrier(dist)
    if rank != 0:
        os._exit(0)  # the peer is gone: no step, no collective, no clean shutdown
    t0 = time.time()
    msg = "no error"
    try:
        eng.step(3)
        eng.sync(timeout_s=10)
    except RuntimeError as e:
        msg = str(e)
    with open(os.path.join(out_dir, "rank0.txt"), "w") as f:
        f.write(f"{time.time() - t0:.2f}\n{msg}")
    os._exit(3 if "communicator aborted" in msg else 4)  # skip teardown with a dead peer


@pytest.mark.parametrize("devices", [False, True], ids=["one-device", "two-devices"])
def test_rccl_dead_peer_aborts_instead_of_hanging(hip, tmp_path, devices):
    """Failure detection (the reference has none, cuda.cu:145-177): a dead peer
    turns into an aborted communicator and a non-zero exit within the step timeout (over
    sockets on one device, and over P2P between two GPUs when the box has them)."""
    import multiprocessing

    if devices:
        _need_devices(hip, 2)
    ctx = multiprocessing.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_dead_peer_worker, args=(r, 2, port, str(tmp_path), devices))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(90)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
        p.join(10)
    assert not alive, "a rank hung with a dead peer"
    assert procs[1].exitcode == 0
    assert procs[0].exitcode == 3, (procs[0].exitcode, (tmp_path / "rank0.txt").read_text()
                                    if (tmp_path / "rank0.txt").exists() else "")
    took, msg = (tmp_path / "rank0.txt").read_text().split("\n", 1)
    assert "communicator aborted" in msg
    assert float(took) < 30.0, took
