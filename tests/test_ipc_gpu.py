"""Cross-process HIP IPC on one GPU (csrc/hip/ipc.hip, tests/ipc_peer.py).

RCCL's intra-node P2P transport, which an 8-GPU node uses for the per-step all-gather
(the reference's MPI_Allgatherv, mpi.c:227-236), maps peer buffers through HIP IPC. A one-GPU
box can only run RCCL over sockets (tests/test_rccl_gpu.py), so this checks the IPC layer
itself: process A exports a device buffer and an interprocess event, process B maps the
buffer, verifies and rewrites it and records the event, A waits on the event and verifies.

The launcher (parallel/launch.py) exports HSA_ENABLE_IPC_MODE_LEGACY=0 because this host's
driver supports only dmabuf IPC; the case without it records what the legacy mode does here.
"""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEER = os.path.join(ROOT, "tests", "ipc_peer.py")
NBYTES = 4 << 20


def _run_pair(env: dict) -> tuple[bool, str]:
    """(both sides OK, transcript)."""
    a = subprocess.Popen([sys.executable, PEER, "export", str(NBYTES)], stdin=subprocess.PIPE,
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env,
                         cwd=ROOT)
    log = []
    try:
        line = ""
        while True:  # (the runtime may print warnings first, e.g. a missing amdgpu.ids)
            line = a.stdout.readline()
            if not line:
                break
            line = line.strip()
            log.append(f"A: {line}")
            if line.startswith(("HANDLES ", "FAIL")):
                break
        if not line.startswith("HANDLES "):
            a.kill()
            rest = a.communicate(timeout=60)[0]
            return False, "\n".join(log) + "\n" + (rest or "")[-2000:]
        _, hm, he = line.split()
        b = subprocess.run([sys.executable, PEER, "import", str(NBYTES), hm, he], env=env,
                           capture_output=True, text=True, timeout=120, cwd=ROOT)
        log.append(f"B (rc {b.returncode}): {(b.stdout + b.stderr).strip()[-1500:]}")
        a.stdin.write("CHECK\n" if b.returncode == 0 else "ABORT\n")
        a.stdin.flush()
        out = a.communicate(timeout=120)[0]
        log.append(f"A (rc {a.returncode}): {out.strip()[-1500:]}")
        return b.returncode == 0 and a.returncode == 0 and "EXPORT OK" in out, "\n".join(log)
    finally:
        if a.poll() is None:
            a.kill()
            a.wait()


def test_ipc_memory_and_event_dmabuf_mode(hip):
    """The launcher's environment: HSA_ENABLE_IPC_MODE_LEGACY=0 (dmabuf). Must work."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    ok, log = _run_pair(env)
    print(f"[ipc] HSA_ENABLE_IPC_MODE_LEGACY=0: {'works' if ok else 'FAILS'}\n{log}")
    assert ok, log


def test_ipc_legacy_mode_recorded(hip):
    """Without HSA_ENABLE_IPC_MODE_LEGACY=0 (the runtime's legacy IPC mode). Recorded, not
    required: the task environment documents it failing with `hipIpcGetMemHandle: invalid
    argument` on this driver, which is why the launcher sets the variable. The test passes
    either way but fails if the legacy mode breaks in some other, unexplained way."""
    env = dict(os.environ)
    env.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)
    ok, log = _run_pair(env)
    print(f"[ipc] HSA_ENABLE_IPC_MODE_LEGACY unset: {'works' if ok else 'fails'}\n{log}")
    assert ok or "FAIL" in log, log
