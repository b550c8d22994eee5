"""One side of the two-process HIP IPC check (tests/test_ipc_gpu.py); run as a script.

    python tests/ipc_peer.py export <nbytes>   # allocate, fill, print handles, wait, verify
    python tests/ipc_peer.py import <nbytes> <mem handle hex> <event handle hex>

The exporter fills a device buffer with a counter pattern, prints `HANDLES <mem> <event>`
and waits for `CHECK` on stdin; the importer maps the buffer (hipIpcOpenMemHandle), checks
the pattern, writes its complement, records the interprocess event and exits; the exporter
then waits on that event on its own stream and checks the complement. Every failure is
printed as `FAIL <step>: <HIP error>` and exits 3.
"""
from __future__ import annotations

import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv: list[str]) -> int:
    import numpy as np

    import gravsim  # noqa: F401
    from gravsim.ops import _native

    lib = _native.hip_lib()
    role, nbytes = argv[0], int(argv[1])
    n = nbytes // 4
    want = np.arange(n, dtype=np.uint32) * np.uint32(2654435761)

    def ok(rc, step):
        if rc != 0:
            print(f"FAIL {step}: {lib.gs_last_error().decode(errors='replace')}", flush=True)
            sys.exit(3)

    if role == "export":
        p = ctypes.c_void_p()
        ok(lib.gs_dev_alloc(0, nbytes, ctypes.byref(p)), "hipMalloc")
        ok(lib.gs_dev_copy(p, want.ctypes.data, nbytes, 1), "fill")
        h = ctypes.create_string_buffer(64)
        ok(lib.gs_ipc_mem_handle(p, h), "hipIpcGetMemHandle")
        ev = ctypes.c_void_p()
        he = ctypes.create_string_buffer(64)
        ok(lib.gs_ipc_event_create(0, ctypes.byref(ev), he), "hipIpcGetEventHandle")
        print(f"HANDLES {h.raw.hex()} {he.raw.hex()}", flush=True)
        line = sys.stdin.readline().strip()
        if line != "CHECK":
            print(f"FAIL protocol: got {line!r}", flush=True)
            return 3
        ok(lib.gs_event_wait_sync(ev), "wait on the peer's interprocess event")
        got = np.empty(n, dtype=np.uint32)
        ok(lib.gs_dev_copy(got.ctypes.data, p, nbytes, 0), "read back")
        if not np.array_equal(got, ~want):
            print(f"FAIL verify: {int((got != ~want).sum())} of {n} words differ", flush=True)
            return 3
        lib.gs_event_destroy(ev)
        lib.gs_dev_free(p)
        print("EXPORT OK", flush=True)
        return 0

    hm, he = bytes.fromhex(argv[2]), bytes.fromhex(argv[3])
    q = ctypes.c_void_p()
    ok(lib.gs_ipc_mem_open(0, hm, ctypes.byref(q)), "hipIpcOpenMemHandle")
    got = np.empty(n, dtype=np.uint32)
    ok(lib.gs_dev_copy(got.ctypes.data, q, nbytes, 0), "read through the mapping")
    if not np.array_equal(got, want):
        print(f"FAIL verify: {int((got != want).sum())} of {n} words differ", flush=True)
        return 3
    inv = ~want
    ok(lib.gs_dev_copy(q, inv.ctypes.data, nbytes, 1), "write through the mapping")
    ev = ctypes.c_void_p()
    ok(lib.gs_ipc_event_open(0, he, ctypes.byref(ev)), "hipIpcOpenEventHandle")
    ok(lib.gs_event_record_sync(ev), "record the interprocess event")
    ok(lib.gs_ipc_mem_close(q), "hipIpcCloseMemHandle")
    print("IMPORT OK", flush=True)
    return 0


def pair(nbytes: int) -> int:
    """Run exporter + importer under this environment and print one JSON verdict line
    (scripts/gpu.sh ipc runs it with and without HSA_ENABLE_IPC_MODE_LEGACY=0)."""
    import json
    import subprocess

    env = dict(os.environ)
    a = subprocess.Popen([sys.executable, __file__, "export", str(nbytes)], stdin=subprocess.PIPE,
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
    log, ok = [], False
    try:
        line = ""
        for raw in a.stdout:
            line = raw.strip()
            log.append("A: " + line)
            if line.startswith(("HANDLES ", "FAIL")):
                break
        if line.startswith("HANDLES "):
            _, hm, he = line.split()
            b = subprocess.run([sys.executable, __file__, "import", str(nbytes), hm, he],
                               capture_output=True, text=True, timeout=120, env=env)
            log.append(f"B rc={b.returncode}: " + (b.stdout + b.stderr).strip()[-800:])
            a.stdin.write("CHECK\n" if b.returncode == 0 else "ABORT\n")
            a.stdin.flush()
            out = a.communicate(timeout=120)[0]
            log.append(f"A rc={a.returncode}: " + out.strip()[-800:])
            ok = b.returncode == 0 and a.returncode == 0 and "EXPORT OK" in out
    finally:
        if a.poll() is None:
            a.kill()
            a.wait()
    print(json.dumps({"HSA_ENABLE_IPC_MODE_LEGACY": env.get("HSA_ENABLE_IPC_MODE_LEGACY"),
                      "ipc_works": ok, "log": log}), flush=True)
    return 0


if __name__ == "__main__":
    if sys.argv[1:2] == ["pair"]:
        sys.exit(pair(int(sys.argv[2]) if len(sys.argv) > 2 else 4 << 20))
    sys.exit(main(sys.argv[1:]))
