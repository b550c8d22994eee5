"""ctypes bindings to the in-tree native libraries (built by csrc/build.py).

libgravsim_cpu.so is host-only. libgravsim_hip.so holds the gfx950 kernels and the GPU
Stepper; torch is imported before it is loaded so that both share one HIP runtime (the
library's libamdhip64.so.7 / librccl.so.1 dependencies bind to the copies torch already
loaded, by soname). Missing libraries are built on demand when a compiler is available, and
otherwise raise NativeUnavailable — there is no silent Python fallback for the GPU path.
"""
from __future__ import annotations

import ctypes
import os
import threading
from ctypes import POINTER, c_double, c_float, c_int32, c_int64, c_uint64, c_void_p
from pathlib import Path

_HERE = Path(__file__).resolve().parent.parent
NATIVE_DIR = Path(os.environ["GRAVSIM_NATIVE_DIR"]) if os.environ.get("GRAVSIM_NATIVE_DIR") \
    else _HERE / "_native"
_REPO = _HERE.parent
_lock = threading.Lock()
_cpu = None
_hip = None


class NativeUnavailable(RuntimeError):
    pass


class GsConfig(ctypes.Structure):
    _fields_ = [
        ("n", c_int64), ("dtype", c_int32), ("kernel", c_int32), ("mode", c_int32),
        ("ipl", c_int32), ("chunk", c_int32), ("rank", c_int32), ("nranks", c_int32),
        ("device", c_int32), ("use_graph", c_int32), ("split_groups", c_int32),
        ("cutoff_mode", c_int32), ("strategy", c_int32), ("dt", c_double), ("G", c_double), ("cutoff", c_double), ("softening", c_double),
    ]


class GsLayout(ctypes.Structure):
    _fields_ = [
        ("n", c_int64), ("n_pad", c_int64), ("n_local", c_int64), ("local_begin", c_int64),
        ("chunk", c_int32), ("n_chunks", c_int32), ("ipl", c_int32), ("kernel", c_int32),
        ("mode", c_int32), ("split_groups", c_int32),
    ]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


GS_FP32, GS_FP64 = 0, 1
KERNEL_IDS = {"auto": 0, "lds": 1, "smem": 2, "mfma": 3}
MODE_IDS = {"auto": 0, "fused": 1, "split": 2, "sym": 3}
CUTOFF_IDS = {"auto": 0, "exact": 1, "fast": 2}
STRATEGY_IDS = {"allgather": 0, "ring": 1}
KERNEL_NAMES = {v: k for k, v in KERNEL_IDS.items()}
MODE_NAMES = {v: k for k, v in MODE_IDS.items()}

_P = c_void_p
_PD = POINTER(c_double)
_PF = POINTER(c_float)


def _build(which: str) -> None:
    import subprocess
    import sys

    script = _REPO / "csrc" / "build.py"
    if not script.exists():
        raise NativeUnavailable(f"{which} library missing and no build script at {script}")
    env = dict(os.environ, GRAVSIM_NATIVE_DIR=str(NATIVE_DIR))
    r = subprocess.run([sys.executable, str(script), "--only", which], capture_output=True,
                       text=True, env=env)
    if r.returncode != 0:
        raise NativeUnavailable(f"building libgravsim_{which}.so failed:\n{r.stdout}\n{r.stderr}")


def _sig(lib, name, res, args, optional=False):
    if optional and not hasattr(lib, name):
        return None
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = args
    return f


def _declare_common(lib) -> None:
    _sig(lib, "gs_last_error", ctypes.c_char_p, [])
    _sig(lib, "gs_layout_compute", c_int32, [POINTER(GsConfig), POINTER(GsLayout)])
    _sig(lib, "gs_sym_geometry", c_int32, [c_int64] + [POINTER(c_int32)] * 5)
    _sig(lib, "gs_sym_bytes", c_int64, [c_int64, c_int32, c_int32])
    _sig(lib, "gs_sym_shell_len", c_int32, [c_int32, c_int32])
    _sig(lib, "gs_sym_imbalance", c_double, [c_int64, c_int32])
    _sig(lib, "gs_sym_rank_rows", c_int32, [c_int64, c_int32, c_int32, POINTER(c_int32),
                                            POINTER(c_int32)])
    _sig(lib, "gs_sym_nodes", c_int32, [c_int64, c_int32, c_int32] + [POINTER(c_int32)] * 5)
    _sig(lib, "gs_sym_pair_live", c_int32, [c_int64, c_int32, c_int32, c_int32], optional=True)
    _sig(lib, "gs_sym_unit_map", c_int64, [c_int64, c_int32, c_int32, c_int64,
                                           POINTER(c_int32), c_int64])
    _sig(lib, "gs_sym_unit_map_ring", c_int64, [c_int64, c_int32, c_int32, c_int64,
                                                POINTER(c_int32), c_int64])
    _sig(lib, "gs_sym_unit_map_kr", c_int64, [c_int64, c_int32, c_int32, c_int64, c_int32,
                                              POINTER(c_int32), c_int64])
    _sig(lib, "gs_sym_split_segments", c_int32, [c_int64])
    # Np-part split segments (round 4); optional only so that A/B runs can load an older
    # library (scripts/build_variant.py of an earlier tree), whose split segments have 2 parts
    _sig(lib, "gs_sym_unit_map_parts", c_int64, [c_int64, c_int32, c_int32, c_int64, c_int32,
                                                 c_int32, POINTER(c_int32), c_int64], optional=True)
    _sig(lib, "gs_sym_split_parts", c_int32, [c_int64], optional=True)
    _sig(lib, "gs_auto_chunk", c_int32, [c_int64])
    _sig(lib, "gs_ic_fill_host", None, [c_int32, c_uint64, c_int64, c_int64, c_int64, _PD, _PD,
                                        _PD])


def cpu_lib():
    """Load (building if needed) libgravsim_cpu.so."""
    global _cpu
    with _lock:
        if _cpu is not None:
            return _cpu
        path = NATIVE_DIR / "libgravsim_cpu.so"
        if not path.exists() or os.environ.get("GRAVSIM_REBUILD"):
            _build("cpu")
        lib = ctypes.CDLL(str(path))
        _declare_common(lib)
        for t, P in (("f64", _PD), ("f32", _PF)):
            T = c_double if t == "f64" else c_float
            _sig(lib, f"gs_cpu_accel_{t}", c_int32, [P, c_int64, c_int64, c_int64, c_int32, T, T, P])
            _sig(lib, f"gs_cpu_step_{t}", c_int32,
                 [P, P, P, c_int64, c_int64, c_int64, c_int32, T, T, T])
        _sig(lib, "gs_cpu_accel_abs_f64", c_int32, [_PD, c_int64, c_int64, c_int64, c_double,
                                                    c_double, _PD])
        _sig(lib, "gs_cpu_accel_abs_ld", c_int32, [_PD, c_int64, c_int64, c_int64, c_double,
                                                    c_double, _PD])
        _sig(lib, "gs_cpu_num_threads", c_int32, [])
        _sig(lib, "gs_cpu_set_threads", c_int32, [c_int32])
        _cpu = lib
        return lib


def hip_lib():
    """Load libgravsim_hip.so (after torch, so the HIP runtime is shared)."""
    global _hip
    with _lock:
        if _hip is not None:
            return _hip
        import torch  # noqa: F401  (binds libamdhip64 / librccl first)

        path = NATIVE_DIR / "libgravsim_hip.so"
        if not path.exists() or os.environ.get("GRAVSIM_REBUILD"):
            _build("hip")
        try:
            lib = ctypes.CDLL(str(path))
        except OSError as e:  # pragma: no cover - depends on the box
            raise NativeUnavailable(f"cannot load {path}: {e}") from e
        _declare_common(lib)
        S = c_void_p
        _sig(lib, "gs_stepper_create", c_int32, [POINTER(GsConfig), POINTER(S)])
        _sig(lib, "gs_stepper_destroy", c_int32, [S])
        _sig(lib, "gs_stepper_layout", c_int32, [S, POINTER(GsLayout)])
        _sig(lib, "gs_stepper_init_ics", c_int32, [S, c_int32, c_uint64])
        _sig(lib, "gs_stepper_set_state", c_int32, [S, _PD, _PD, _PD])
        _sig(lib, "gs_stepper_get_state", c_int32, [S, _PD, _PD, _PD])
        _sig(lib, "gs_stepper_step", c_int32, [S, c_int32])
        _sig(lib, "gs_stepper_sync", c_int32, [S])
        _sig(lib, "gs_stepper_wait", c_int32, [S, c_double])
        _sig(lib, "gs_stepper_accel", c_int32, [S, _PD])
        _sig(lib, "gs_stepper_accel_step_path", c_int32, [S, _PD])
        _sig(lib, "gs_stepper_count_nonfinite", c_int64, [S])
        _sig(lib, "gs_stepper_steps_done", c_int64, [S])
        _sig(lib, "gs_stepper_period_start", c_int32, [S])
        _sig(lib, "gs_stepper_phase_ms", c_int32, [S, _PF, _PF, _PF])
        _sig(lib, "gs_stepper_set_timing", c_int32, [S, c_int32])
        _sig(lib, "gs_stepper_phase_stats", c_int32, [S, _PD])
        _sig(lib, "gs_stepper_set_overlap", c_int32, [S, c_int32])
        _sig(lib, "gs_stepper_set_schedule", c_int32, [S, c_int32, c_int32])
        _sig(lib, "gs_stepper_get_overlap", c_int32, [S])
        _sig(lib, "gs_stepper_get_dyn_cap", c_int32, [S])
        _sig(lib, "gs_stepper_set_cutoff_mode", c_int32, [S, c_int32])
        _sig(lib, "gs_stepper_set_tuning", c_int32, [S, c_int32, c_int32])
        _sig(lib, "gs_stepper_set_persist", c_int32, [S, c_int32], optional=True)
        _sig(lib, "gs_stepper_audit", c_int32, [S, POINTER(c_uint64), POINTER(c_uint64)])
        _sig(lib, "gs_stepper_audit_reset", c_int32, [S])
        # (optional: A/B runs load round-5 builds, which have neither)
        _sig(lib, "gs_stepper_clock", c_int32, [S, _PD], optional=True)
        _sig(lib, "gs_sym_tile_shape", c_int32, [c_int32] + [POINTER(c_int32)] * 3,
             optional=True)
        _sig(lib, "gs_stepper_graph_info", c_int32, [S, POINTER(c_int32), POINTER(c_int32)])
        _sig(lib, "gs_stepper_graph_steps", c_int32, [S], optional=True)
        _sig(lib, "gs_stepper_mem_entry", c_int32,
             [S, c_int32, POINTER(ctypes.c_char_p), POINTER(c_uint64)])
        _sig(lib, "gs_stepper_set_timeout", c_int32, [S, c_double])
        _sig(lib, "gs_stepper_unit_trace", c_int64, [S, c_void_p, c_int64])
        _sig(lib, "gs_stepper_compute_stream", c_void_p, [S])
        _sig(lib, "gs_stepper_force_mode", c_int32, [S, POINTER(c_int32), POINTER(c_double)])
        _sig(lib, "gs_group_step", c_int32, [POINTER(S), c_int32, c_int32])
        _sig(lib, "gs_rccl_unique_id", c_int32, [c_void_p])
        _sig(lib, "gs_stepper_comm_init", c_int32, [S, c_void_p, c_int32, c_int32])
        _sig(lib, "gs_stepper_comm_check", c_int32, [S])
        _sig(lib, "gs_stepper_comm_stage", c_int32, [S])
        _sig(lib, "gs_stepper_abort", c_int32, [S])
        _sig(lib, "gs_stepper_comm_info", c_int32, [S] + [POINTER(c_int32)] * 3, optional=True)
        _sig(lib, "gs_hip_device_count", c_int32, [])
        VP = POINTER(c_void_p)
        _sig(lib, "gs_dev_alloc", c_int32, [c_int32, c_uint64, VP])
        _sig(lib, "gs_dev_free", c_int32, [c_void_p])
        _sig(lib, "gs_dev_copy", c_int32, [c_void_p, c_void_p, c_uint64, c_int32])
        _sig(lib, "gs_ipc_mem_handle", c_int32, [c_void_p, c_void_p])
        _sig(lib, "gs_ipc_mem_open", c_int32, [c_int32, c_void_p, VP])
        _sig(lib, "gs_ipc_mem_close", c_int32, [c_void_p])
        _sig(lib, "gs_ipc_event_create", c_int32, [c_int32, VP, c_void_p])
        _sig(lib, "gs_ipc_event_open", c_int32, [c_int32, c_void_p, VP])
        for f in ("gs_event_record_sync", "gs_event_wait_sync", "gs_event_destroy"):
            _sig(lib, f, c_int32, [c_void_p])
        _sig(lib, "gs_hip_kernel_info", ctypes.c_char_p, [])
        _hip = lib
        return lib


def sym_tile_shape(fp64: bool) -> dict:
    """Compiled register-tile shape of the sym force kernels (nbody_sym.hip Shape<T>): waves
    per workgroup and i / j bodies per lane."""
    lib = hip_lib()
    if not hasattr(lib, "gs_sym_tile_shape"):  # (a round-5 build loaded for an A/B run)
        return {}
    w, i, j = c_int32(), c_int32(), c_int32()
    lib.gs_sym_tile_shape(int(bool(fp64)), ctypes.byref(w), ctypes.byref(i), ctypes.byref(j))
    return {"waves": w.value, "ipl": i.value, "jpl": j.value}


def sym_kernel_label(fp64: bool) -> str:
    """bench.py's description of the sym force kernel, from the compiled tile shape."""
    t = sym_tile_shape(fp64)
    if not t:
        return "sym: register tile (this library does not report its tile shape)"
    tile = (f"{t['ipl']} i x {t['jpl']} j per lane, "
            + ("fp64" if fp64 else "j-pair packed fp32" if t["jpl"] == 2 else "fp32"))
    return (f"sym: register tile (LDS-staged j, DPP carriers), {tile}, {t['waves']} waves, "
            "cyclic half-shell of 2048-body chunks")


def check(lib, rc: int, what: str) -> None:
    if rc != 0:
        msg = lib.gs_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed: {msg}")


def loaded_libraries() -> list[str]:
    out = []
    if _cpu is not None:
        out.append(str(NATIVE_DIR / "libgravsim_cpu.so"))
    if _hip is not None:
        out.append(str(NATIVE_DIR / "libgravsim_hip.so"))
    return out


def dptr(a):
    """ctypes double* of a contiguous float64 NumPy array."""
    return a.ctypes.data_as(_PD)


def fptr(a):
    return a.ctypes.data_as(_PF)
