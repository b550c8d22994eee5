"""Build the gravsim native libraries in-tree.

  libgravsim_cpu.so : g++ -O3 -fopenmp, host-only CPU engine + layout/IC helpers.
  libgravsim_hip.so : hipcc --offload-arch=gfx950, kernels + Stepper runtime, links RCCL.
  gravsim_bench     : standalone C++ driver (csrc/tools/gravsim_main.cpp), no Python needed.

  probes (--tools)  : microbench, sym_probe, trans_probe, graph_event_probe, overlap_probe
                      (csrc/tools/*.hip);
                      measurement instruments, never part of the production build: a broken
                      probe cannot fail build_all() (the driver's build check).

Outputs land in <package>/_native/ so they travel with the repo snapshot to the GPU box.
Rebuilds only when a source or header is newer than the target. Usage:
    python csrc/build.py [--force] [--only cpu|hip|tool|microbench|sym_probe|trans_probe|
                          graph_event_probe|overlap_probe] [--tools]
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
PKG = ROOT / "gravity-simulator-using-mpi-spark-and-cuda_amd"
OUT = Path(os.environ["GRAVSIM_NATIVE_DIR"]) if os.environ.get("GRAVSIM_NATIVE_DIR") else \
    PKG / "_native"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("GRAVSIM_ARCH", "gfx950")

HEADERS = sorted((CSRC / "include").glob("*.h"))
CPU_SRC = [CSRC / "common" / "layout.cpp", CSRC / "cpu" / "cpu_engine.cpp"]
HIP_SRC = [CSRC / "common" / "layout.cpp", CSRC / "hip" / "nbody_kernels.hip",
           CSRC / "hip" / "nbody_sym.hip",
           CSRC / "hip" / "nbody_mfma.hip", CSRC / "hip" / "comm_model.hip",
           CSRC / "hip" / "ipc.hip", CSRC / "hip" / "stepper.hip",
           CSRC / "hip" / "stepper_comm.hip", CSRC / "hip" / "stepper_plan.hip"]
TOOL_SRC = [CSRC / "tools" / "gravsim_main.cpp"]

CPU_LIB = OUT / "libgravsim_cpu.so"
HIP_LIB = OUT / "libgravsim_hip.so"
TOOL_BIN = OUT / "gravsim_bench"
MICRO_SRC = CSRC / "tools" / "microbench.hip"
MICRO_BIN = OUT / "microbench"
PROBE_SRC = CSRC / "tools" / "sym_probe.hip"
PROBE_BIN = OUT / "sym_probe"
TRANS_SRC = CSRC / "tools" / "trans_probe.hip"
TRANS_BIN = OUT / "trans_probe"
GEV_SRC = CSRC / "tools" / "graph_event_probe.hip"
GEV_BIN = OUT / "graph_event_probe"
OVL_SRC = CSRC / "tools" / "overlap_probe.hip"
OVL_BIN = OUT / "overlap_probe"


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps if d.exists())


def _run(cmd: list[str]) -> None:
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def hipcc() -> str:
    p = ROCM / "bin" / "hipcc"
    return str(p) if p.exists() else (shutil.which("hipcc") or "hipcc")


def build_cpu(force: bool = False) -> Path:
    OUT.mkdir(parents=True, exist_ok=True)
    if force or _stale(CPU_LIB, CPU_SRC + HEADERS):
        cxx = os.environ.get("CXX", "g++")
        tmp = CPU_LIB.with_suffix(".so.tmp")
        _run([cxx, "-O3", "-std=c++17", "-fopenmp", "-march=x86-64-v3", "-ffp-contract=off",
              "-fPIC", "-shared", f"-I{CSRC / 'include'}", *map(str, CPU_SRC), "-o", str(tmp)])
        os.replace(tmp, CPU_LIB)
    return CPU_LIB


# SLP vectorisation packs the per-lane i-bodies into v_pk_{add,mul,fma}_f32; GRAVSIM_SLP=0
# builds the scalar-VALU variant for A/B runs.
HIP_FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fPIC"]
# The backend's max-ILP machine scheduler: same instructions (same bits), better interleaving
# of the packed-f32 / v_rsq streams. Alternating builds: 1M sym 164.9-165.2 vs 165.5 ms, 65K
# 0.717-0.718 vs 0.721-0.722 ms, 256K split 15.07-15.09 vs 16.56 ms, 8K fused 0.165 vs
# 0.198 ms, 128K sym -0.5 %, 256K fp64 split -1.8 %, 512K fp64 sym even
# (profiles/r2_sched_strategy_ab.jsonl, r2_sched_max_ilp_*_ab.jsonl). The auto schedule
# thresholds still hold with it (profiles/r2_s4_sizes_maxilp.txt).
if os.environ.get("GRAVSIM_SCHED", "max-ilp") != "default":
    HIP_FLAGS += ["-mllvm", f"-amdgpu-sched-strategy={os.environ.get('GRAVSIM_SCHED', 'max-ilp')}"]
# Loops aligned to 64-byte instruction-fetch lines: the sym force kernel's loops span 20-38 KB;
# with their heads left where the code happens to fall, the 1M step ran 1.0 % slower after an
# unrelated code change (164.0-164.2 vs 162.4-162.5 ms alternating on one box; aligned: 162.4-
# 162.5, profiles/r4_ab_align_loops.jsonl). Aligning pins the layout instead of leaving it to luck.
HIP_FLAGS += ["-falign-loops=64"]
if os.environ.get("GRAVSIM_SLP", "1") == "0":
    HIP_FLAGS.append("-fno-slp-vectorize")
HIP_FLAGS += os.environ.get("GRAVSIM_HIP_EXTRA", "").split()


OBJ = OUT / "obj"


def _objects(force: bool) -> list[Path]:
    """One object per HIP source (the same PIC objects go into the library and the tool),
    compiled in parallel: each translation unit is independent (no device code crosses them),
    and nbody_sym.hip alone takes most of a serial build."""
    from concurrent.futures import ThreadPoolExecutor

    OBJ.mkdir(parents=True, exist_ok=True)
    objs = [OBJ / (src.stem + ("_c" if src.suffix == ".cpp" else "") + ".o") for src in HIP_SRC]
    todo = [(src, o) for src, o in zip(HIP_SRC, objs) if force or _stale(o, [src, *HEADERS])]

    def one(job):
        src, o = job
        tmp = o.with_suffix(".o.tmp")
        cmd = [hipcc(), *HIP_FLAGS, "-c", f"-I{CSRC / 'include'}", str(src), "-o", str(tmp)]
        print("+", " ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            sys.stderr.write(r.stdout + r.stderr)
            raise subprocess.CalledProcessError(r.returncode, cmd)
        os.replace(tmp, o)

    jobs = int(os.environ.get("GRAVSIM_BUILD_JOBS", "0") or 0) or min(8, os.cpu_count() or 1)
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(one, todo))
    return objs


def build_hip(force: bool = False) -> Path:
    OUT.mkdir(parents=True, exist_ok=True)
    if force or _stale(HIP_LIB, HIP_SRC + HEADERS):
        objs = _objects(force)
        tmp = HIP_LIB.with_suffix(".so.tmp")
        _run([hipcc(), *HIP_FLAGS, "-shared", *map(str, objs), f"-L{ROCM / 'lib'}", "-lrccl",
              "-o", str(tmp)])
        os.replace(tmp, HIP_LIB)
    return HIP_LIB


def build_tool(force: bool = False) -> Path:
    OUT.mkdir(parents=True, exist_ok=True)
    deps = TOOL_SRC + HIP_SRC + HEADERS
    if all(p.exists() for p in TOOL_SRC) and (force or _stale(TOOL_BIN, deps)):
        objs = _objects(force)
        main_o = OBJ / "gravsim_main.o"  # (compiled apart: hipcc's -x hip would take the
        _run([hipcc(), *HIP_FLAGS, "-c", f"-I{CSRC / 'include'}", *map(str, TOOL_SRC),  # .o
              "-o", str(main_o)])                                            # as sources)
        tmp = TOOL_BIN.with_suffix(".tmp")
        _run([hipcc(), *HIP_FLAGS, str(main_o), *map(str, objs), f"-L{ROCM / 'lib'}", "-lrccl",
              f"-Wl,-rpath,{ROCM / 'lib'}", "-o", str(tmp)])
        os.replace(tmp, TOOL_BIN)
    return TOOL_BIN


def build_microbench(force: bool = False) -> Path:
    OUT.mkdir(parents=True, exist_ok=True)
    if MICRO_SRC.exists() and (force or _stale(MICRO_BIN, [MICRO_SRC])):
        tmp = MICRO_BIN.with_suffix(".tmp")
        _run([hipcc(), "-O3", "-std=c++17", f"--offload-arch={ARCH}", str(MICRO_SRC), "-o",
              str(tmp)])
        os.replace(tmp, MICRO_BIN)
    return MICRO_BIN


def build_sym_probe(force: bool = False) -> Path:
    """DPP issue-cost / sym register-tile probe (csrc/tools/sym_probe.hip)."""
    OUT.mkdir(parents=True, exist_ok=True)
    deps = [PROBE_SRC, *HEADERS]
    if PROBE_SRC.exists() and (force or _stale(PROBE_BIN, deps)):
        tmp = PROBE_BIN.with_suffix(".tmp")
        _run([hipcc(), "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fno-slp-vectorize",
              f"-I{CSRC / 'include'}", str(PROBE_SRC), "-o", str(tmp)])
        os.replace(tmp, PROBE_BIN)
    return PROBE_BIN


def build_trans_probe(force: bool = False) -> Path:
    """Transcendental / packed-VALU issue probe (csrc/tools/trans_probe.hip)."""
    OUT.mkdir(parents=True, exist_ok=True)
    if TRANS_SRC.exists() and (force or _stale(TRANS_BIN, [TRANS_SRC])):
        tmp = TRANS_BIN.with_suffix(".tmp")
        _run([hipcc(), "-O3", "-std=c++17", f"--offload-arch={ARCH}", str(TRANS_SRC), "-o",
              str(tmp)])
        os.replace(tmp, TRANS_BIN)
    return TRANS_BIN


def build_graph_event_probe(force: bool = False) -> Path:
    """External event-record / wait graph-node probe (csrc/tools/graph_event_probe.hip)."""
    OUT.mkdir(parents=True, exist_ok=True)
    if GEV_SRC.exists() and (force or _stale(GEV_BIN, [GEV_SRC])):
        tmp = GEV_BIN.with_suffix(".tmp")
        _run([hipcc(), "-O2", "-std=c++17", f"--offload-arch={ARCH}", str(GEV_SRC), "-o",
              str(tmp)])
        os.replace(tmp, GEV_BIN)
    lib = OUT / "libgraph_event_probe.so"  # the same probe, loaded under torch's HIP runtime
    if GEV_SRC.exists() and (force or _stale(lib, [GEV_SRC])):
        tmp = lib.with_suffix(".so.tmp")
        _run([hipcc(), "-O2", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-shared",
              "-DGS_PROBE_LIB", str(GEV_SRC), "-o", str(tmp)])
        os.replace(tmp, lib)
    return GEV_BIN


def build_overlap_probe(force: bool = False) -> Path:
    """Reduction-beside-force concurrency probe (csrc/tools/overlap_probe.hip)."""
    OUT.mkdir(parents=True, exist_ok=True)
    if OVL_SRC.exists() and (force or _stale(OVL_BIN, [OVL_SRC])):
        tmp = OVL_BIN.with_suffix(".tmp")
        _run([hipcc(), "-O3", "-std=c++17", f"--offload-arch={ARCH}", str(OVL_SRC), "-o",
              str(tmp)])
        os.replace(tmp, OVL_BIN)
    return OVL_BIN


def build_all(force: bool = False) -> None:
    """The production artefacts only: the CPU engine, the HIP library and gravsim_bench."""
    build_cpu(force)
    build_hip(force)
    build_tool(force)


def build_tools(force: bool = False) -> None:
    """The measurement probes (opt-in: --tools or --only <probe>)."""
    build_microbench(force)
    build_sym_probe(force)
    build_trans_probe(force)
    build_graph_event_probe(force)
    build_overlap_probe(force)


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["cpu", "hip", "tool", "microbench", "sym_probe",
                                          "trans_probe", "graph_event_probe", "overlap_probe"])
    ap.add_argument("--tools", action="store_true", help="also build the measurement probes")
    a = ap.parse_args(argv)
    if a.only == "cpu":
        build_cpu(a.force)
    elif a.only == "hip":
        build_hip(a.force)
    elif a.only == "tool":
        build_tool(a.force)
    elif a.only == "microbench":
        build_microbench(a.force)
    elif a.only == "sym_probe":
        build_sym_probe(a.force)
    elif a.only == "trans_probe":
        build_trans_probe(a.force)
    elif a.only == "graph_event_probe":
        build_graph_event_probe(a.force)
    elif a.only == "overlap_probe":
        build_overlap_probe(a.force)
    else:
        build_all(a.force)
        if a.tools:
            build_tools(a.force)
    return 0


if __name__ == "__main__":
    sys.exit(main())
