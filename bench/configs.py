"""Run every BASELINE.json configuration that one MI355X (or the CPU) can measure.

  #1 1,024 bodies fp64, 100 steps, CPU engine (mpi.c world_size=1)        -> measured
  #2 65,536 bodies fp32, 1 GPU                                            -> measured
  #3 1,048,576 fp32, 8 GPUs  -> 1-GPU measurement + per-rank emulation of P = 8
  #4 4,194,304 fp64, 8 GPUs  -> per-rank emulation of P = 8 (rank 7 of 8)
  #5 16,777,216 fp32, 8 GPUs -> per-rank emulation of P = 8 (rank 7 of 8)

Per-rank emulation (GRAVSIM_EMULATE_RANK=1) runs one rank's exact launch shapes. Its
collectives are modeled (csrc/hip/comm_model.hip): the all-gather (1M fp32, P = 8: 14.7 MB
received per GPU) and the node-sum exchange (10.5 MB) become kernels of those byte counts
on the comm stream that stay resident for latency + bytes / rate, at a conservative
--comm-gbps (default 64 GB/s per rank, 15 us per collective; xGMI is 7 links x ~153 GB/s).
Whole-node body-updates/s is predicted as N / ms(rank) with that comm cost included. Writes
one JSON line per config and a markdown table (--md).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def gpu_run(n, dtype, steps, warmup, P=1, rank=0, overlap=None, **kw):
    from gravsim.config import SimConfig
    from gravsim.runtime.engines import HipEngine

    cfg = SimConfig(n=n, dtype=dtype, device="gpu", **kw)
    e = HipEngine(cfg, rank, P)
    if overlap is not None:
        e.set_overlap(overlap)
    e.init_ics("solar+random", cfg.seed)
    e.step(warmup)
    e.sync()
    e.clock()  # (reset: the engine clock of the timed steps only)
    t0 = time.perf_counter()
    e.step(steps)
    e.sync()
    ms = 1e3 * (time.perf_counter() - t0) / steps
    ghz = e.clock()["ghz"] or None  # (None: a schedule without clock stamps)
    lay = dict(e.native_layout, engine_clock_ghz=ghz)
    phase = None
    if P > 1:  # comm split of two more event-timed steps, replayed from the segmented plan
        e.align_period()
        e.set_timing(True)
        e.step(2)
        phase = e.phase_stats()
        e.set_timing(False)
    e.close()
    return ms, lay, phase


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="1,2,3,4,5,6")
    ap.add_argument("--md", default=None)
    ap.add_argument("--comm-gbps", type=float, default=64.0,
                    help="modeled per-rank collective rate of the 8-GPU emulations (0: free)")
    ap.add_argument("--comm-us", type=float, default=15.0)
    ap.add_argument("--overlap", type=int, default=3,
                    help="sym overlap mode of the 8-GPU emulations (default 3: the gated launch "
                         "bench.py's --overlap auto picks for multi-rank sym runs)")
    a = ap.parse_args()
    want = {int(x) for x in a.only.split(",")}
    rows = []

    if 1 in want:
        r = subprocess.run([sys.executable, "-m", "gravsim", "--n", "1024", "--steps", "100",
                            "--device", "cpu", "--dtype", "fp64", "--log-format", "none"],
                           cwd=ROOT, capture_output=True, text=True, timeout=600)
        m = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
        rows.append(dict(config="#1 1,024 fp64 CPU, 100 steps", gpus=0, how="measured",
                         ms_per_step=m["ms_per_step"], body_updates_per_s=m["body_updates_per_s"]))
        print(json.dumps(rows[-1]), flush=True)

    os.environ["GRAVSIM_EMULATE_RANK"] = "1"
    os.environ["GRAVSIM_EMU_COMM"] = f"{a.comm_gbps},{a.comm_us}"  # GB/s, latency us
    how8 = (f"per-rank emulation, modeled comm {a.comm_gbps:g} GB/s + {a.comm_us:g} us"
            if a.comm_gbps > 0 else "per-rank emulation, comm free")
    import torch  # noqa: F401

    import gravsim  # noqa: F401

    if 2 in want:
        ms, lay, _ = gpu_run(65536, "fp32", 300, 20)  # (bench.py --n 65536 --steps 300)
        rows.append(dict(config="#2 65,536 fp32", gpus=1, how="measured", ms_per_step=ms,
                         body_updates_per_s=65536 / (ms * 1e-3), layout=lay))
        print(json.dumps(rows[-1]), flush=True)
    if 3 in want:
        n = 1 << 20
        ms1, lay1, _ = gpu_run(n, "fp32", 5, 1)
        rows.append(dict(config="#3 1,048,576 fp32", gpus=1, how="measured", ms_per_step=ms1,
                         body_updates_per_s=n / (ms1 * 1e-3), layout=lay1))
        print(json.dumps(rows[-1]), flush=True)
        ms8, lay8, ph = gpu_run(n, "fp32", 5, 1, P=8, rank=7, overlap=a.overlap)
        rows.append(dict(config="#3 1,048,576 fp32", gpus=8, how=how8,
                         ms_per_step=ms8, body_updates_per_s=n / (ms8 * 1e-3),
                         predicted_efficiency=ms1 / (8 * ms8), layout=lay8, phase=ph))
        print(json.dumps(rows[-1]), flush=True)
    if 4 in want:
        n = 1 << 22
        ms8, lay8, ph = gpu_run(n, "fp64", 1, 1, P=8, rank=7, overlap=a.overlap)
        rows.append(dict(config="#4 4,194,304 fp64", gpus=8, how=how8,
                         ms_per_step=ms8, body_updates_per_s=n / (ms8 * 1e-3), layout=lay8,
                         phase=ph))
        print(json.dumps(rows[-1]), flush=True)
    if 6 in want:
        # the reference's own CUDA workload (cuda.cu:121-123: N = 50,000, fp32, 1 GPU)
        ms, lay, _ = gpu_run(50000, "fp32", 200, 10)
        rows.append(dict(config="cuda.cu's 50,000 fp32", gpus=1, how="measured", ms_per_step=ms,
                         body_updates_per_s=50000 / (ms * 1e-3), layout=lay))
        print(json.dumps(rows[-1]), flush=True)
    if 5 in want:
        n = 1 << 24
        ms8, lay8, ph = gpu_run(n, "fp32", 1, 0, P=8, rank=7, overlap=a.overlap)
        rows.append(dict(config="#5 16,777,216 fp32", gpus=8, how=how8,
                         ms_per_step=ms8, body_updates_per_s=n / (ms8 * 1e-3), layout=lay8,
                         phase=ph))
        print(json.dumps(rows[-1]), flush=True)

    if a.md:
        with open(a.md, "w") as f:
            from gravsim.ops._native import MODE_NAMES

            f.write("| config | GPUs | how | schedule | ms/step | engine GHz | body-updates/s | "
                    "comm ms | exposed comm ms |\n|---|---|---|---|---|---|---|---|---|\n")
            for r in rows:
                mode = MODE_NAMES.get(r.get("layout", {}).get("mode"), "cpu")
                ph = r.get("phase") or {}
                c = f"{ph['comm_ms']:.3f}" if ph else "-"
                x = f"{ph['exposed_comm_ms']:.3f}" if ph else "-"
                g = (r.get("layout") or {}).get("engine_clock_ghz")
                g = f"{g:.3f}" if g else "-"
                f.write(f"| {r['config']} | {r['gpus']} | {r['how']} | {mode} | "
                        f"{r['ms_per_step']:.3f} | {g} | {r['body_updates_per_s']:.4g} | {c} | "
                        f"{x} |\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
