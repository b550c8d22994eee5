"""Simulation configuration.

The reference has no configuration system: N, dt, steps and cores are source literals
(cuda.cu:121-123,155; mpi.c:107,146-148; pyspark.py:48,168-173,183-188). Here every knob is
a field of SimConfig and a CLI flag (gravsim/cli.py). Defaults reproduce the reference run:
dt = 3600 s, 500 steps, Sun/Earth/Mars + uniform random bodies, cutoff 1e-10 m, G = 6.67430e-11.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Optional

G_SI = 6.67430e-11  # cuda.cu:11, mpi.c:9, pyspark.py:46

DTYPES = ("fp32", "fp64")
DEVICES = ("auto", "cpu", "gpu")
KERNELS = ("auto", "lds", "smem", "mfma")
MODES = ("auto", "fused", "split", "sym")
COMMS = ("auto", "rccl", "gloo", "none")
LOG_FORMATS = ("mpi", "spark", "cuda", "none")


@dataclass
class SimConfig:
    n: int = 1024                 # bodies (cuda.cu:121 uses 50,000; mpi.c:107 uses 8)
    dt: float = 3600.0            # seconds (cuda.cu:123, mpi.c:148, pyspark.py:186)
    steps: int = 500              # (cuda.cu:155, mpi.c:147, pyspark.py:188)
    dtype: str = "fp64"           # fp32 (cuda.cu) | fp64 (mpi.c, pyspark.py)
    device: str = "auto"          # auto -> gpu when a HIP device is visible
    init: str = "solar+random"    # IC family, see gravsim.models.initial_conditions
    seed: int = 20250307
    G: float = G_SI
    cutoff: float = 1e-10         # hard cutoff radius (cuda.cu:39, mpi.c:64, pyspark.py:38)
    softening: float = 0.0        # Plummer softening length (0 = reference semantics)
    cutoff_mode: str = "auto"     # GPU: exact (select) | fast (overflow-safe core) | auto
    integrator: str = "kd"        # kd (reference kick-drift) | leapfrog (staggered KDK)
    kernel: str = "auto"          # GPU j-source variant: lds | smem
    mode: str = "auto"            # GPU schedule: fused | split | sym (Newton-3, fp32)
    ipl: int = 0                  # i-bodies per lane (0 = auto)
    chunk: int = 0                # canonical j-chunk (0 = auto from n)
    split_groups: int = 0
    graph: bool = True            # hipGraph replay of the step loop (single rank)
    graph_comm: bool = False      # also capture the multi-rank step, RCCL collectives included.
                                  # Off by default: over RCCL's socket transport the capture
                                  # crashes inside hipStreamEndCapture (a SIGSEGV no fallback
                                  # can catch; docs/DESIGN.md "hipGraph and RCCL").
    comm: str = "auto"            # rccl (GPU) | gloo (CPU) | none
    strategy: str = "allgather"   # multi-rank exchange: allgather | ring (pipelined send/recv)
    overlap: int = -1             # sym work beside the all-gather: 0 none, 3 gated local-first
                                  # launch; -1 native default (3 for P > 1 after a bitwise
                                  # self-check, as bench.py runs; GRAVSIM_SYM_OVERLAP overrides)
    threads: int = 0              # CPU engine OpenMP threads (0 = default)
    step_timeout_s: Optional[float] = None  # multi-rank hang detection: abort RCCL when no
                                  # step completes for this long; None = derived from the
                                  # measured step time (max(60 s, 20 x step), at most 240 s;
                                  # start-up is bounded by 180 s); 0 = unbounded
    # observability / IO
    log_dir: Optional[str] = None     # directory for the text log (None = no file)
    log_format: str = "mpi"           # mpi | spark | cuda | none
    progress_every: int = 100         # "Step s/steps" progress lines (mpi.c:192, cuda.cu:164)
    print_positions: int = 10         # final-position lines on stdout (cuda.cu:101)
    dump_path: Optional[str] = None   # final state dump (text, mpi.c format) or .npz
    dump_every: int = 0               # also dump positions (mpi.c format) every k steps
    checkpoint_dir: Optional[str] = None
    checkpoint_every: int = 0
    resume: Optional[str] = None
    record_every: int = 0             # trajectory recorder (pyspark.py:105,114-115)
    record_path: Optional[str] = None
    nan_check_every: int = 0          # NaN/Inf guard period (0 = only at the end)
    diagnostics: bool = False         # total energy, momentum, angular momentum at the start and
                                      # the end of the run (exact-cutoff potential, O(N^2) pass)
    diag_every: int = 0               # ... and every k steps (the passes are excluded from wall)
    metrics_json: Optional[str] = None
    phase_timing: bool = False        # GPU: per-step phase events (comm/compute split in the
                                      # metrics; eager steps, no graph replay)

    def validate(self) -> "SimConfig":
        if self.n < 1:
            raise ValueError("n must be >= 1")
        if self.steps < 0:
            raise ValueError("steps must be >= 0")
        if self.dtype not in DTYPES:
            raise ValueError(f"dtype must be one of {DTYPES}")
        if self.device not in DEVICES:
            raise ValueError(f"device must be one of {DEVICES}")
        if self.kernel not in KERNELS:
            raise ValueError(f"kernel must be one of {KERNELS}")
        if self.mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}")
        if self.comm not in COMMS:
            raise ValueError(f"comm must be one of {COMMS}")
        if self.log_format not in LOG_FORMATS:
            raise ValueError(f"log_format must be one of {LOG_FORMATS}")
        if self.kernel == "mfma" and (self.dtype != "fp32" or self.ipl > 1 or
                                      self.mode == "fused"):
            raise ValueError("kernel mfma is fp32, ipl 0/1, split schedule only")
        if self.mode == "sym" and self.kernel == "mfma":
            raise ValueError("mode sym has its own kernels (not --kernel mfma)")
        if self.ipl not in (0, 1, 2, 4, 8) or (self.ipl == 8 and self.dtype != "fp32"):
            raise ValueError("ipl must be 0, 1, 2, 4 (or 8 for fp32)")
        if self.chunk and self.chunk % 1024:
            raise ValueError("chunk must be a multiple of 1024")
        if self.integrator not in ("kd", "leapfrog"):
            raise ValueError("integrator must be kd or leapfrog")
        if self.cutoff_mode not in ("auto", "exact", "fast"):
            raise ValueError("cutoff_mode must be auto, exact or fast")
        if self.strategy not in ("allgather", "ring"):
            raise ValueError("strategy must be allgather or ring")
        if self.overlap not in (-1, 0, 3):
            raise ValueError("overlap must be -1 (default), 0 or 3")
        if self.diag_every < 0:
            raise ValueError("diag_every must be >= 0")
        if self.step_timeout_s is not None and self.step_timeout_s < 0:
            raise ValueError("step_timeout_s must be None (derived), or >= 0 (0 = unbounded)")
        if self.cutoff < 0 or self.softening < 0:
            raise ValueError("cutoff and softening must be >= 0")
        return self

    def replace(self, **kw) -> "SimConfig":
        return dataclasses.replace(self, **kw)

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)
