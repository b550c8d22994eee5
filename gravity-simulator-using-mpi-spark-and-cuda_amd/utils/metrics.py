"""Machine-readable run metrics (one JSON line per run) and timing helpers.

The reference reports only wall time: "Total execution time" / "Average time per step"
(mpi.c:245-247, pyspark.py:191-193) and "Simulation took" (cuda.cu:171). The headline
metric of this project (BASELINE.json) is body-updates/s = N * steps / wall, plus
effective_interactions_per_s = N^2 * steps / wall (the ordered pair terms a one-sided direct
sum evaluates) and pair_evals_per_s, the pair evaluations actually performed: N(N-1)/2 per
step for the Newton-3 sym schedule, N^2 otherwise. `extra` carries the comm/compute split of
multi-rank GPU runs (comm_ms, exposed_comm_ms; --phase-timing).
"""
from __future__ import annotations

import json
import time
from dataclasses import asdict, dataclass, field


@dataclass
class RunMetrics:
    n: int
    steps: int
    dt: float
    dtype: str
    device: str
    nranks: int
    wall_s: float
    kernel: str = ""
    mode: str = ""
    extra: dict = field(default_factory=dict)

    @property
    def ms_per_step(self) -> float:
        return 1e3 * self.wall_s / self.steps if self.steps else 0.0

    @property
    def body_updates_per_s(self) -> float:
        return self.n * self.steps / self.wall_s if self.wall_s > 0 else 0.0

    @property
    def effective_interactions_per_s(self) -> float:
        return float(self.n) * self.n * self.steps / self.wall_s if self.wall_s > 0 else 0.0

    @property
    def pair_evals_per_s(self) -> float:
        if self.wall_s <= 0:
            return 0.0
        pairs = self.n * (self.n - 1) / 2 if self.mode == "sym" else float(self.n) * self.n
        return pairs * self.steps / self.wall_s

    def to_json(self) -> str:
        d = asdict(self)
        d.update(ms_per_step=self.ms_per_step, body_updates_per_s=self.body_updates_per_s,
                 effective_interactions_per_s=self.effective_interactions_per_s,
                 pair_evals_per_s=self.pair_evals_per_s)
        return json.dumps(d, sort_keys=True)


class Stopwatch:
    def __init__(self):
        self.t0 = time.perf_counter()

    def elapsed(self) -> float:
        return time.perf_counter() - self.t0
