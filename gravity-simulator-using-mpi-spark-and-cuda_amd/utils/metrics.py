"""Machine-readable run metrics (one JSON line per run) and timing helpers.

The reference reports only wall time: "Total execution time" / "Average time per step"
(mpi.c:245-247, pyspark.py:191-193) and "Simulation took" (cuda.cu:171). The headline
metric of this project (BASELINE.json) is body-updates/s = N * steps / wall, plus
interactions/s = N^2 * steps / wall for the direct O(N^2) sum.
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
    def interactions_per_s(self) -> float:
        return float(self.n) * self.n * self.steps / self.wall_s if self.wall_s > 0 else 0.0

    def to_json(self) -> str:
        d = asdict(self)
        d.update(ms_per_step=self.ms_per_step, body_updates_per_s=self.body_updates_per_s,
                 interactions_per_s=self.interactions_per_s)
        return json.dumps(d, sort_keys=True)


class Stopwatch:
    def __init__(self):
        self.t0 = time.perf_counter()

    def elapsed(self) -> float:
        return time.perf_counter() - self.t0
