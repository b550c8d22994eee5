"""Gaps between consecutive kernels of a rocprofv3 --kernel-trace CSV: how long the GPU sits
idle between the force launch and the tail kernel of a step, between the two steps of one
replayed hipGraph period, and between two graph launches.

  python scripts/kernel_gaps.py <kernel_trace.csv> [--match force_sym,sym_tail]

Only kernels whose name contains one of the --match substrings are kept (the timed loop's
kernels); the sequence is then force, tail, force, tail, ... and the tail -> force gaps
alternate between "inside a period" and "between graph launches" (a period is two steps).
"""
from __future__ import annotations

import argparse
import csv
import statistics as st


def load(path: str, match: list[str]) -> list[tuple[int, int, str]]:
    out = []
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name") or row.get("KernelName") or ""
            if not any(m in name for m in match):
                continue
            out.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), name))
    out.sort()
    return out


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--match", default="force_sym,sym_tail")
    a = ap.parse_args(argv)
    print(summarise(load(a.csv, a.match.split(","))))
    return 0


def summarise(ks: list[tuple[int, int, str]]) -> dict:
    """Durations and gaps (us) of a force / tail kernel sequence sorted by start time."""
    kinds = ["tail" if "tail" in n else "force" for _, _, n in ks]
    gaps: dict[str, list[float]] = {"force->tail": [], "tail->force": []}
    for i in range(1, len(ks)):
        key = f"{kinds[i - 1]}->{kinds[i]}"
        if key in gaps:
            gaps[key].append((ks[i][0] - ks[i - 1][1]) / 1e3)
    tf = gaps["tail->force"]
    # the two interleaved classes of tail -> force gaps (which is the graph boundary is the
    # one with the larger median)
    even, odd = tf[0::2], tf[1::2]
    med = lambda v: round(st.median(v), 2) if v else None  # noqa: E731
    dur = {k: [] for k in ("force", "tail")}
    for (s, e, _), k in zip(ks, kinds):
        dur[k].append((e - s) / 1e3)
    # gaps inside the step loop (longer ones are host pauses between bench phases)
    allgaps = [g for g in gaps["force->tail"] + tf if g < 100.0]
    steps = max(1, len(ks) // 2)
    return ({"kernels": len(ks), "force_us": med(dur["force"]), "tail_us": med(dur["tail"]),
           "idle_between_kernels_us_per_step": round(sum(g for g in allgaps if g > 0) / steps, 2),
           "gaps_over_5us": sum(1 for g in allgaps if g > 5.0),
           "gap_force_tail_us": med(gaps["force->tail"]),
           "gap_tail_force_even_us": med(even), "gap_tail_force_odd_us": med(odd),
           "step_us_median": med([(ks[i + 2][0] - ks[i][0]) / 1e3
                                  for i in range(0, len(ks) - 2, 2)])})


if __name__ == "__main__":
    raise SystemExit(main())
