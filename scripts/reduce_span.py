"""Per-step wall span of the sym reduction kernels (node / block / row reduce, finalize) from
a rocprofv3 kernel-trace CSV: from the first reduce kernel's start after a force launch to the
last one's end before the next force launch. Usage: python scripts/reduce_span.py trace.csv"""
import csv
import statistics
import sys


def main(path: str) -> int:
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    spans, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if "force_sym_kernel" in name:
            if cur:
                spans.append(cur[1] - cur[0])
            cur = None
        elif any(k in name for k in ("node_reduce", "block_reduce", "row_reduce", "finalize")):
            cur = [t0, t1] if cur is None else [min(cur[0], t0), max(cur[1], t1)]
    if cur:
        spans.append(cur[1] - cur[0])
    us = [s / 1e3 for s in spans]
    print(f"{len(us)} steps: reduce span median {statistics.median(us):.1f} us, "
          f"min {min(us):.1f}, max {max(us):.1f}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
