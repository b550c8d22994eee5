"""Comm/compute overlap from a rocprofv3 kernel trace (virtual ranks: the all-gather runs as
blit copies on the comm stream; per-rank emulation: comm_model kernels; real RCCL: nccl
kernels).

For every exchange kernel (copy or nccl) reports how much of its duration ran concurrently
with a force kernel, and the per-step timeline summary.
    python scripts/overlap_report.py <kernel_trace.csv>
"""
import csv
import sys


def main(path: str) -> int:
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
           r.get("Stream_Id", "?")) for r in rows]
    force = [(s, e) for s, e, n, _ in ks if "force_" in n]
    comm = [(s, e, n, st) for s, e, n, st in ks
            if "copyBuffer" in n or "nccl" in n.lower() or "comm_model" in n]
    if not force or not comm:
        print("no force or exchange kernels in trace")
        return 1
    # union of force-kernel busy intervals
    busy = []
    for s, e in sorted(force):
        if busy and s <= busy[-1][1]:
            busy[-1][1] = max(busy[-1][1], e)
        else:
            busy.append([s, e])
    first = busy[0][0]
    comm = [c for c in comm if c[0] >= first]  # exchanges of the stepping phase only
    t_ex = t_ov = 0
    for s, e, _, _ in comm:
        t_ex += e - s
        for bs, be in busy:
            t_ov += max(0, min(e, be) - max(s, bs))
    streams = sorted({st for *_, st in comm})
    fstreams = sorted({r.get("Stream_Id", "?") for r in rows if "force_" in r["Kernel_Name"]})
    print(f"exchange kernels: {len(comm)} on streams {streams}; force kernels: {len(force)} "
          f"on streams {fstreams}")
    print(f"exchange time {t_ex / 1e3:.1f} us, of which overlapped with force kernels "
          f"{t_ov / 1e3:.1f} us ({100.0 * t_ov / max(t_ex, 1):.1f} %)")
    # concurrency of the force kernels themselves (local vs remote streams)
    fs = sorted(force)
    conc = sum(max(0, min(a[1], b[1]) - max(a[0], b[0])) for i, a in enumerate(fs)
               for b in fs[i + 1:i + 8])
    tot = sum(e - s for s, e in fs)
    print(f"force kernel time {tot / 1e6:.2f} ms; pairwise concurrent force time "
          f"{conc / 1e6:.2f} ms (local and remote launches sharing the GPU)")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
