"""The serial chain after each step's main force launch, from a rocprofv3 kernel trace of one
process (bench/rank_shape.py or bench.py): per step, the time from the end of the main sym
force kernel to the start of the next one on the compute queue (the
P = 8 target is <= 0.12 ms), and the kernels in between with their durations and the gaps
before them.
    python scripts/post_force_chain.py <kernel_trace.csv> [--steps K] [--print-steps K]
Prints one JSON summary line (chain_us per step: median / min / max) and the kernel lists of
the last --print-steps steps.
"""
import argparse
import csv
import json
import statistics


def short(name: str) -> str:
    n = name.split("(gs::")[0].replace("void gs::(anonymous namespace)::", "")
    return n.replace("void ", "").replace("gs::(anonymous namespace)::", "")


def is_main_force(n: str) -> bool:
    # force_sym_kernel_f32<EXACT, DEFER, DYN[, PF]>: every instance but the deferred-unit launch
    if not n.startswith("force_sym_kernel"):
        return False
    args = [t.strip() for t in n[n.index("<") + 1:n.index(">")].split(",")]
    return not (len(args) > 1 and args[1] == "true")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--print-steps", type=int, default=2)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                  r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rows), key=lambda k: k[0])
    forces = [k for k in ks if is_main_force(k[2])]
    if len(forces) < 2:
        print(json.dumps({"error": "fewer than two force launches in the trace"}))
        return 1
    fq = forces[0][3]
    chains, listing = [], []
    for f0, f1 in zip(forces, forces[1:]):
        between = [k for k in ks if f0[1] <= k[0] < f1[0] and k[3] == fq]
        chains.append((f1[0] - f0[1]) / 1e3)
        items, t = [], f0[1]
        for s, e, n, q in between:
            items.append({"kernel": n[:60], "gap_us": round((s - t) / 1e3, 1),
                          "dur_us": round((e - s) / 1e3, 1)})
            t = e
        items.append({"kernel": "(next force)", "gap_us": round((f1[0] - t) / 1e3, 1)})
        comm = [k for k in ks if f0[1] <= k[0] < f1[0] and k[3] != fq]
        listing.append({"chain_us": round(chains[-1], 1), "compute_queue": items,
                        "other_queues": [{"kernel": n[:50], "start_us": round((s - f0[1]) / 1e3, 1),
                                          "dur_us": round((e - s) / 1e3, 1)}
                                         for s, e, n, q in comm]})
    c = chains[1:] or chains  # (the first step after the warm-up may carry a graph build)
    print(json.dumps({"steps": len(chains), "chain_us_median": round(statistics.median(c), 1),
                      "chain_us_min": round(min(c), 1), "chain_us_max": round(max(c), 1),
                      "force_ms_median": round(statistics.median(
                          [(f[1] - f[0]) / 1e6 for f in forces]), 3)}))
    for item in listing[-a.print_steps:]:
        print(json.dumps(item))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
