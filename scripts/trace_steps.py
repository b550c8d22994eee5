"""Per-step kernel timeline of a rocprofv3 kernel trace of the sym step (one process):
force / group-reduce / row-reduce / finalize durations and the idle gaps between them on the
compute stream, split by schedule (overlap 3 steps contain the deferred-unit launch).
    python scripts/trace_steps.py <kernel_trace.csv>
"""
import collections
import csv
import sys


def short(name: str) -> str:
    n = name.split("(gs::")[0].replace("void gs::(anonymous namespace)::", "")
    return n.replace("void ", "")


def is_main_force(n: str) -> bool:
    # force_sym_kernel_f32<EXACT, DEFER, DYN[, PF]>: every instance but the deferred-unit launch
    if not n.startswith("force_sym_kernel"):
        return False
    args = [t.strip() for t in n[n.index("<") + 1:n.index(">")].split(",")]
    return not (len(args) > 1 and args[1] == "true")


def main(path: str) -> int:
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                  r.get("Stream_Id", "?")) for r in rows), key=lambda k: k[0])
    # steps: from one main force launch to the next finalize
    steps, cur = [], None
    for s, e, n, st in ks:
        if is_main_force(n) and (cur is None or cur.get("fin")):
            if cur and cur.get("fin"):
                steps.append(cur)
            cur = {"k": []}
        if cur is not None:
            cur["k"].append((s, e, n))
            if n.startswith("sym_finalize"):
                cur["fin"] = True
    if cur and cur.get("fin"):
        steps.append(cur)
    agg = collections.defaultdict(list)
    for stp in steps:
        k = stp["k"]
        deferred = any("false, true" in n or "true, true" in n for _, _, n in k)
        comp = [x for x in k if not x[2].startswith("comm_model") and not x[2].startswith("gate_set")
                and "copyBuffer" not in x[2]]
        span = (comp[-1][1] - comp[0][0]) / 1e3
        busy = sum(e - s for s, e, _ in comp) / 1e3
        force = sum(e - s for s, e, n in comp if n.startswith("force_sym")) / 1e3
        agg["ov3" if deferred else "ov0/1"].append((span, busy, force))
    for key, v in agg.items():
        n = len(v)
        print(f"{key}: {n} steps; step span {sum(x[0] for x in v)/n:.1f} us, compute-stream busy "
              f"{sum(x[1] for x in v)/n:.1f} us, force kernels {sum(x[2] for x in v)/n:.1f} us, "
              f"gaps {sum(x[0]-x[1] for x in v)/n:.1f} us")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
