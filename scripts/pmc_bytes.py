"""HBM traffic and duration per kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs with
--kernel-trace (one counter pass per directory, joined on Dispatch_Id):
    python scripts/pmc_bytes.py <dir with FETCH_SIZE> [<dir with WRITE_SIZE>]
Prints one JSON line per kernel name: dispatches, mean duration (us), mean MB fetched / written
per dispatch, and the fetch bandwidth (TB/s). FETCH_SIZE / WRITE_SIZE are in KB (TCC)."""
import collections
import csv
import glob
import json
import sys


def short(n: str) -> str:
    return n.split("(gs::")[0].replace("void gs::(anonymous namespace)::", "").replace("void ", "")


def load(d: str):
    cnt = collections.defaultdict(float)   # (dispatch, counter) -> value
    names, dur = {}, {}
    for p in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            k = int(r["Dispatch_Id"])
            cnt[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            names[k] = short(r["Kernel_Name"])
    for p in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return cnt, names, dur


def main() -> int:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        cnt, names, dur = load(d)
        for (k, c), v in cnt.items():
            agg[names[k]][c].append(v)
            if k in dur:
                agg[names[k]]["_us"].append(dur[k])
    for n, m in sorted(agg.items()):
        us = m.get("_us", [])
        out = {"kernel": n[:70], "dispatches": len(m.get("FETCH_SIZE", m.get("WRITE_SIZE", []))),
               "us": round(sum(us) / len(us), 1) if us else None}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            if m.get(c):
                out[c.lower() + "_mb"] = round(sum(m[c]) / len(m[c]) / 1024, 1)
        if out.get("fetch_size_mb") and out["us"]:
            out["fetch_tb_s"] = round(out["fetch_size_mb"] / out["us"], 2)
        print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
