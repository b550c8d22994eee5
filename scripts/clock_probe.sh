#!/bin/bash
# Effective engine clock of the 1M force kernel (one GPU box):
#   bash scripts/clock_probe.sh  -> gpurun_out/pmc_clock/ (+ the per-dispatch table on stdout)
# One --pmc pass (kernel trace only). GRBM_GUI_ACTIVE counts engine cycles summed over the 8
# XCDs, so per dispatch GRBM_GUI_ACTIVE / 8 / duration is the clock the kernel ran at
# (profiles/r4s2_clock_pmc.txt: the cycle count is constant, the duration follows the clock).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_clock
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES -d gpurun_out/pmc_clock -o pmc --output-format csv \
  -- python bench.py --steps 2 --warmup 1 --check-samples 0 --phase-steps 0 --exact-steps 0 \
  --no-replay-audit --no-energy > gpurun_out/pmc_clock.log 2>&1 || { tail -20 gpurun_out/pmc_clock.log; exit 1; }
python - <<'PY'
import collections, csv, glob
cc = glob.glob("gpurun_out/pmc_clock/**/*counter_collection.csv", recursive=True)[0]
kt = glob.glob("gpurun_out/pmc_clock/**/*kernel_trace.csv", recursive=True)[0]
agg = collections.defaultdict(dict)
for r in csv.DictReader(open(cc)):
    a = agg[r["Dispatch_Id"]]
    a[r["Counter_Name"]] = a.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    a["name"] = r["Kernel_Name"]
trace = {r["Dispatch_Id"]: r for r in csv.DictReader(open(kt))}
for d, a in agg.items():
    if "force_sym" not in a["name"] or d not in trace:
        continue
    t = trace[d]
    dur = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) * 1e-9
    print(f"dispatch {d}: {dur * 1e3:.2f} ms, GRBM_GUI_ACTIVE {a['GRBM_GUI_ACTIVE']:.4e}, "
          f"{a['GRBM_GUI_ACTIVE'] / 8 / dur / 1e9:.3f} GHz, VALU {a['SQ_INSTS_VALU']:.4e}")
PY
