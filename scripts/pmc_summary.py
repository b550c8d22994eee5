"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc_*/**/pmc_counter_collection.csv) for the
force kernels: per-counter totals over the profiled dispatches."""
import collections
import csv
import glob
import sys

rows = collections.defaultdict(float)
kern = collections.Counter()
for path in glob.glob(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_*/**/*counter_collection.csv",
                      recursive=True):
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name", "")
        if not any(k in name for k in ("force_split_kernel", "force_fused_kernel",
                                       "force_sym_kernel")):
            continue
        kern[name] += 1
        rows[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(rows.items()):
    print(f"{k:32s} {v:.6g}")
print("kernels:", dict(kern))
# The tiles issue one v_rsq (f32 or f64) per pair evaluation (per wave: 64 of them), so
# wave-level VALU instructions per trans instruction = VALU issue per pair, rsq included.
for kind in ("F32", "F64"):
    trans = rows.get(f"SQ_INSTS_VALU_TRANS_{kind}", 0.0)
    if not trans:
        continue
    print(f"{'VALU instructions per rsq_' + kind.lower():32s} {rows['SQ_INSTS_VALU'] / trans:.3f}"
          if rows.get("SQ_INSTS_VALU") else "")
    for c in ("FMA", "MUL", "ADD"):
        v = rows.get(f"SQ_INSTS_VALU_{c}_{kind}")
        if v:
            print(f"{'  ' + c + '_' + kind + ' per rsq':32s} {v / trans:.3f}")
    if rows.get("SQ_INSTS_LDS"):
        print(f"{'LDS instructions per rsq':32s} {rows['SQ_INSTS_LDS'] / trans:.3f}")
if rows.get("SQ_ACTIVE_INST_VALU") and rows.get("SQ_BUSY_CYCLES"):
    print(f"{'VALU-active / busy (per SQ)':32s} "
          f"{rows['SQ_ACTIVE_INST_VALU'] / rows['SQ_WAVE_CYCLES']:.3f} of wave-cycles")
if rows.get("SQ_LDS_BANK_CONFLICT") is not None and rows.get("SQ_LDS_IDX_ACTIVE"):
    print(f"{'LDS bank-conflict / active cycles':32s} "
          f"{rows['SQ_LDS_BANK_CONFLICT'] / rows['SQ_LDS_IDX_ACTIVE']:.3f}")
