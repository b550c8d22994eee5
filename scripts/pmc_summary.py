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
# fp32 tiles issue one v_rsq_f32 per pair-evaluation (per wave: 64 of them), so wave-level
# VALU instructions per trans instruction = VALU issue per pair, rsq included.
trans = rows.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
if trans and rows.get("SQ_INSTS_VALU"):
    print(f"{'VALU instructions per rsq':32s} {rows['SQ_INSTS_VALU'] / trans:.3f}")
if rows.get("SQ_INSTS_LDS") and trans:
    print(f"{'LDS instructions per rsq':32s} {rows['SQ_INSTS_LDS'] / trans:.3f}")
if rows.get("SQ_LDS_BANK_CONFLICT") is not None and rows.get("SQ_LDS_IDX_ACTIVE"):
    print(f"{'LDS bank-conflict / active cycles':32s} "
          f"{rows['SQ_LDS_BANK_CONFLICT'] / rows['SQ_LDS_IDX_ACTIVE']:.3f}")
