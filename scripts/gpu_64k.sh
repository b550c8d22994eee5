#!/bin/bash
# 64K fp32 config: kernel trace (graph replay gaps, reduce cost) + focused tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "fused_engine or variants" > gpurun_out/pytest_64k.log 2>&1 || { tail -30 gpurun_out/pytest_64k.log; exit 1; }
tail -1 gpurun_out/pytest_64k.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_64k -o p --output-format csv -- python bench.py --n 65536 --steps 100 --warmup 10 > gpurun_out/prof_64k.log 2>&1 || exit $?
tail -1 gpurun_out/prof_64k.log | cut -c1-300
f=$(find gpurun_out/prof_64k -name "*kernel_stats.csv" | head -1); cut -d, -f1-6 "$f"
t=$(find gpurun_out/prof_64k -name "*kernel_trace.csv" | head -1)
python - "$t" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
force = [r for r in rows if "force_split" in r["Kernel_Name"]]
red = [r for r in rows if "reduce_integrate" in r["Kernel_Name"]]
print("force n", len(force), "reduce n", len(red))
# steady-state step: consecutive force kernel starts
st = [int(r["Start_Timestamp"]) for r in force][-60:]
d = [(b - a) / 1e3 for a, b in zip(st, st[1:])]
print("step period us: min %.1f median %.1f" % (min(d), sorted(d)[len(d)//2]))
fd = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in force[-60:])
rd = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in red[-60:])
print("force us median %.1f, reduce us median %.1f" % (fd[len(fd)//2], rd[len(rd)//2]))
gaps = []
for a, b in zip(rows[-120:], rows[-119:]):
    gaps.append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
gaps.sort()
print("inter-kernel gap us: median %.1f max %.1f" % (gaps[len(gaps)//2], gaps[-1]))
PY
