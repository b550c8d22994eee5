#!/bin/bash
# Kernel-trace evidence of exchange/compute overlap with 4 virtual ranks on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/overlap -o ov --output-format csv -- python bench/virtual_scaling.py --n 262144 --ranks 4 --steps 4 > gpurun_out/overlap.log 2>&1 || { tail -20 gpurun_out/overlap.log; exit 1; }
t=$(find gpurun_out/overlap -name "*kernel_trace.csv" | head -1)
python scripts/overlap_report.py "$t" | tee gpurun_out/overlap_report.txt
