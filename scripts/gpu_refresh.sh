#!/bin/bash
# Refresh the committed evidence for the current build: headline kernel stats, PMC passes
# (+ summary), 65K bench, the BASELINE configs table (incl. per-rank emulation of P = 8).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 > gpurun_out/prof_final.log 2>&1 || { tail -20 gpurun_out/prof_final.log; exit 1; }
cut -d, -f1-5 gpurun_out/prof_final/bench_kernel_stats.csv | head -6
bash scripts/profile_pmc.sh || exit $?
python scripts/pmc_summary.py > gpurun_out/pmc_summary.txt 2>&1; cat gpurun_out/pmc_summary.txt
timeout -k 10 200 python bench.py --num-bodies 65536 --steps 200 --warmup 20 > gpurun_out/b65.log 2>&1 || { tail -20 gpurun_out/b65.log; exit 1; }
tail -1 gpurun_out/b65.log | cut -c1-200
timeout -k 10 900 python bench/configs.py --md gpurun_out/baseline_configs.md > gpurun_out/baseline_configs.log 2>&1 || { tail -20 gpurun_out/baseline_configs.log; exit 1; }
cat gpurun_out/baseline_configs.md
