#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python bench/configs.py --md gpurun_out/baseline_configs.md > gpurun_out/baseline_configs.log 2>&1 || { tail -20 gpurun_out/baseline_configs.log; exit 1; }
cat gpurun_out/baseline_configs.md
bash scripts/profile_pmc.sh || exit $?
python scripts/pmc_summary.py > gpurun_out/pmc_summary.txt 2>&1; cat gpurun_out/pmc_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 > gpurun_out/prof_final.log 2>&1 || exit $?
