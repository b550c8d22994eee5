#!/bin/bash
# Profiles of the default (sym) headline path: kernel stats, PMC passes, per-rank emulation.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 > gpurun_out/prof_final.log 2>&1 || { tail -20 gpurun_out/prof_final.log; exit 1; }
bash scripts/profile_pmc.sh || exit $?
python scripts/pmc_summary.py > gpurun_out/pmc_summary.txt 2>&1; cat gpurun_out/pmc_summary.txt
timeout -k 10 600 python bench/rank_shape.py --n 1048576 --ranks 1,2,4,8 --mode sym > gpurun_out/rank_shape_sym.jsonl 2>&1 || { tail -20 gpurun_out/rank_shape_sym.jsonl; exit 1; }
cat gpurun_out/rank_shape_sym.jsonl
