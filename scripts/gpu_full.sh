#!/bin/bash
# Full GPU check: all gpu tests, smoke, default bench, BASELINE configs, kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
timeout -k 10 900 python bench/configs.py --md gpurun_out/baseline_configs.md > gpurun_out/baseline_configs.log 2>&1 || { tail -20 gpurun_out/baseline_configs.log; exit 1; }
cat gpurun_out/baseline_configs.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 > gpurun_out/prof_final.log 2>&1 || { tail -20 gpurun_out/prof_final.log; exit 1; }
head -5 gpurun_out/prof_final/bench_kernel_stats.csv
