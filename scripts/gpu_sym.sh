#!/bin/bash
# Newton-3 sym schedule: GPU tests, then 1M fp32 bench sym vs split, kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sym.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_sym.log 2>&1 || { tail -60 gpurun_out/pytest_sym.log; exit 1; }
tail -3 gpurun_out/pytest_sym.log
timeout -k 10 300 python bench.py --mode sym --steps 5 --warmup 1 > gpurun_out/bench_sym.log 2>&1 || { tail -20 gpurun_out/bench_sym.log; exit 1; }
tail -1 gpurun_out/bench_sym.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sym -o sym --output-format csv -- python bench.py --mode sym --steps 2 --warmup 1 > gpurun_out/prof_sym.log 2>&1 || { tail -20 gpurun_out/prof_sym.log; exit 1; }
find gpurun_out/prof_sym -name "*kernel_stats.csv" -exec cat {} \;
