#!/bin/bash
# sym GPU tests, then every BASELINE config (bench/configs.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sym.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_sym.log 2>&1 || { tail -60 gpurun_out/pytest_sym.log; exit 1; }
tail -1 gpurun_out/pytest_sym.log
timeout -k 10 900 python bench/configs.py --md gpurun_out/baseline_configs.md > gpurun_out/baseline_configs.log 2>&1 || { tail -20 gpurun_out/baseline_configs.log; exit 1; }
cat gpurun_out/baseline_configs.md
