#!/bin/bash
# sym GPU tests + the RCCL one-rank schedule tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_sym.py tests/test_rccl_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_sym.log 2>&1 || { tail -60 gpurun_out/pytest_sym.log; exit 1; }
tail -1 gpurun_out/pytest_sym.log
