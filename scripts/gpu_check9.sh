#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -rs > gpurun_out/pytest_gpu.log 2>&1; prc=$?
tail -3 gpurun_out/pytest_gpu.log; grep -E "^FAILED|^E  " gpurun_out/pytest_gpu.log | head -20
exit $prc
