#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -rs > gpurun_out/pytest_gpu.log 2>&1; prc=$?
tail -4 gpurun_out/pytest_gpu.log; grep -E "^FAILED|SKIPPED" gpurun_out/pytest_gpu.log | head
[ $prc -le 1 ] || exit $prc
timeout -k 10 600 python bench/sweep.py --n 524288 --dtype fp64 --steps 2 --rounds 2 --grid "kernel=lds,smem;ipl=1,2,4;mode=split" > gpurun_out/sweep_fp64_halley.log 2>&1 || exit $?
sed -n '/summary/,$p' gpurun_out/sweep_fp64_halley.log
exit $prc
