#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -rs > gpurun_out/pytest_gpu.log 2>&1; prc=$?
tail -2 gpurun_out/pytest_gpu.log; grep -E "^FAILED" gpurun_out/pytest_gpu.log | head
[ $prc -le 1 ] || exit $prc
timeout -k 10 300 python bench/sweep.py --n 65536 --steps 20 --rounds 3 --grid "kernel=lds,smem;ipl=2,4,8;mode=split" > gpurun_out/sweep_64k_v2.log 2>&1 || exit $?
sed -n '/summary/,$p' gpurun_out/sweep_64k_v2.log | head -7
timeout -k 10 300 python bench/sweep.py --n 262144 --steps 5 --rounds 2 --grid "kernel=lds,smem;ipl=4,8;mode=split" > gpurun_out/sweep_256k.log 2>&1 || exit $?
sed -n '/summary/,$p' gpurun_out/sweep_256k.log | head -5
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | cut -c1-300
exit $prc
