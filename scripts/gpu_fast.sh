#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; prc=$?
tail -3 gpurun_out/pytest_gpu.log; grep -E "^FAILED" gpurun_out/pytest_gpu.log | head
[ $prc -le 1 ] || exit $prc
G="kernel=lds,smem;ipl=4,8;mode=split;cutoff_mode=exact,fast"
timeout -k 10 600 python bench/sweep.py --n 1048576 --steps 3 --rounds 2 --grid "$G" > gpurun_out/sweep_fast.log 2>&1 || exit $?
sed -n '/summary/,$p' gpurun_out/sweep_fast.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fast -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 > gpurun_out/prof_fast.log 2>&1 || exit $?

timeout -k 10 600 python bench/sweep.py --n 524288 --dtype fp64 --steps 2 --rounds 2 --grid "kernel=lds,smem;ipl=1,2,4;mode=split;cutoff_mode=exact,fast" > gpurun_out/sweep_fp64.log 2>&1 || exit $?
sed -n '/summary/,$p' gpurun_out/sweep_fp64.log
exit $prc
