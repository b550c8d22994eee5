#!/bin/bash
# GPU round: full gpu tests, microbenchmarks, kernel/schedule sweep, rocprofv3 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; prc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $prc -le 1 ] || exit $prc
timeout -k 10 120 ./gravity-simulator-using-mpi-spark-and-cuda_amd/_native/microbench > gpurun_out/microbench.jsonl 2>&1 || exit $?
cat gpurun_out/microbench.jsonl | cut -c1-200
timeout -k 10 600 python bench/sweep.py --n 1048576 --steps 3 --rounds 2 --grid "kernel=lds,smem;ipl=1,2,4;mode=fused,split" > gpurun_out/sweep_1m.log 2>&1 || exit $?
sed -n '/summary/,$p' gpurun_out/sweep_1m.log
timeout -k 10 300 python bench/sweep.py --n 65536 --steps 20 --rounds 3 --grid "kernel=lds,smem;ipl=1,2,4;mode=split" > gpurun_out/sweep_64k.log 2>&1 || exit $?
sed -n '/summary/,$p' gpurun_out/sweep_64k.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 > gpurun_out/prof_bench.log 2>&1 || exit $?
find gpurun_out/prof_bench -name "*stats*" | head
exit $prc
