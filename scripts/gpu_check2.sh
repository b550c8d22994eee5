#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; prc=$?
tail -2 gpurun_out/pytest_gpu.log; grep -E "^FAILED" gpurun_out/pytest_gpu.log | head
[ $prc -le 1 ] || exit $prc
timeout -k 10 120 ./gravity-simulator-using-mpi-spark-and-cuda_amd/_native/microbench > gpurun_out/microbench3.jsonl 2>&1 || exit $?
grep -E "f64|accuracy" gpurun_out/microbench3.jsonl
timeout -k 10 120 ./gravity-simulator-using-mpi-spark-and-cuda_amd/_native/gravsim_bench --n 65536 --steps 50 --log-dir gpurun_out/native_logs > gpurun_out/native_bench.log 2>&1 || exit $?
tail -1 gpurun_out/native_bench.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | cut -c1-400
exit $prc
