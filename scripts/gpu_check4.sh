#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -rs > gpurun_out/pytest_gpu.log 2>&1; prc=$?
tail -2 gpurun_out/pytest_gpu.log; grep -E "^FAILED" gpurun_out/pytest_gpu.log | head
[ $prc -le 1 ] || exit $prc
G="kernel=smem,lds;ipl=2,4;mode=split"
for v in _native _native_newton _native _native_newton; do
  GRAVSIM_NATIVE_DIR=$PWD/gravity-simulator-using-mpi-spark-and-cuda_amd/$v timeout -k 10 300 python bench/sweep.py --n 524288 --dtype fp64 --steps 2 --rounds 1 --grid "$G" > gpurun_out/sweep_fp64_$v.log 2>&1 || exit $?
  echo "== $v"; sed -n '/summary/,$p' gpurun_out/sweep_fp64_$v.log | head -3
done
timeout -k 10 600 python bench/virtual_scaling.py --n 1048576 --ranks 1,2,4,8 --steps 3 > gpurun_out/virtual_scaling.log 2>&1 || exit $?
cat gpurun_out/virtual_scaling.log
exit $prc
