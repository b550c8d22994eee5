#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in _native _native_nopf; do
  export GRAVSIM_NATIVE_DIR=$PWD/gravity-simulator-using-mpi-spark-and-cuda_amd/$v
  timeout -k 10 300 python bench/sweep.py --n 1048576 --steps 3 --rounds 2 --grid "kernel=smem,lds;ipl=4" > gpurun_out/pf_1m_$v.log 2>&1 || exit $?
  echo "== 1M $v"; sed -n '/summary/,$p' gpurun_out/pf_1m_$v.log | head -3
  timeout -k 10 300 python bench/rank_shape.py --n 16777216 --ranks 8 --ipl 4 --kernel smem,lds --steps 1 > gpurun_out/pf_16m_$v.log 2>&1 || exit $?
  echo "== 16M P=8 $v"; cut -c1-140 gpurun_out/pf_16m_$v.log | grep '^{'
done
