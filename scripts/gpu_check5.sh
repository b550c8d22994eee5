#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench/rank_shape.py --n 1048576 --ranks 1,2,4,8 > gpurun_out/rank_shape.log 2>&1 || exit $?
cut -c1-230 gpurun_out/rank_shape.log
timeout -k 10 600 python bench/rank_shape.py --n 1048576 --ranks 8 --ipl 8 > gpurun_out/rank_shape_ipl8.log 2>&1 || exit $?
timeout -k 10 600 python bench/rank_shape.py --n 1048576 --ranks 8 --ipl 2 > gpurun_out/rank_shape_ipl2.log 2>&1 || exit $?
cut -c1-200 gpurun_out/rank_shape_ipl8.log gpurun_out/rank_shape_ipl2.log
G="kernel=lds,smem;ipl=4,8;mode=split"
for v in _native _native_tile8k _native _native_tile8k; do
  GRAVSIM_NATIVE_DIR=$PWD/gravity-simulator-using-mpi-spark-and-cuda_amd/$v timeout -k 10 300 python bench/sweep.py --n 1048576 --steps 2 --rounds 1 --grid "$G" > gpurun_out/sweep_tile_$v.log 2>&1 || exit $?
  echo "== $v"; sed -n '/summary/,$p' gpurun_out/sweep_tile_$v.log | head -3
done
