#!/bin/bash
# A/B: SLP-packed vs scalar-VALU build, ipl 2/4/8, plus microbench v2 and gpu tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; prc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $prc -le 1 ] || exit $prc
timeout -k 10 120 ./gravity-simulator-using-mpi-spark-and-cuda_amd/_native/microbench > gpurun_out/microbench2.jsonl 2>&1 || exit $?
cut -c1-220 gpurun_out/microbench2.jsonl | grep -v layout
G="kernel=lds,smem;ipl=2,4,8;mode=fused,split"
timeout -k 10 600 python bench/sweep.py --n 1048576 --steps 3 --rounds 2 --grid "$G" > gpurun_out/sweep_slp.log 2>&1 || exit $?
echo "== SLP"; sed -n '/summary/,$p' gpurun_out/sweep_slp.log | head -8
GRAVSIM_NATIVE_DIR=$PWD/gravity-simulator-using-mpi-spark-and-cuda_amd/_native_noslp timeout -k 10 600 python bench/sweep.py --n 1048576 --steps 3 --rounds 2 --grid "kernel=lds;ipl=2,4,8;mode=fused,split" > gpurun_out/sweep_noslp.log 2>&1 || exit $?
echo "== no SLP"; sed -n '/summary/,$p' gpurun_out/sweep_noslp.log | head -8
exit $prc
