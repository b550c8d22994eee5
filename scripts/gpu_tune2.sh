#!/bin/bash
# Retune after the explicit-pk kernel: 1M sweep, 64K sweep, per-rank shapes for P=2/4/8 by ipl
# and kernel, fp64 512K sweep. All in-process interleaved sweeps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench/sweep.py --n 1048576 --steps 3 --rounds 2 --grid "kernel=lds,smem;ipl=2,4,8;mode=split" > gpurun_out/t2_sweep_1m.log 2>&1 || exit $?
sed -n '/summary/,$p' gpurun_out/t2_sweep_1m.log
timeout -k 10 300 python bench/sweep.py --n 65536 --steps 20 --rounds 3 --grid "kernel=lds,smem;ipl=1,2,4,8;mode=split,fused" > gpurun_out/t2_sweep_64k.log 2>&1 || exit $?
sed -n '/summary/,$p' gpurun_out/t2_sweep_64k.log
timeout -k 10 600 python bench/rank_shape.py --n 1048576 --ranks 8,4,2 --ipl 2,4,8 --kernel lds,smem --steps 5 > gpurun_out/t2_rank_shape.jsonl 2>&1 || exit $?
cut -c1-200 gpurun_out/t2_rank_shape.jsonl
timeout -k 10 600 python bench/sweep.py --n 524288 --dtype fp64 --steps 2 --rounds 2 --grid "kernel=lds,smem;ipl=1,2,4;mode=split" > gpurun_out/t2_sweep_512k_fp64.log 2>&1 || exit $?
sed -n '/summary/,$p' gpurun_out/t2_sweep_512k_fp64.log
