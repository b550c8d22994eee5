#!/bin/bash
# Ring-pass strategy: bitwise tests (virtual shards + 1-rank live RCCL) and emulated per-rank
# step times for all-gather vs ring at 1M fp32.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_rccl_gpu.py -x -q -m gpu \
  -k "ring or rccl or virtual" > gpurun_out/pytest_ring.log 2>&1 || { tail -30 gpurun_out/pytest_ring.log; exit 1; }
tail -3 gpurun_out/pytest_ring.log
timeout -k 10 600 python bench/rank_shape.py --n 1048576 --ranks 1,2,4,8 --strategy allgather,ring \
  --steps 5 > gpurun_out/rank_shape_ring.jsonl 2>&1 || { tail -20 gpurun_out/rank_shape_ring.jsonl; exit 1; }
cat gpurun_out/rank_shape_ring.jsonl | cut -c1-220
