#!/bin/bash
# A/B of sym kernel variants at 1M fp32 (each variant is a separately built libgravsim_hip.so).
# Usage: [BENCH_ARGS="..."] bash scripts/gpu_sym_ab.sh dir:name [dir:name ...]
#        (dir "_native" = in-tree default; BENCH_ARGS default "--steps 5 --warmup 1")
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/sym_ab.jsonl
for v in "$@"; do
  dir=${v%%:*}; name=${v##*:}
  [ "$dir" = "_native" ] && dir=gravity-simulator-using-mpi-spark-and-cuda_amd/_native
  GRAVSIM_NATIVE_DIR=$PWD/$dir timeout -k 10 300 python bench.py --mode sym ${BENCH_ARGS:---steps 5 --warmup 1} > gpurun_out/ab_$name.log 2>&1 || { tail -20 gpurun_out/ab_$name.log; exit 1; }
  echo "{\"variant\": \"$name\", \"bench\": $(tail -1 gpurun_out/ab_$name.log)}" >> $out
  tail -1 gpurun_out/ab_$name.log | python -c "import json,sys; d=json.load(sys.stdin); print('$name', d['ms_per_step'], d['value'])"
done
