#!/bin/bash
# auto vs explicit schedules across N, one in-process interleaved sweep per size:
#   bash scripts/size_sweep.sh <dtype> <grid> <n> [<n> ...]
# e.g. bash scripts/size_sweep.sh fp64 "mode=auto,split" 16384 50000 100000
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
dtype=$1; grid=$2; shift 2
for n in "$@"; do
  st=$((20000000000 / (n * n / 1000) + 5)); [ $st -gt 400 ] && st=400
  [ "$dtype" = fp64 ] && st=$(( (st + 3) / 4 ))
  timeout -k 10 150 python bench/sweep.py --n $n --dtype $dtype --steps $st --rounds 3 \
    --grid "$grid" > gpurun_out/size_${dtype}_$n.log 2>&1 || exit $?
  echo "n=$n $dtype"; grep -A3 summary gpurun_out/size_${dtype}_$n.log | tail -3
done
