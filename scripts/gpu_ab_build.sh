#!/bin/bash
# A/B: default build (B) vs the _native_ab build (A: built with the flag under test).
# Optional: $1 = pytest selection run first on the default build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=("--kernel smem" "--kernel smem --ipl 8" "--kernel lds --ipl 8" "--kernel lds --ipl 4")
[ -n "$AB_ARGS" ] && IFS=';' read -r -a ARGS <<< "$AB_ARGS"  # e.g. AB_ARGS="--n 65536;--ipl 2"
A=$PWD/gravity-simulator-using-mpi-spark-and-cuda_amd/_native_ab
if [ -n "$1" ]; then
  timeout -k 10 900 python -m pytest tests -x -q -m gpu -k "$1" > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 1; }
  tail -2 gpurun_out/pytest_ab.log
fi
: > gpurun_out/ab_drain.jsonl
for rep in 1 2 3; do
  for v in A B; do
    for args in "${ARGS[@]}"; do
      if [ $v = A ]; then export GRAVSIM_NATIVE_DIR=$A; else unset GRAVSIM_NATIVE_DIR; fi
      timeout -k 10 300 python bench.py --steps 5 --warmup 1 $args > gpurun_out/ab_tmp.log 2>&1 || { cat gpurun_out/ab_tmp.log; exit 1; }
      echo "{\"variant\": \"$v\", \"args\": \"$args\", \"line\": $(tail -1 gpurun_out/ab_tmp.log)}" >> gpurun_out/ab_drain.jsonl
    done
  done
done
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ab_drain.jsonl"):
    r = json.loads(l)
    d[(r["args"], r["variant"])].append(r["line"]["ms_per_step"])
for k in sorted(d):
    print(k, ["%.2f" % x for x in d[k]], "min %.2f" % min(d[k]))
PY
