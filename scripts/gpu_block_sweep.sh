#!/bin/bash
# Workgroup-size sweep: 128 / 256 (default) / 512 threads, SMEM kernel,
# interleaved builds in one call. Build the variants first:
#   GRAVSIM_NATIVE_DIR=.../_native_b128 GRAVSIM_HIP_EXTRA="-DGS_BLOCK=128 -DGS_TILE_BYTES=4096" python csrc/build.py --only hip
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=$PWD/gravity-simulator-using-mpi-spark-and-cuda_amd
: > gpurun_out/block_sweep.jsonl
for rep in 1 2; do
  for b in 256 128 512; do
    for args in "--kernel smem" "--kernel smem --ipl 4" "--n 262144 --kernel smem --ipl 4"; do
      if [ $b = 256 ]; then unset GRAVSIM_NATIVE_DIR; else export GRAVSIM_NATIVE_DIR=$P/_native_b$b; fi
      timeout -k 10 300 python bench.py --steps 5 --warmup 2 $args > gpurun_out/bs_tmp.log 2>&1 || { cat gpurun_out/bs_tmp.log; exit 1; }
      echo "{\"block\": $b, \"args\": \"$args\", \"line\": $(tail -1 gpurun_out/bs_tmp.log)}" >> gpurun_out/block_sweep.jsonl
    done
  done
done
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/block_sweep.jsonl"):
    r = json.loads(l)
    d[(r["args"], r["block"])].append(r["line"]["ms_per_step"])
for k in sorted(d):
    print(k, ["%.2f" % x for x in d[k]], "min %.2f" % min(d[k]))
PY
