#!/bin/bash
# A/B of native builds on one GPU box, alternating runs (compile-time variants):
#   bash scripts/ab_lib.sh <variant dir>[,<variant dir>...] <rounds> <bench.py args...>
# Arm "A" is the in-tree build (_native/); every other arm is a variant directory loaded
# through GRAVSIM_NATIVE_DIR and tagged with its path. One JSON line per run goes to
# gpurun_out/ab_lib.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
IFS=, read -r -a dirs <<< "$1"; rounds=$2; shift 2
for r in $(seq 1 "$rounds"); do
  for arm in A "${dirs[@]}"; do
    if [ "$arm" = A ]; then
      line=$(timeout -k 10 300 python bench.py "$@" | grep '^{') || exit $?
    else
      line=$(GRAVSIM_NATIVE_DIR="$arm" timeout -k 10 300 python bench.py "$@" | grep '^{') || exit $?
    fi
    ms=$(echo "$line" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"])')
    echo "{\"arm\": \"$arm\", \"round\": $r, \"args\": \"$*\", \"ms_per_step\": $ms}" | tee -a gpurun_out/ab_lib.jsonl
  done
done
