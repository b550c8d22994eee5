#!/bin/bash
# Alternating bench.py runs of native builds (GRAVSIM_NATIVE_DIR) and of other source trees
# on one box: bash scripts/ab_native.sh <rounds> <arm>[ <arm>...] -- <bench.py args>
# arm: "tree:<dir>" runs <dir>/bench.py (another source tree with its own build), "lib:<dir>"
# runs this tree's bench.py on the native build in <dir>, "head" this tree as it is.
# Appends {"arm", "round", "ms_per_step"} lines to gpurun_out/ab_native.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rounds=$1; shift
arms=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do arms+=("$1"); shift; done
shift
for r in $(seq 1 "$rounds"); do
  for arm in "${arms[@]}"; do
    log=gpurun_out/ab_native_${r}_$(echo "$arm" | tr '/:' '__').log
    case "$arm" in
      tree:*) cmd=(python "${arm#tree:}/bench.py") ;;
      lib:*) cmd=(env GRAVSIM_NATIVE_DIR="${arm#lib:}" python bench.py) ;;
      *) cmd=(python bench.py) ;;
    esac
    timeout -k 10 300 "${cmd[@]}" --exact-steps 0 --phase-steps 0 --no-replay-audit --no-energy \
      --check-samples 0 "$@" > "$log" 2>&1 || { tail -20 "$log"; exit 1; }
    ms=$(grep -o '"ms_per_step": [0-9.]*' "$log" | grep -o '[0-9.]*$')
    echo "{\"arm\": \"$arm\", \"round\": $r, \"ms_per_step\": $ms}" | tee -a gpurun_out/ab_native.jsonl
  done
done
