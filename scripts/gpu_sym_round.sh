#!/bin/bash
# sym tests (+ RCCL 1-rank), size sweep sym vs split, default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_sym_tests.sh || exit 1
bash scripts/gpu_sym_sizes.sh || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | python -c "import json,sys; d=json.load(sys.stdin); print('default 1M', d['ms_per_step'], d['value'])"
