#!/bin/bash
# fp64 sym: GPU sym tests, then fp64 512K bench sym vs split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sym.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_sym.log 2>&1 || { tail -60 gpurun_out/pytest_sym.log; exit 1; }
tail -3 gpurun_out/pytest_sym.log
for m in sym split; do
  timeout -k 10 300 python bench.py --dtype fp64 --n 524288 --mode $m --steps 3 --warmup 1 > gpurun_out/bench64_$m.log 2>&1 || { tail -20 gpurun_out/bench64_$m.log; exit 1; }
  tail -1 gpurun_out/bench64_$m.log | python -c "import json,sys; d=json.load(sys.stdin); print('fp64 512K $m', d['ms_per_step'], d['value'])"
done
