#!/bin/bash
# First-contact GPU check: tests, smoke, bench variants, rocprofv3 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== rocminfo"; (rocm-smi --showproductname 2>&1 | head -20) > gpurun_out/device.txt
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/smoke.log
for args in "--kernel lds" "--kernel smem" "--kernel lds --ipl 1" "--kernel lds --ipl 4" "--n 65536" "--n 65536 --kernel smem"; do
  echo "== bench $args"
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 $args > gpurun_out/bench_tmp.log 2>&1 || { cat gpurun_out/bench_tmp.log; exit 1; }
  tail -1 gpurun_out/bench_tmp.log | tee -a gpurun_out/bench_variants.jsonl
done
exit $rc
