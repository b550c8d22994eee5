set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
# after the per-link emulation option: the emulation / overlap / driver tests, smoke, bench
timeout -k 10 900 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_driver.py tests/test_rccl_gpu.py \
  -x -q -m gpu --timeout 300 --timeout-method thread > $O/r6V_tests.log 2>&1 || { tail -40 $O/r6V_tests.log; exit 1; }
tail -1 $O/r6V_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > $O/r6V_smoke.log 2>&1 || { tail -20 $O/r6V_smoke.log; exit 1; }
tail -1 $O/r6V_smoke.log
timeout -k 10 400 python bench.py > $O/r6V_bench_default.log 2>&1 || { tail -20 $O/r6V_bench_default.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"engine_clock_ghz": [0-9.]*\|"cycles_per_pair_eval": [0-9.]*\|"work_audit": "[a-z]*"' $O/r6V_bench_default.log | head -4
