set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
# graph_steps_per_launch in the bench JSON: the driver tests and the default bench
timeout -k 10 600 python -u -m pytest tests/test_gpu_driver.py tests/test_gpu_sym.py -x -q -m gpu --timeout 300 \
  --timeout-method thread > $O/r6AA_tests.log 2>&1 || { tail -40 $O/r6AA_tests.log; exit 1; }
tail -1 $O/r6AA_tests.log
timeout -k 10 400 python bench.py > $O/r6AA_bench_default.log 2>&1 || { tail -20 $O/r6AA_bench_default.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"engine_clock_ghz": [0-9.]*\|"graph": "[a-z]*"\|"graph_steps_per_launch": [0-9]*\|"work_audit": "[a-z]*"' $O/r6AA_bench_default.log | head -6
