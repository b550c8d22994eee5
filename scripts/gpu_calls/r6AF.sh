set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
# final tree (end of round 6): whole GPU suite, smoke, default bench
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  --durations=20 > $O/r6AF_pytest_gpu_full.log 2>&1 || { tail -40 $O/r6AF_pytest_gpu_full.log; exit 1; }
tail -3 $O/r6AF_pytest_gpu_full.log
timeout -k 10 300 python __graft_entry__.py smoke > $O/r6AF_smoke.log 2>&1 || { tail -20 $O/r6AF_smoke.log; exit 1; }
tail -1 $O/r6AF_smoke.log
timeout -k 10 400 python bench.py > $O/r6AF_bench_default.log 2>&1 || { tail -20 $O/r6AF_bench_default.log; exit 1; }
grep '^{' $O/r6AF_bench_default.log | cut -c1-400
