set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
# the per-link exchange price test
timeout -k 10 400 python -u -m pytest tests/test_gpu_overlap.py -x -v -m gpu -k "per_link or phase_split" --timeout 300 \
  --timeout-method thread > $O/r6AE_tests.log 2>&1 || { tail -40 $O/r6AE_tests.log; exit 1; }
tail -4 $O/r6AE_tests.log
