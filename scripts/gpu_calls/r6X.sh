set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
B="--check-samples 0 --phase-steps 0 --exact-steps 0 --no-replay-audit --no-energy"
# 32-step graphs by default up to 256K: the sym / kernel / audit tests, the 65K bench
timeout -k 10 900 python -u -m pytest tests/test_gpu_sym.py tests/test_gpu_kernels.py tests/test_gpu_audit.py \
  -x -q -m gpu --timeout 300 --timeout-method thread > $O/r6X_tests.log 2>&1 || { tail -40 $O/r6X_tests.log; exit 1; }
tail -1 $O/r6X_tests.log
timeout -k 10 300 python bench.py --n 65536 --steps 640 --warmup 64 $B > $O/r6X_65k.log 2>&1 || { tail -20 $O/r6X_65k.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"engine_clock_ghz": [0-9.]*\|"cycles_per_pair_eval": [0-9.]*\|"work_audit": "[a-z]*"' $O/r6X_65k.log | head -4
