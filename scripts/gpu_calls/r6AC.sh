set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
# after check_topology(): the audit / RCCL tests and a two-rank rehearsal bench (topology recorded)
timeout -k 10 700 python -u -m pytest tests/test_gpu_audit.py tests/test_rccl_gpu.py tests/test_guard_gpu.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/r6AC_tests.log 2>&1 || { tail -40 $O/r6AC_tests.log; exit 1; }
tail -1 $O/r6AC_tests.log
GRAVSIM_RCCL_RANK_HOSTS=1 timeout -k 10 400 python bench.py --gpus 2 --n 65536 --steps 3 --warmup 1 > $O/r6AC_bench2.log 2>&1 || { tail -20 $O/r6AC_bench2.log; exit 1; }
grep '^{' $O/r6AC_bench2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['status'], d['work_audit'], d['audit']['p_independence'], d['config']['topology']['enforced'], d['config']['topology']['problems'][:1])"
