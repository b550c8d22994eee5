set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
B="--check-samples 0 --phase-steps 0 --exact-steps 0 --no-replay-audit --no-energy"
# paired units: bitwise + audit first (bounded: a barrier mismatch would hang the kernel)
timeout -k 10 240 python -u -m pytest tests/test_gpu_sym.py -x -v -m gpu -k "paired" \
  --timeout 120 --timeout-method thread > $O/r6J_tests.log 2>&1 || { tail -40 $O/r6J_tests.log; exit 1; }
tail -1 $O/r6J_tests.log
: > $O/r6J_pair_ab.jsonl
for cfg in "65536:300:20" "131072:80:8" "262144:30:4" "1048576:6:2"; do
  IFS=: read -r n st wu <<< "$cfg"
  for r in 1 2; do for arm in pair0 pair1; do
    timeout -k 10 300 env GRAVSIM_SYM_PAIR=${arm#pair} python bench.py --n $n --steps $st --warmup $wu $B > $O/r6J_$arm.log 2>&1 || { tail -20 $O/r6J_$arm.log; exit 1; }
    echo "{\"n\": $n, \"arm\": \"$arm\", \"round\": $r, $(grep -o '"ms_per_step": [0-9.]*' $O/r6J_$arm.log), $(grep -o '"engine_clock_ghz": [0-9.a-z]*' $O/r6J_$arm.log | head -1), $(grep -o '"work_audit": "[a-z]*"' $O/r6J_$arm.log | head -1)}" | tee -a $O/r6J_pair_ab.jsonl
  done; done
done
