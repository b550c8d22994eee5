set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
B="--check-samples 0 --phase-steps 0 --exact-steps 0 --no-replay-audit --no-energy"
timeout -k 10 600 python -u -m pytest tests/test_gpu_sym.py tests/test_gpu_audit.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/r6I_tests.log 2>&1 || { tail -40 $O/r6I_tests.log; exit 1; }
tail -1 $O/r6I_tests.log
: > $O/r6I_ab.jsonl
for cfg in "65536:300:20" "131072:80:8" "262144:30:4" "1048576:6:2"; do
  IFS=: read -r n st wu <<< "$cfg"
  for r in 1 2; do for arm in head r5head; do
    if [ $arm = head ]; then env_=(env); else env_=(env GRAVSIM_NATIVE_DIR=abv/$arm); fi
    timeout -k 10 300 "${env_[@]}" python bench.py --n $n --steps $st --warmup $wu $B > $O/r6I_$arm.log 2>&1 || { tail -20 $O/r6I_$arm.log; exit 1; }
    echo "{\"n\": $n, \"arm\": \"$arm\", \"round\": $r, $(grep -o '"ms_per_step": [0-9.]*' $O/r6I_$arm.log), $(grep -o '"engine_clock_ghz": [0-9.a-z]*' $O/r6I_$arm.log | head -1)}" | tee -a $O/r6I_ab.jsonl
  done; done
done
