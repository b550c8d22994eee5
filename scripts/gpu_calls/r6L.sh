set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
# carriers rotated by ds_bpermute (LDS pipe) at the step top, the j-side FMA chain starting
# from them (GS_SYM_CARRY_BPERM): tests on this tree, then alternating A/B against the build
# before the change (abv/base) and the variant without the step-top scheduling barrier (abv/bp1)
B="--check-samples 0 --phase-steps 0 --exact-steps 0 --no-replay-audit --no-energy"
timeout -k 10 900 python -u -m pytest tests/test_gpu_sym.py tests/test_gpu_kernels.py tests/test_gpu_audit.py \
  -x -q -m gpu --timeout 300 --timeout-method thread > $O/r6L_tests.log 2>&1 || { tail -40 $O/r6L_tests.log; exit 1; }
tail -1 $O/r6L_tests.log
: > $O/r6L_ab.jsonl
for cfg in "1048576:6:2:fp32" "65536:300:20:fp32" "524288:6:2:fp64"; do
  IFS=: read -r n st wu dt <<< "$cfg"
  for r in 1 2; do for arm in head base bp1; do
    if [ $arm = head ]; then env_=(env); else env_=(env GRAVSIM_NATIVE_DIR=abv/$arm); fi
    timeout -k 10 300 "${env_[@]}" python bench.py --n $n --steps $st --warmup $wu --dtype $dt $B > $O/r6L_$arm.log 2>&1 || { tail -20 $O/r6L_$arm.log; exit 1; }
    echo "{\"n\": $n, \"dtype\": \"$dt\", \"arm\": \"$arm\", \"round\": $r, $(grep -o '"ms_per_step": [0-9.]*' $O/r6L_$arm.log), $(grep -o '"engine_clock_ghz": [0-9.a-z]*' $O/r6L_$arm.log | head -1), $(grep -o '"cycles_per_pair_eval": [0-9.a-z]*' $O/r6L_$arm.log | head -1)}" | tee -a $O/r6L_ab.jsonl
  done; done
done
