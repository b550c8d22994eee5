set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
B="--check-samples 0 --phase-steps 0 --exact-steps 0 --no-replay-audit --no-energy"
timeout -k 10 600 python -u -m pytest tests/test_gpu_sym.py -x -q -m gpu -k "fused_tail or oracle" \
  --timeout 300 --timeout-method thread > $O/r6D_tests.log 2>&1 || { tail -40 $O/r6D_tests.log; exit 1; }
tail -2 $O/r6D_tests.log
: > $O/r6D_tail_ab.jsonl
for cfg in "65536:300:20" "131072:80:8" "262144:30:4"; do
  IFS=: read -r n st wu <<< "$cfg"
  for r in 1 2; do for arm in split1 split0 r5head; do
    case $arm in
      split1) env_=(env GRAVSIM_TAIL_SPLIT=1) ;;
      split0) env_=(env GRAVSIM_TAIL_SPLIT=0) ;;
      r5head) env_=(env GRAVSIM_NATIVE_DIR=abv/r5head) ;;
    esac
    timeout -k 10 300 "${env_[@]}" python bench.py --n $n --steps $st --warmup $wu $B > $O/r6D_$arm.log 2>&1 || { tail -20 $O/r6D_$arm.log; exit 1; }
    echo "{\"n\": $n, \"arm\": \"$arm\", \"round\": $r, $(grep -o '"ms_per_step": [0-9.]*' $O/r6D_$arm.log), $(grep -o '"engine_clock_ghz": [0-9.]*' $O/r6D_$arm.log | head -1 || echo '"engine_clock_ghz": null')}" | tee -a $O/r6D_tail_ab.jsonl
  done; done
done
