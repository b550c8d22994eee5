set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
B="--check-samples 0 --phase-steps 0 --exact-steps 0 --no-replay-audit --no-energy"
# 1. small-N segments twice as long (abv/l2small: L 4 / 8 / 16 at 65K / 128K / 256K) vs head
: > $O/r6F_l2small_ab.jsonl
for cfg in "65536:300:20" "131072:80:8" "262144:30:4"; do
  IFS=: read -r n st wu <<< "$cfg"
  for r in 1 2; do for arm in head l2small; do
    if [ $arm = head ]; then env_=(env); else env_=(env GRAVSIM_NATIVE_DIR=abv/$arm); fi
    timeout -k 10 300 "${env_[@]}" python bench.py --n $n --steps $st --warmup $wu $B > $O/r6F_$arm.log 2>&1 || { tail -20 $O/r6F_$arm.log; exit 1; }
    echo "{\"n\": $n, \"arm\": \"$arm\", \"round\": $r, $(grep -o '"ms_per_step": [0-9.]*' $O/r6F_$arm.log), $(grep -o '"engine_clock_ghz": [0-9.]*' $O/r6F_$arm.log | head -1)}" | tee -a $O/r6F_l2small_ab.jsonl
  done; done
done
# 2. every BASELINE config on this box
timeout -k 10 900 python bench/configs.py --md $O/r6_baseline_configs.md > $O/r6F_configs.log 2>&1 || { tail -30 $O/r6F_configs.log; exit 1; }
cat $O/r6_baseline_configs.md
