set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
B="--check-samples 0 --phase-steps 0 --exact-steps 0 --no-replay-audit --no-energy"
# graphs of 32 steps against 8 at small N
: > $O/r6W_ab.jsonl
for cfg in "16384:3200:64" "65536:640:64" "262144:64:32"; do
  IFS=: read -r n st wu <<< "$cfg"
  for r in 1 2; do for gs in 32 8; do
    timeout -k 10 300 env GRAVSIM_GRAPH_STEPS=$gs python bench.py --n $n --steps $st --warmup $wu $B > $O/r6W_$gs.log 2>&1 || { tail -20 $O/r6W_$gs.log; exit 1; }
    echo "{\"n\": $n, \"graph_steps\": $gs, \"round\": $r, $(grep -o '"ms_per_step": [0-9.]*' $O/r6W_$gs.log), $(grep -o '"engine_clock_ghz": [0-9.a-z]*' $O/r6W_$gs.log | head -1), $(grep -o '"cycles_per_pair_eval": [0-9.a-z]*' $O/r6W_$gs.log | head -1)}" | tee -a $O/r6W_ab.jsonl
  done; done
done
