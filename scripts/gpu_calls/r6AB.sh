set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
B="--check-samples 0 --phase-steps 0 --exact-steps 0 --no-replay-audit --no-energy"
# the 65K config on this box with the final tree (three runs), and the 1M default bench
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --n 65536 --steps 640 --warmup 64 $B > $O/r6AB_65k.log 2>&1 || { tail -20 $O/r6AB_65k.log; exit 1; }
  echo "{\"n\": 65536, \"round\": $r, $(grep -o '"ms_per_step": [0-9.]*' $O/r6AB_65k.log), $(grep -o '"engine_clock_ghz": [0-9.a-z]*' $O/r6AB_65k.log | head -1), $(grep -o '"cycles_per_pair_eval": [0-9.a-z]*' $O/r6AB_65k.log | head -1)}" | tee -a $O/r6AB_65k.jsonl
done
