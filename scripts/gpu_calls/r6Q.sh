set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
B="--check-samples 0 --phase-steps 0 --exact-steps 0 --no-replay-audit --no-energy"
# one-rank graphs of 8 steps per launch (GRAVSIM_GRAPH_STEPS, default up to 2M bodies)
timeout -k 10 900 python -u -m pytest tests/test_gpu_sym.py tests/test_gpu_kernels.py tests/test_gpu_audit.py \
  tests/test_gpu_overlap.py tests/test_gpu_driver.py -x -q -m gpu --timeout 300 --timeout-method thread \
  > $O/r6Q_tests.log 2>&1 || { tail -40 $O/r6Q_tests.log; exit 1; }
tail -1 $O/r6Q_tests.log
: > $O/r6Q_ab.jsonl
for cfg in "16384:2000:40" "65536:400:24" "131072:120:8" "1048576:10:2"; do
  IFS=: read -r n st wu <<< "$cfg"
  for r in 1 2; do for gs in 8 2; do
    timeout -k 10 300 env GRAVSIM_GRAPH_STEPS=$gs python bench.py --n $n --steps $st --warmup $wu $B > $O/r6Q_$gs.log 2>&1 || { tail -20 $O/r6Q_$gs.log; exit 1; }
    echo "{\"n\": $n, \"graph_steps\": $gs, \"round\": $r, $(grep -o '"ms_per_step": [0-9.]*' $O/r6Q_$gs.log), $(grep -o '"engine_clock_ghz": [0-9.a-z]*' $O/r6Q_$gs.log | head -1), $(grep -o '"cycles_per_pair_eval": [0-9.a-z]*' $O/r6Q_$gs.log | head -1)}" | tee -a $O/r6Q_ab.jsonl
  done; done
done
rm -rf $O/kt65q
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt65q -o kt --output-format csv -- python bench.py --n 65536 --steps 64 --warmup 8 $B > $O/r6Q_kt65.log 2>&1 || { tail -20 $O/r6Q_kt65.log; exit 1; }
python scripts/kernel_gaps.py "$(find $O/kt65q -name '*kernel_trace.csv' | head -1)" | tee $O/r6Q_gaps65.txt
