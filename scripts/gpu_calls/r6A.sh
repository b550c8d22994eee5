set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
# 1. the round's new failure-path / topology tests + smoke
timeout -k 10 900 python -u -m pytest tests/test_gpu_overlap.py tests/test_guard_gpu.py \
  tests/test_rccl_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "give_up or beats or stalled or dead_peer or distinct or graph_comm_distinct or guard or match_single_rank and (8-allgather-sym-fp32-40000 or 3-allgather-sym-fp32-40000)" \
  > $O/r6A_tests.log 2>&1 || { tail -40 $O/r6A_tests.log; exit 1; }
tail -3 $O/r6A_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > $O/r6A_smoke.log 2>&1 || { tail -20 $O/r6A_smoke.log; exit 1; }
# 2. the headline bench with the clock fields
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/r6A_bench.log 2>&1 || { tail -20 $O/r6A_bench.log; exit 1; }
grep '^{' $O/r6A_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('ms_per_step','engine_clock_ghz','cycles_per_pair_eval')}, d['config']['clock'], d['config']['kernel'])"
# 3. clock stamps vs round-5 build, alternating (1M and 65K)
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 3 head lib:abv/r5head -- --steps 8 --warmup 2 || exit 1
mv $O/ab_native.jsonl $O/r6A_ab_1m.jsonl
bash scripts/ab_native.sh 3 head lib:abv/r5head -- --n 65536 --steps 300 --warmup 20 || exit 1
mv $O/ab_native.jsonl $O/r6A_ab_65k.jsonl
# 4. in-kernel clock against the PMC clock (GRBM_GUI_ACTIVE / 8 / dispatch time), same run
rm -rf $O/pmc_clock
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES -d $O/pmc_clock -o pmc --output-format csv \
  -- python bench.py --steps 2 --warmup 1 --check-samples 0 --phase-steps 0 --exact-steps 0 \
  --no-replay-audit --no-energy > $O/r6A_pmc_clock.log 2>&1 || { tail -20 $O/r6A_pmc_clock.log; exit 1; }
grep -o '"engine_clock_ghz": [0-9.]*' $O/r6A_pmc_clock.log
# 5. RANK_HOSTS rehearsal: the new topology / p-audit fields (2 ranks on this one GPU)
timeout -k 10 300 env GRAVSIM_RCCL_RANK_HOSTS=1 python bench.py --gpus 2 --steps 3 --warmup 1 --n 65536 > $O/r6A_rehearsal2.log 2>&1 || { tail -30 $O/r6A_rehearsal2.log; exit 1; }
grep '^{' $O/r6A_rehearsal2.log | cut -c1-400
