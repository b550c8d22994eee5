set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
B="--check-samples 0 --phase-steps 0 --exact-steps 0 --no-replay-audit --no-energy"
# 1. clock stamps vs the round-5 build, alternating (1M and 65K)
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 3 head lib:abv/r5head -- --steps 8 --warmup 2 || exit 1
mv $O/ab_native.jsonl $O/r6B_ab_1m.jsonl
bash scripts/ab_native.sh 3 head lib:abv/r5head -- --n 65536 --steps 300 --warmup 20 || exit 1
mv $O/ab_native.jsonl $O/r6B_ab_65k.jsonl
# 2. in-kernel clock against the PMC clock (GRBM_GUI_ACTIVE / 8 / dispatch time), same run
rm -rf $O/pmc_clock
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES -d $O/pmc_clock -o pmc --output-format csv \
  -- python bench.py --steps 2 --warmup 1 $B > $O/r6B_pmc_clock.log 2>&1 || { tail -20 $O/r6B_pmc_clock.log; exit 1; }
grep -o '"engine_clock_ghz": [0-9.]*' $O/r6B_pmc_clock.log
# 3. PMC of the shipped force kernel, 1M and 65K (one pass per counter group, kernel trace only)
for cfg in "1m:--steps 2 --warmup 1" "65k:--n 65536 --steps 40 --warmup 4"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  for pass in "valu SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
              "cycles SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS" \
              "lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32"; do
    set -- $pass; p=$1; shift
    rm -rf $O/pmc6_${tag}_$p
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" -d $O/pmc6_${tag}_$p -o pmc \
      --output-format csv -- python bench.py $args $B > $O/pmc6_${tag}_$p.log 2>&1 \
      || { tail -20 $O/pmc6_${tag}_$p.log; exit 1; }
  done
  python scripts/pmc_summary.py "$O/pmc6_${tag}_*/**/*counter_collection.csv" > $O/r6B_pmc_${tag}_summary.txt 2>&1
  cat $O/r6B_pmc_${tag}_summary.txt
done
# 4. raw TCC read requests of the reduce kernels (what FETCH_SIZE is derived from), 1M one GPU
rm -rf $O/pmc6_tcc
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCC_BUBBLE_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum \
  TCC_EA0_RDREQ_DRAM_sum -d $O/pmc6_tcc -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 $B \
  > $O/pmc6_tcc.log 2>&1 || { tail -20 $O/pmc6_tcc.log; exit 1; }
rm -rf $O/pmc6_fetch
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc6_fetch -o pmc --output-format csv \
  -- python bench.py --steps 2 --warmup 1 $B > $O/pmc6_fetch.log 2>&1 || { tail -20 $O/pmc6_fetch.log; exit 1; }
# 5. kernel-trace stats of the 1M and 65K bench (no counters)
rm -rf $O/prof6_1m $O/prof6_65k
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof6_1m -o b --output-format csv -- python bench.py --steps 6 --warmup 2 $B > $O/prof6_1m.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof6_65k -o b --output-format csv -- python bench.py --n 65536 --steps 200 --warmup 20 $B > $O/prof6_65k.log 2>&1 || exit 1
find $O/prof6_1m $O/prof6_65k -name "*kernel_stats.csv" | xargs -I{} sh -c 'echo {}; head -6 {}'
# 6. RANK_HOSTS rehearsal: the new topology / p-audit fields (2 ranks on this one GPU)
timeout -k 10 300 env GRAVSIM_RCCL_RANK_HOSTS=1 python bench.py --gpus 2 --steps 3 --warmup 1 --n 65536 > $O/r6B_rehearsal2.log 2>&1 || { tail -30 $O/r6B_rehearsal2.log; exit 1; }
grep '^{' $O/r6B_rehearsal2.log | cut -c1-300
