set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
# 1. the sym invariants on the two-half Ti order (fused tail vs three kernels, P shards, graph,
#    bands, oracle accuracy)
timeout -k 10 900 python -u -m pytest tests/test_gpu_sym.py tests/test_gpu_kernels.py \
  tests/test_gpu_audit.py tests/test_gpu_scale.py -x -q -m gpu --timeout 300 \
  --timeout-method thread > $O/r6C_tests.log 2>&1 || { tail -40 $O/r6C_tests.log; exit 1; }
tail -2 $O/r6C_tests.log
# 2. the two-half row reduce / fused tail against the round-5 build, alternating
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 3 head lib:abv/r5head -- --n 65536 --steps 300 --warmup 20 || exit 1
mv $O/ab_native.jsonl $O/r6C_ab_65k.jsonl
bash scripts/ab_native.sh 2 head lib:abv/r5head -- --n 262144 --steps 30 --warmup 4 || exit 1
mv $O/ab_native.jsonl $O/r6C_ab_256k.jsonl
bash scripts/ab_native.sh 2 head lib:abv/r5head lib:abv/l2x -- --steps 8 --warmup 2 || exit 1
mv $O/ab_native.jsonl $O/r6C_ab_1m.jsonl
# 3. rank 7 of 8 (1M, modeled comm 64 GB/s): head, round 5, segments of 2 chunks (l2x)
: > $O/r6C_rank8.jsonl
for r in 1 2; do for arm in head r5head l2x; do
  if [ $arm = head ]; then unset GRAVSIM_NATIVE_DIR; else export GRAVSIM_NATIVE_DIR=abv/$arm; fi
  timeout -k 10 300 python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 12 > $O/r6C_rs_$arm.log 2>&1 || exit 1
  echo "{\"arm\": \"$arm\", \"round\": $r, $(grep -o '"ms_per_step": [0-9.]*' $O/r6C_rs_$arm.log | tail -1)}" | tee -a $O/r6C_rank8.jsonl
done; done
unset GRAVSIM_NATIVE_DIR
# 4. 65K unit timeline + tail kernel time with the new tail
rm -rf $O/prof6c_65k
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof6c_65k -o b --output-format csv -- python bench.py --n 65536 --steps 200 --warmup 20 --check-samples 0 --phase-steps 0 --exact-steps 0 --no-replay-audit --no-energy > $O/prof6c_65k.log 2>&1 || exit 1
head -4 $O/prof6c_65k/b_kernel_stats.csv
