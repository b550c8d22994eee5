set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 3 head lib:abv/nt -- --steps 10 --warmup 2 || exit 1
cp $O/ab_native.jsonl $O/r5_nt_ab_1m.jsonl
for v in head nt; do
  rm -rf $O/tr_$v
  if [ $v = nt ]; then export GRAVSIM_NATIVE_DIR=abv/nt; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$v -o tr --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 8 > $O/tr_$v.log 2>&1 || exit 1
  t=$(find $O/tr_$v -name "*kernel_trace.csv" | head -1)
  python scripts/post_force_chain.py "$t" --print-steps 1 > $O/chain_$v.txt
  head -1 $O/chain_$v.txt
  find $O/tr_$v -name "*kernel_stats.csv" -exec cp {} $O/stats_$v.csv \;
  grep -h "reduce" $O/stats_$v.csv | cut -d, -f1-4
  unset GRAVSIM_NATIVE_DIR
done
