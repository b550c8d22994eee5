set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 3 head lib:abv/prev2 -- --steps 10 --warmup 2 || exit 1
bash scripts/ab_native.sh 2 head lib:abv/prev2 -- --n 262144 --steps 40 --warmup 4 || exit 1
cp $O/ab_native.jsonl $O/r5_node_row_p1_ab.jsonl
for v in head prev2; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  rm -rf $O/p1s_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p1s_$v -o tr --output-format csv -- python bench.py --steps 4 --warmup 2 --exact-steps 0 --phase-steps 0 --no-replay-audit --no-energy --check-samples 0 > $O/p1s_$v.log 2>&1 || exit 1
  echo "$v"; find $O/p1s_$v -name "*kernel_stats.csv" -exec grep -h "reduce\|node_row\|finalize" {} \; | awk -F'",' '{print $1" | "$2}' | cut -c1-150
  unset GRAVSIM_NATIVE_DIR
done
