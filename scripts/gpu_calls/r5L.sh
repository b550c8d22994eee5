set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
for v in head tu16 tu32; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  rm -rf $O/p65_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p65_$v -o tr --output-format csv -- python bench.py --n 65536 --steps 100 --warmup 10 --exact-steps 0 --phase-steps 0 --no-replay-audit --no-energy --check-samples 0 > $O/p65_$v.log 2>&1 || exit 1
  find $O/p65_$v -name "*kernel_stats.csv" -exec cp {} $O/p65stats_${v}.csv \;
  echo "$v"; head -4 $O/p65stats_${v}.csv | awk -F'",' '{print $1" | "$2}' | cut -c1-160
  unset GRAVSIM_NATIVE_DIR
done
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 3 head lib:abv/tu16 lib:abv/tu32 -- --n 65536 --steps 300 --warmup 10 || exit 1
cp $O/ab_native.jsonl $O/r5_tail_u_ab.jsonl
