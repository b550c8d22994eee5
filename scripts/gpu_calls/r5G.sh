set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
for r in 1 2; do
for v in head nt3; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  rm -rf $O/p1_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p1_$v -o tr --output-format csv -- python bench.py --steps 6 --warmup 2 --exact-steps 0 --phase-steps 0 --no-replay-audit --no-energy --check-samples 0 > $O/p1_$v.log 2>&1 || exit 1
  find $O/p1_$v -name "*kernel_stats.csv" -exec cp {} $O/p1stats3_${v}_$r.csv \;
  echo "$v $r"; grep -h "reduce\|finalize" $O/p1stats3_${v}_$r.csv | cut -d, -f1-4
  unset GRAVSIM_NATIVE_DIR
done
done
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 3 head lib:abv/nt3 -- --steps 10 --warmup 2 || exit 1
bash scripts/ab_native.sh 3 head lib:abv/nt3 -- --n 65536 --steps 300 --warmup 10 || exit 1
cp $O/ab_native.jsonl $O/r5_nt3_ab.jsonl
