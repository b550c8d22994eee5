set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
for r in 1 2; do
for v in head c1 c1u16; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  rm -rf $O/p1_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p1_$v -o tr --output-format csv -- python bench.py --steps 4 --warmup 2 --exact-steps 0 --phase-steps 0 --no-replay-audit --no-energy --check-samples 0 > $O/p1_$v.log 2>&1 || exit 1
  find $O/p1_$v -name "*kernel_stats.csv" -exec cp {} $O/p1statsI_${v}_$r.csv \;
  echo "$v $r P1"; grep -h "node_reduce\|row_reduce" $O/p1statsI_${v}_$r.csv | cut -d, -f1-4
  rm -rf $O/p8_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p8_$v -o tr --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 8 > $O/p8_$v.log 2>&1 || exit 1
  t=$(find $O/p8_$v -name "*kernel_trace.csv" | head -1)
  python scripts/post_force_chain.py "$t" --print-steps 1 > $O/chainI_${v}_$r.txt
  echo "$v $r P8"; head -1 $O/chainI_${v}_$r.txt
  find $O/p8_$v -name "*kernel_stats.csv" -exec cp {} $O/p8statsI_${v}_$r.csv \;
  grep -h "node_reduce\|row_reduce" $O/p8statsI_${v}_$r.csv | cut -d, -f1-4
  unset GRAVSIM_NATIVE_DIR
done
done
