set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
for r in 1 2; do for v in head k1; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  rm -rf $O/p8_$v
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p8_$v -o tr --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 12 > $O/p8_$v.log 2>&1 || exit 1
  t=$(find $O/p8_$v -name "*kernel_trace.csv" | head -1)
  python scripts/post_force_chain.py "$t" --print-steps 1 > $O/chainT_${v}_$r.txt
  echo "$v $r $(head -1 $O/chainT_${v}_$r.txt)"
  unset GRAVSIM_NATIVE_DIR
done; done
for r in 1 2; do for v in head k1; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  timeout -k 10 300 python bench/rank_shape.py --n 1048576 --ranks 8 --rank 0,7 --comm-gbps 64 --steps 16 > $O/rs_$v.log 2>&1 || exit 1
  echo "plain $v $r $(grep -o '"rank": [0-9]*\|"ms_per_step": [0-9.]*\|"exposed_comm_ms": [0-9.]*' $O/rs_$v.log | tr '\n' ' ')"
  unset GRAVSIM_NATIVE_DIR
done; done
