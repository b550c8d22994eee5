set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
for P in 2 4; do for r in 1 2; do for v in head ntoff; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  rm -rf $O/tv
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tv -o tr --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks $P --rank 1 --comm-gbps 64 --steps 8 > $O/tv.log 2>&1 || exit 1
  t=$(find $O/tv -name "*kernel_trace.csv" | head -1)
  python scripts/post_force_chain.py "$t" --print-steps 1 > $O/chainV_${P}_${v}_$r.txt
  echo "P=$P $v $r $(head -1 $O/chainV_${P}_${v}_$r.txt)"
  unset GRAVSIM_NATIVE_DIR
done; done; done
