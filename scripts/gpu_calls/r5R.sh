set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
for r in 1 2; do for v in head prev; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  rm -rf $O/p8_$v
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p8_$v -o tr --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 12 > $O/p8_$v.log 2>&1 || exit 1
  t=$(find $O/p8_$v -name "*kernel_trace.csv" | head -1)
  python scripts/post_force_chain.py "$t" --print-steps 1 > $O/chainR_${v}_$r.txt
  echo "$v $r $(head -1 $O/chainR_${v}_$r.txt) $(grep -o '"ms_per_step": [0-9.]*' $O/p8_$v.log | tail -1)"
  unset GRAVSIM_NATIVE_DIR
done; done
for r in 1 2; do for v in head prev; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  timeout -k 10 300 python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 16 > $O/rs_$v.log 2>&1 || exit 1
  echo "plain $v $r $(grep -o '"ms_per_step": [0-9.]*' $O/rs_$v.log | tail -1)"
  unset GRAVSIM_NATIVE_DIR
done; done
bash scripts/gpu.sh 'tests:overlap+or+rccl+or+audit+or+gated+or+defer' || exit 1
C=1048576:fp32:auto:8,1048576:fp32:auto:7
timeout -k 10 400 python -u scripts/state_hash.py --steps 2 --cases $C > $O/hash2_r.jsonl 2>&1 || exit 1
grep -h sha $O/hash2_r.jsonl
