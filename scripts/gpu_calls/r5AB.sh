set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
bash scripts/gpu.sh 'tests:overlap+or+rccl+or+audit+or+gated' || exit 1
C=1048576:fp32:auto:8,1048576:fp32:auto:7,1048576:fp32:auto:3
timeout -k 10 400 python -u scripts/state_hash.py --steps 2 --cases $C > $O/hash2_ab.jsonl 2>&1 || exit 1
grep -h sha $O/hash2_ab.jsonl
for P in 8 4; do for r in 1 2; do for v in head prev5; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  rm -rf $O/tc
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tc -o tr --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks $P --rank $((P-1)) --comm-gbps 64 --steps 10 > $O/tc.log 2>&1 || exit 1
  t=$(find $O/tc -name "*kernel_trace.csv" | head -1)
  python scripts/post_force_chain.py "$t" --print-steps 1 > $O/chainAB_${P}_${v}_$r.txt
  echo "P=$P $v $r $(head -1 $O/chainAB_${P}_${v}_$r.txt)"
  unset GRAVSIM_NATIVE_DIR
done; done; done
for r in 1 2; do for v in head prev5; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  timeout -k 10 300 python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 16 > $O/rsc_$v.log 2>&1 || exit 1
  echo "plain P8 $v $r $(grep -o '"ms_per_step": [0-9.]*\|"exposed_comm_ms": [0-9.]*' $O/rsc_$v.log | tr '\n' ' ')"
  unset GRAVSIM_NATIVE_DIR
done; done
