set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
bash scripts/gpu.sh 'tests:overlap+or+rccl+or+guard' || exit 1
C=1048576:fp32:auto:1,1048576:fp32:auto:8,1048576:fp32:auto:7
timeout -k 10 400 python -u scripts/state_hash.py --steps 2 --cases $C > $O/hash2_h.jsonl 2>&1 || exit 1
grep -h sha $O/hash2_h.jsonl
for r in 1 2; do
  rm -rf $O/p8h
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p8h -o tr --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 8 > $O/p8h.log 2>&1 || exit 1
  t=$(find $O/p8h -name "*kernel_trace.csv" | head -1)
  python scripts/post_force_chain.py "$t" --print-steps 1 > $O/chain_h_$r.txt
  head -2 $O/chain_h_$r.txt | cut -c1-1500
done
