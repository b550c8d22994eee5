set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
bash scripts/gpu.sh tests:rccl+or+guard+or+overlap+or+unit_timeline || exit 1
rm -f $O/r5_sync_ab.jsonl
for i in 1 2; do
  for sync in flags events; do
    timeout -k 10 300 env GRAVSIM_SYNC=$sync python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 8 > $O/rs_$sync.log 2>&1 || exit 1
    grep '^{' $O/rs_$sync.log | sed "s/^{/{\"sync\": \"$sync\", /" >> $O/r5_sync_ab.jsonl
  done
done
rm -rf $O/trace5
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace5 -o tr --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 6 > $O/trace5.log 2>&1 || exit 1
t=$(find $O/trace5 -name "*kernel_trace.csv" | head -1)
python scripts/post_force_chain.py "$t" --print-steps 2 > $O/r5_chain_flags.txt
cat $O/r5_chain_flags.txt | cut -c1-400
timeout -k 10 300 python bench/unit_timeline.py --n 65536 --ranks 1 --out $O/ut65k_r5.npz > $O/ut65k_r5.txt 2>&1 && cat $O/ut65k_r5.txt | tail -1 | cut -c1-300
