set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
bash scripts/gpu.sh 'tests:overlap+or+rccl+or+scale+or+guard' || exit 1
C=1048576:fp32:auto:1,1048576:fp32:auto:8,1048576:fp32:auto:7
timeout -k 10 400 python -u scripts/state_hash.py --steps 2 --cases $C > $O/hash2_c.jsonl 2>&1 || exit 1
grep -h sha $O/hash2_c.jsonl
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 3 head lib:abv/r4 -- --steps 10 --warmup 2 || exit 1
bash scripts/ab_native.sh 3 head lib:abv/r4 -- --n 65536 --steps 300 --warmup 10 || exit 1
cp $O/ab_native.jsonl $O/r5_ab_vs_r4.jsonl
rm -rf $O/trace6
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace6 -o tr --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 6 > $O/trace6.log 2>&1 || exit 1
t=$(find $O/trace6 -name "*kernel_trace.csv" | head -1)
python scripts/post_force_chain.py "$t" --print-steps 2 > $O/r5_chain_final.txt
head -1 $O/r5_chain_final.txt
timeout -k 10 300 python bench/unit_timeline.py --n 65536 --ranks 1 --out $O/ut65k_r5b.npz > $O/ut65k_r5b.txt 2>&1 && tail -1 $O/ut65k_r5b.txt | cut -c1-300
timeout -k 10 900 python bench/rank_shape.py --n 1048576 --ranks 1,8,2,4 --rank all --comm-gbps 64 --steps 16 > $O/r5_predicted_scaling_b.jsonl 2>&1 || exit 1
timeout -k 120 300 python scripts/graph_event_probe_torch.py 2 2000 > $O/gev_torch2.txt 2>&1; echo "torch rc=$?" >> $O/gev_torch2.txt
head -3 $O/gev_torch2.txt
