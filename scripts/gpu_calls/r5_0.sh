set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
bash scripts/gpu.sh tests || exit 1
C=65536:fp32:auto:1,1048576:fp32:auto:1,262144:fp32:auto:3,1048576:fp32:auto:8,524288:fp64:auto:1,1048576:fp32:auto:5
timeout -k 10 400 python -u scripts/state_hash.py --cases $C > $O/hash_vec.jsonl 2>&1 || exit 1
timeout -k 10 400 env GRAVSIM_REDUCE_VEC=0 python -u scripts/state_hash.py --cases $C > $O/hash_scalar.jsonl 2>&1 || exit 1
timeout -k 10 400 env GRAVSIM_NATIVE_DIR=abv/r4 python -u scripts/state_hash.py --cases $C > $O/hash_r4b.jsonl 2>&1 || exit 1
grep -h sha $O/hash_vec.jsonl $O/hash_scalar.jsonl $O/hash_r4b.jsonl
rm -f $O/r5_sync_ab.jsonl $O/r5_vec_ab.jsonl
for i in 1 2; do
  for sync in flags events; do
    timeout -k 10 300 env GRAVSIM_SYNC=$sync python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 8 > $O/rs_$sync.log 2>&1 || exit 1
    grep '^{' $O/rs_$sync.log | sed "s/^{/{\"sync\": \"$sync\", /" >> $O/r5_sync_ab.jsonl
  done
  for vec in 1 0; do
    timeout -k 10 300 env GRAVSIM_REDUCE_VEC=$vec python bench.py --steps 10 --warmup 2 --exact-steps 0 --phase-steps 0 --no-replay-audit --no-energy --check-samples 0 > $O/vec_$vec.log 2>&1 || exit 1
    echo "{\"vec\": $vec, \"round\": $i, \"ms\": $(grep -o '"ms_per_step": [0-9.]*' $O/vec_$vec.log | grep -o '[0-9.]*$')}" >> $O/r5_vec_ab.jsonl
  done
done
cat $O/r5_vec_ab.jsonl
rm -rf $O/trace5
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace5 -o tr --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 6 > $O/trace5.log 2>&1 || exit 1
t=$(find $O/trace5 -name "*kernel_trace.csv" | head -1)
python scripts/post_force_chain.py "$t" --print-steps 2 > $O/r5_chain_flags.txt
head -1 $O/r5_chain_flags.txt
timeout -k 10 300 python bench/unit_timeline.py --n 65536 --ranks 1 --out $O/ut65k_r5.npz > $O/ut65k_r5.txt 2>&1 && tail -1 $O/ut65k_r5.txt | cut -c1-300
timeout -k 10 120 ./gravity-simulator-using-mpi-spark-and-cuda_amd/_native/graph_event_probe 4 5000 > $O/gev_standalone.txt 2>&1; echo "standalone rc=$?" >> $O/gev_standalone.txt
timeout -k 10 180 python scripts/graph_event_probe_torch.py 4 5000 > $O/gev_torch.txt 2>&1; echo "torch rc=$?" >> $O/gev_torch.txt
tail -4 $O/gev_standalone.txt $O/gev_torch.txt
