set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
rm -f $O/r5_sync_ab.jsonl $O/r5_vec_ab.jsonl $O/r5_prefetch_ab.jsonl
ab() {  # $1 tag, $2 env assignment, rest: bench args
  tag=$1; envs=$2; shift 2
  timeout -k 10 300 env $envs python bench.py --exact-steps 0 --phase-steps 0 --no-replay-audit --no-energy --check-samples 0 "$@" > $O/ab_tmp.log 2>&1 || { tail -20 $O/ab_tmp.log; exit 1; }
  echo "{\"tag\": \"$tag\", \"env\": \"$envs\", \"args\": \"$*\", \"ms\": $(grep -o '"ms_per_step": [0-9.]*' $O/ab_tmp.log | grep -o '[0-9.]*$')}"
}
for i in 1 2; do
  for sync in flags events; do
    timeout -k 10 300 env GRAVSIM_SYNC=$sync python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 8 > $O/rs_$sync.log 2>&1 || exit 1
    grep '^{' $O/rs_$sync.log | sed "s/^{/{\"sync\": \"$sync\", /" >> $O/r5_sync_ab.jsonl
  done
  for v in 1 0; do ab vec GRAVSIM_REDUCE_VEC=$v --steps 10 --warmup 2 >> $O/r5_vec_ab.jsonl || exit 1; done
  for p in 1 0; do ab pf65k GRAVSIM_SYM_PREFETCH=$p --n 65536 --steps 200 --warmup 10 >> $O/r5_prefetch_ab.jsonl || exit 1; done
  for p in 1 0; do ab pf1m GRAVSIM_SYM_PREFETCH=$p --steps 10 --warmup 2 >> $O/r5_prefetch_ab.jsonl || exit 1; done
done
cat $O/r5_vec_ab.jsonl $O/r5_prefetch_ab.jsonl
rm -rf $O/trace5
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace5 -o tr --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 6 > $O/trace5.log 2>&1 || exit 1
t=$(find $O/trace5 -name "*kernel_trace.csv" | head -1)
python scripts/post_force_chain.py "$t" --print-steps 2 > $O/r5_chain_flags.txt
head -1 $O/r5_chain_flags.txt
timeout -k 10 300 python bench/unit_timeline.py --n 65536 --ranks 1 --out $O/ut65k_r5.npz > $O/ut65k_r5.txt 2>&1 && tail -1 $O/ut65k_r5.txt | cut -c1-300
timeout -k 10 600 python bench/rank_shape.py --n 1048576 --ranks 1,2,4,8,3,5,6,7 --rank all --comm-gbps 64 --steps 6 > $O/r5_predicted_scaling.jsonl 2>&1 || exit 1
python - <<'PY'
import json
rows=[json.loads(l) for l in open("gpurun_out/r5_predicted_scaling.jsonl") if l.startswith("{")]
base=[r["ms_per_step"] for r in rows if r["P"]==1][0]
for P in sorted({r["P"] for r in rows}):
    ms=max(r["ms_per_step"] for r in rows if r["P"]==P)
    print(P, round(ms,3), round(base/(P*ms),4))
PY
C=1048576:fp32:auto:1,1048576:fp32:auto:8,1048576:fp32:auto:7
timeout -k 10 400 python -u scripts/state_hash.py --steps 2 --cases $C > $O/hash2_new.jsonl 2>&1 || exit 1
grep -h sha $O/hash2_new.jsonl
timeout -k 10 120 ./gravity-simulator-using-mpi-spark-and-cuda_amd/_native/graph_event_probe 4 5000 > $O/gev_standalone.txt 2>&1; echo "standalone rc=$?" >> $O/gev_standalone.txt
timeout -k 10 180 python scripts/graph_event_probe_torch.py 4 5000 > $O/gev_torch.txt 2>&1; echo "torch rc=$?" >> $O/gev_torch.txt
tail -4 $O/gev_standalone.txt $O/gev_torch.txt
