set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
bash scripts/gpu.sh 'tests:persistent+or+gated+or+segmented' || exit 1
for r in 1 2 3; do for v in head prev3; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  timeout -k 10 300 python bench/rank_shape.py --n 1048576 --ranks 2 --rank 1 --comm-gbps 64 --steps 8 > $O/rsw_$v.log 2>&1 || exit 1
  echo "P2 $v $r $(grep -o '"ms_per_step": [0-9.]*' $O/rsw_$v.log | tail -1)"
  unset GRAVSIM_NATIVE_DIR
done; done
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 2 head lib:abv/prev3 -- --n 65536 --steps 300 --warmup 10 || exit 1
bash scripts/ab_native.sh 2 head lib:abv/prev3 -- --steps 6 --warmup 2 || exit 1
cp $O/ab_native.jsonl $O/r5_persist2_ab.jsonl
