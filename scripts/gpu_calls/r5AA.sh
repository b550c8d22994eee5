set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 3 head lib:abv/s15 lib:abv/s20 -- --n 65536 --steps 300 --warmup 10 || exit 1
bash scripts/ab_native.sh 2 head lib:abv/s15 lib:abv/s20 -- --n 262144 --steps 40 --warmup 4 || exit 1
cp $O/ab_native.jsonl $O/r5_slack_ab.jsonl
for r in 1 2; do for v in head s15 s20; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  timeout -k 10 300 python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 12 > $O/rsa_$v.log 2>&1 || exit 1
  echo "P8 $v $r $(grep -o '"ms_per_step": [0-9.]*' $O/rsa_$v.log | tail -1)"
  unset GRAVSIM_NATIVE_DIR
done; done
