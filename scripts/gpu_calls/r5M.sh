set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 3 head lib:abv/kr8 lib:abv/kr4 -- --n 65536 --steps 300 --warmup 10 || exit 1
bash scripts/ab_native.sh 2 head lib:abv/kr8 lib:abv/kr4 -- --n 131072 --steps 100 --warmup 10 || exit 1
cp $O/ab_native.jsonl $O/r5_kr_small_n_ab.jsonl
for v in head kr8; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  timeout -k 10 300 python bench/unit_timeline.py --n 65536 --ranks 1 --out $O/ut65k_$v.npz > $O/ut65k_$v.txt 2>&1 || exit 1
  tail -1 $O/ut65k_$v.txt | cut -c1-330
  unset GRAVSIM_NATIVE_DIR
done
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 3 head lib:abv/r4loop lib:abv/r4 -- --steps 10 --warmup 2 || exit 1
bash scripts/ab_native.sh 3 head lib:abv/r4loop -- --n 65536 --steps 300 --warmup 10 || exit 1
cp $O/ab_native.jsonl $O/r5_r4loop_ab.jsonl
for r in 1 2; do for v in head r4loop; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  timeout -k 10 300 python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 12 > $O/rs_$v.log 2>&1 || exit 1
  echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/rs_$v.log | tail -1)"
  unset GRAVSIM_NATIVE_DIR
done; done
