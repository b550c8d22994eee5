set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 3 head lib:abv/age20 lib:abv/age40 lib:abv/age80 -- --n 65536 --steps 300 --warmup 10 || exit 1
bash scripts/ab_native.sh 2 head lib:abv/age40 -- --steps 6 --warmup 2 || exit 1
cp $O/ab_native.jsonl $O/r5_age_ab.jsonl
for v in head age20 age40 age80; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  timeout -k 10 300 python bench/unit_timeline.py --n 65536 --ranks 1 --out $O/ut65k_$v.npz > $O/ut65k_$v.txt 2>&1 || exit 1
  echo "$v $(tail -1 $O/ut65k_$v.txt | cut -c1-250)"
  unset GRAVSIM_NATIVE_DIR
done
