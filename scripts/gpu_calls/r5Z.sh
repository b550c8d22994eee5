set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
bash scripts/gpu.sh 'tests:gated+or+segmented+or+deferred+or+audit' || exit 1
for r in 1 2 3; do for v in head prev4; do
  if [ $v != head ]; then export GRAVSIM_NATIVE_DIR=abv/$v; fi
  timeout -k 10 300 python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 12 > $O/rsz_$v.log 2>&1 || exit 1
  echo "P8 $v $r $(grep -o '"ms_per_step": [0-9.]*' $O/rsz_$v.log | tail -1)"
  timeout -k 10 300 python bench/rank_shape.py --n 1048576 --ranks 2 --rank 1 --comm-gbps 64 --steps 4 > $O/rsz2_$v.log 2>&1 || exit 1
  echo "P2 $v $r $(grep -o '"ms_per_step": [0-9.]*' $O/rsz2_$v.log | tail -1)"
  unset GRAVSIM_NATIVE_DIR
done; done
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 2 head lib:abv/prev4 -- --steps 6 --warmup 2 || exit 1
C=1048576:fp32:auto:8,1048576:fp32:auto:7
timeout -k 10 400 python -u scripts/state_hash.py --steps 2 --cases $C > $O/hash2_z.jsonl 2>&1 || exit 1
grep -h sha $O/hash2_z.jsonl
