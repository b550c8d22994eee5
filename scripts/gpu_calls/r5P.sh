set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
bash scripts/gpu.sh 'tests:persistent+or+dynamic+or+rezero+or+audit+or+fused' || exit 1
C=1048576:fp32:auto:1,65536:fp32:auto:1
timeout -k 10 400 python -u scripts/state_hash.py --steps 2 --cases $C > $O/hash2_p.jsonl 2>&1 || exit 1
grep -h sha $O/hash2_p.jsonl
rm -f $O/ab_native.jsonl
bash scripts/ab_native.sh 3 head lib:abv/r4 -- --steps 10 --warmup 2 || exit 1
bash scripts/ab_native.sh 3 head lib:abv/r4 -- --n 65536 --steps 300 --warmup 10 || exit 1
cp $O/ab_native.jsonl $O/r5_persist_final_ab_vs_r4.jsonl
