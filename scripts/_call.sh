set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
C=65536:fp32:exact:1,1048576:fp32:exact:1,262144:fp32:exact:3,65536:fp32:auto:1
bash scripts/gpu.sh 'tests:exact+or+cutoff' &&
timeout -k 10 300 python -u scripts/state_hash.py --cases $C > gpurun_out/hash_new.jsonl 2>&1 &&
timeout -k 10 300 env GRAVSIM_NATIVE_DIR=abv/r4 python -u scripts/state_hash.py --cases $C > gpurun_out/hash_r4.jsonl 2>&1 &&
cat gpurun_out/hash_new.jsonl gpurun_out/hash_r4.jsonl | grep sha &&
rm -f gpurun_out/ab_native.jsonl &&
bash scripts/ab_native.sh 3 head lib:abv/r4 -- --cutoff-mode exact --steps 10 --warmup 2 &&
bash scripts/ab_native.sh 2 head lib:abv/r4 -- --steps 10 --warmup 2
