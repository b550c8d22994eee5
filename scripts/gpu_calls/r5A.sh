set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
bash scripts/gpu.sh tests || exit 1
C=65536:fp32:auto:1,1048576:fp32:auto:1,262144:fp32:auto:3,1048576:fp32:auto:8,524288:fp64:auto:1,1048576:fp32:auto:5
timeout -k 10 400 python -u scripts/state_hash.py --cases $C > $O/hash_vec.jsonl 2>&1 || exit 1
timeout -k 10 400 env GRAVSIM_REDUCE_VEC=0 python -u scripts/state_hash.py --cases $C > $O/hash_scalar.jsonl 2>&1 || exit 1
timeout -k 10 400 env GRAVSIM_NATIVE_DIR=abv/r4 python -u scripts/state_hash.py --cases $C > $O/hash_r4b.jsonl 2>&1 || exit 1
grep -h sha $O/hash_vec.jsonl $O/hash_scalar.jsonl $O/hash_r4b.jsonl
timeout -k 10 120 ./gravity-simulator-using-mpi-spark-and-cuda_amd/_native/graph_event_probe 4 5000 > $O/gev_standalone.txt 2>&1; echo "standalone rc=$?" >> $O/gev_standalone.txt
timeout -k 10 180 python scripts/graph_event_probe_torch.py 4 5000 > $O/gev_torch.txt 2>&1; echo "torch rc=$?" >> $O/gev_torch.txt
tail -4 $O/gev_standalone.txt $O/gev_torch.txt
