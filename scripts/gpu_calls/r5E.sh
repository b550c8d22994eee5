set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 ./gravity-simulator-using-mpi-spark-and-cuda_amd/_native/overlap_probe 60000 3 > $O/overlap_probe.jsonl 2>&1 || exit 1
cat $O/overlap_probe.jsonl
