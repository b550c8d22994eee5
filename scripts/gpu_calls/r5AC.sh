set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu.sh smoke 'tests:sym+or+overlap+or+rccl' 'bench:--steps+5+--warmup+2' || exit 1
