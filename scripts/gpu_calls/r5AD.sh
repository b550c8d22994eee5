set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu.sh 'tests:counter_collection+or+segmented_plan' || exit 1
