set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu.sh 'tests:fp64_512k+or+exact_cutoff_boundary' &&
bash scripts/gpu.sh 'bench:--dtype+fp64+--n+524288+--steps+10+--warmup+2' &&
bash scripts/gpu.sh perturb64
