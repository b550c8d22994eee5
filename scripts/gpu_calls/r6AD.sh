set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
# the torchrun / self-launch / CLI multi-rank rehearsal on the final tree (incl. --gpus 8 at 1M)
timeout -k 10 1000 bash scripts/gpu_torchrun.sh > $O/r6_torchrun_rehearsal_final.txt 2>&1 || { tail -30 $O/r6_torchrun_rehearsal_final.txt; exit 1; }
tail -7 $O/r6_torchrun_rehearsal_final.txt | cut -c1-300
