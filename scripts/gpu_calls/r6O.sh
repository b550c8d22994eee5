set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
# every BASELINE config on the final tree
timeout -k 10 1000 python bench/configs.py --md $O/r6_baseline_configs_final.md > $O/r6O_configs.log 2>&1 || { tail -30 $O/r6O_configs.log; exit 1; }
cat $O/r6_baseline_configs_final.md
