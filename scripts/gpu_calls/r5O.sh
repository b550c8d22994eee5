set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python scripts/first_wave_ab.py --n 65536,131072 --waves 512 --caps 3,4,6,8,2 --rounds 3 > $O/r5_cap_small_n.jsonl 2>&1 || exit 1
cat $O/r5_cap_small_n.jsonl | grep ms_per
