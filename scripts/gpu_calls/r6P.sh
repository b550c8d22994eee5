set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
B="--check-samples 0 --phase-steps 0 --exact-steps 0 --no-replay-audit --no-energy"
# kernel trace of the 65K bench: gaps between kernels inside a two-step graph and between graphs
rm -rf $O/kt65
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt65 -o kt --output-format csv -- python bench.py --n 65536 --steps 60 --warmup 6 $B > $O/r6P_kt65.log 2>&1 || { tail -20 $O/r6P_kt65.log; exit 1; }
find $O/kt65 -name "*kernel_trace.csv" | head -3
python scripts/kernel_gaps.py "$(find $O/kt65 -name '*kernel_trace.csv' | head -1)" | tee $O/r6P_gaps65.txt
