set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/pmcF $O/pmcW $O/pmcF1 $O/pmcW1
# PMC collection serializes dispatches: flag sync's cross-stream wait kernels would wait for
# a signal queued behind them, so the multi-rank shape runs with event ordering here
# (the stepper switches to event ordering by itself when ROCPROF_COUNTER_COLLECTION is set)
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmcF -o p --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 2 > $O/pmcF.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmcW -o p --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks 8 --rank 7 --comm-gbps 64 --steps 2 > $O/pmcW.log 2>&1 || exit 1
python scripts/pmc_bytes.py $O/pmcF $O/pmcW > $O/r5_pmc_bytes_rank7of8.jsonl
cat $O/r5_pmc_bytes_rank7of8.jsonl

timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmcF1 -o p --output-format csv -- python bench.py --steps 2 --warmup 1 --exact-steps 0 --phase-steps 0 --no-replay-audit --no-energy --check-samples 0 > $O/pmcF1.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmcW1 -o p --output-format csv -- python bench.py --steps 2 --warmup 1 --exact-steps 0 --phase-steps 0 --no-replay-audit --no-energy --check-samples 0 > $O/pmcW1.log 2>&1 || exit 1
python scripts/pmc_bytes.py $O/pmcF1 $O/pmcW1 > $O/r5_pmc_bytes_1m_p1.jsonl
cat $O/r5_pmc_bytes_1m_p1.jsonl
