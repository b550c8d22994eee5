set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
B="--check-samples 0 --phase-steps 0 --exact-steps 0 --no-replay-audit --no-energy"
# board power and clocks while the 1M force kernel runs (is the engine clock power-limited?)
: > $O/r6M_power.txt
(rocm-smi --showmaxpower --showpower --showclocks --showtemp >> $O/r6M_power.txt 2>&1; echo "=== idle above" >> $O/r6M_power.txt) || true
timeout -k 10 200 python bench.py --steps 150 --warmup 2 $B > $O/r6M_bench.log 2>&1 &
pid=$!
sleep 12
for i in $(seq 1 14); do
  (date +%T.%N; rocm-smi --showpower --showclocks --showtemp) >> $O/r6M_power.txt 2>&1 || true
  sleep 1.5
done
wait $pid || { tail -20 $O/r6M_bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"engine_clock_ghz": [0-9.]*' $O/r6M_bench.log | head -2
grep -i "power\|sclk\|Temperature (Sensor junction)" $O/r6M_power.txt | head -40
