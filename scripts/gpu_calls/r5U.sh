set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
for P in 2 4; do
  rm -rf $O/tp$P
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tp$P -o tr --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks $P --rank 1 --comm-gbps 64 --steps 8 > $O/tp$P.log 2>&1 || exit 1
  t=$(find $O/tp$P -name "*kernel_trace.csv" | head -1)
  python scripts/post_force_chain.py "$t" --print-steps 1 > $O/chainU_$P.txt
  echo "P=$P"; head -2 $O/chainU_$P.txt | cut -c1-1500
done
rm -rf $O/tp1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tp1 -o tr --output-format csv -- python bench/rank_shape.py --n 1048576 --ranks 1 --steps 4 > $O/tp1.log 2>&1 || exit 1
t=$(find $O/tp1 -name "*kernel_trace.csv" | head -1)
python scripts/post_force_chain.py "$t" --print-steps 1 > $O/chainU_1.txt
echo "P=1"; head -2 $O/chainU_1.txt | cut -c1-1000
