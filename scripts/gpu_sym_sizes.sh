#!/bin/bash
# sym vs one-sided split across N (fp32, 1 GPU): where should mode auto switch?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/sym_sizes.jsonl
: > $out
for n in 65536 131072 262144 524288; do
  for m in sym split; do
    timeout -k 10 300 python bench.py --n $n --mode $m --steps 20 --warmup 3 > gpurun_out/sz.log 2>&1 || { tail -20 gpurun_out/sz.log; exit 1; }
    tail -1 gpurun_out/sz.log >> $out
    tail -1 gpurun_out/sz.log | python -c "import json,sys; d=json.load(sys.stdin); print($n, '$m', round(d['ms_per_step'],3), '%.4g' % d['value'])"
  done
done
