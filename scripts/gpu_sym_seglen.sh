#!/bin/bash
# Segment length L (GRAVSIM_SYM_L, in 128-body quanta) of the sym schedule across N (fp32,
# 1 GPU): fewer, longer segments cut the i-side partial traffic (Pi) but give fewer
# workgroups. "def" is the built-in rule.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/sym_seglen.jsonl
: > $out
for n in ${SIZES:-65536 131072 262144 524288}; do
  for l in ${LS:-def 1 2 4 8 16}; do
    if [ "$l" = def ]; then unset GRAVSIM_SYM_L; else export GRAVSIM_SYM_L=$l; fi
    steps=$(( n > 300000 ? 10 : 100 ))
    timeout -k 10 300 python bench.py --num-bodies $n --mode sym --steps $steps --warmup 5 > gpurun_out/sl.log 2>&1 || { tail -20 gpurun_out/sl.log; exit 1; }
    tail -1 gpurun_out/sl.log | python -c "import json,sys; d=json.load(sys.stdin); d['L']='$l'; print(json.dumps(d))" >> $out
    tail -1 gpurun_out/sl.log | python -c "import json,sys; d=json.load(sys.stdin); print($n, 'L=$l', round(d['ms_per_step'],4), '%.4g' % d['value'])"
  done
done
