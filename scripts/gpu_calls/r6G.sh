set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
# 1. predicted 1M scaling: every rank of P = 1 / 2 / 4 / 8 emulated with modeled comm (one box)
timeout -k 10 900 python bench/rank_shape.py --n 1048576 --ranks 1,8,2,4 --rank all --comm-gbps 64 --steps 12 > $O/r6_predicted_scaling.jsonl 2>&1 || { tail -20 $O/r6_predicted_scaling.jsonl; exit 1; }
grep -h '^{' $O/r6_predicted_scaling.jsonl | python -c "
import json,sys
rows=[json.loads(l) for l in sys.stdin]
p1=[r['ms_per_step'] for r in rows if r['P']==1][0]
for P in (2,4,8):
    m=max(r['ms_per_step'] for r in rows if r['P']==P)
    print(P, round(m,3), 'efficiency', round(p1/(P*m),4))"
# 2. the torchrun / self-launch / CLI multi-rank rehearsal on this one GPU
timeout -k 10 900 bash scripts/gpu_torchrun.sh > $O/r6_torchrun_rehearsal.txt 2>&1 || { tail -30 $O/r6_torchrun_rehearsal.txt; exit 1; }
tail -5 $O/r6_torchrun_rehearsal.txt
