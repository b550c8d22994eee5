set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
# predicted 1M scaling on the final tree, every rank emulated (one 64 GB/s pipe per rank)
timeout -k 10 1000 python bench/rank_shape.py --n 1048576 --ranks 1,8,2,4,3,5,6,7 --rank all --comm-gbps 64 --steps 10 > $O/r6_predicted_scaling_final.jsonl 2>&1 || { tail -20 $O/r6_predicted_scaling_final.jsonl; exit 1; }
grep -h '^{' $O/r6_predicted_scaling_final.jsonl | python -c "
import json,sys
rows=[json.loads(l) for l in sys.stdin]
p1=[r for r in rows if r['P']==1][0]
print('P=1', round(p1['ms_per_step'],3), 'GHz', round(p1['engine_clock_ghz'],3))
for P in (2,4,8,3,5,6,7):
    rs=[r for r in rows if r['P']==P]
    m=max(r['ms_per_step'] for r in rs); c=max(r['step_mcycles'] for r in rs)
    print(P, round(m,3), 'eff', round(p1['ms_per_step']/(P*m),4), 'eff_cycles', round(p1['step_mcycles']/(P*c),4), 'ghz', [round(r['engine_clock_ghz'],3) for r in rs])"
