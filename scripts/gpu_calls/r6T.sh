set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
# predicted 1M scaling, every rank emulated, node-sum exchange priced per xGMI link (64 GB/s
# per source peer, peers in parallel) next to the one-pipe price of the same box
for W in 64; do
timeout -k 10 1100 python bench/rank_shape.py --n 1048576 --ranks 1,7,8,3,5,6 --rank all --comm-gbps 64 --steps 10 --links --comm-wgs $W > $O/r6_predicted_scaling_links_w$W.jsonl 2>&1 || { tail -20 $O/r6_predicted_scaling_links_w$W.jsonl; exit 1; }
grep -h '^{' $O/r6_predicted_scaling_links_w$W.jsonl | python -c "
import json,sys
rows=[json.loads(l) for l in sys.stdin]
p1=[r for r in rows if r['P']==1][0]
for P in (2,4,8,3,5,6,7):
    rs=[r for r in rows if r['P']==P]
    if not rs: continue
    m=max(r['ms_per_step'] for r in rs); c=max(r['step_mcycles'] for r in rs)
    x=max(r['phase']['exposed_exchange_ms'] for r in rs)
    print(P, round(m,3), 'eff', round(p1['ms_per_step']/(P*m),4), 'eff_cycles', round(p1['step_mcycles']/(P*c),4), 'max exposed exchange', round(x,3))"
done
