set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
# predicted 1M scaling at uneven P on ONE box, both prices of the node-sum exchange:
# one 64 GB/s pipe per rank (16 workgroups, as every earlier prediction) and per xGMI link
# (64 GB/s per source peer, peers in parallel, 64 workgroups)
summ() { grep -h '^{' "$1" | python -c "
import json,sys
rows=[json.loads(l) for l in sys.stdin]
p1=[r for r in rows if r['P']==1][0]
for P in (2,4,8,3,5,6,7):
    rs=[r for r in rows if r['P']==P]
    if not rs: continue
    m=max(r['ms_per_step'] for r in rs); c=max(r['step_mcycles'] for r in rs)
    x=max(r['phase']['exposed_exchange_ms'] for r in rs)
    print(rows[-1]['exchange_model'], P, round(m,3), 'eff', round(p1['ms_per_step']/(P*m),4), 'eff_cycles', round(p1['step_mcycles']/(P*c),4), 'max exposed exchange', round(x,3))"; }
timeout -k 10 900 python bench/rank_shape.py --n 1048576 --ranks 1,7,8,3,5,6 --rank all --comm-gbps 64 --steps 10 > $O/r6U_onepipe.jsonl 2>&1 || { tail -20 $O/r6U_onepipe.jsonl; exit 1; }
summ $O/r6U_onepipe.jsonl
timeout -k 10 900 python bench/rank_shape.py --n 1048576 --ranks 1,7,8,3,5,6 --rank all --comm-gbps 64 --steps 10 --links --comm-wgs 64 > $O/r6U_links.jsonl 2>&1 || { tail -20 $O/r6U_links.jsonl; exit 1; }
summ $O/r6U_links.jsonl
