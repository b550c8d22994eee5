set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1000 python bench/rank_shape.py --n 1048576 --ranks 1,8,2,4 --rank all --comm-gbps 64 --steps 16 > $O/r5_predicted_scaling_final3.jsonl 2>&1 || exit 1
python - <<'PY'
import json
rows=[json.loads(l) for l in open("gpurun_out/r5_predicted_scaling_final3.jsonl") if l.startswith("{")]
by={}
for r in rows:
    if r.get("predicted_efficiency") is None and r.get("P")!=1: continue
    by.setdefault(r["P"],[]).append(r)
for P,rs in sorted(by.items()):
    w=max(rs,key=lambda r:r["ms_per_step"])
    print(P, "slowest", round(w["ms_per_step"],3), "eff", w.get("predicted_efficiency"))
PY
